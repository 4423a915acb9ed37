# product scan: one-slot ring, per-wave wave-tiles, 3 workgroups of 4 waves per CU -- A/B vs the previous design, GPU suite, bench
set -e
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 150 ./tools/ubench/scan_ablate > $O/scan_ablate.txt 2>&1
timeout -k 10 150 ./tools/ubench/scan_occ > $O/scan_occ.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
echo ok
