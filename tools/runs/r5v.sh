# round-5 (session 2): the packed anchor state -- anchor model tests, in-process
# A/B against the 32-bit gear scan, bench, full GPU suite
set -e
export TMPDIR=/tmp
O=gpurun_out/r5v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_anchors.py -x -v --timeout 120 --timeout-method thread > $O/pytest_anchors.txt 2>&1
timeout -k 10 120 tools/ubench/scan_gear_ab > $O/scan_gear_ab.txt 2>&1
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras > $O/bench.jsonl 2> $O/bench.err
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
echo ok
