# round-5 (session 2): lane-span / workgroup A/B; grid keys written to the
# host by the metadata kernel -- full GPU suite, traced and plain bench
set -e
export TMPDIR=/tmp
O=gpurun_out/r5aa
mkdir -p $O
timeout -k 10 180 tools/ubench/scan_geom_ab > $O/scan_geom_ab.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$O/tr" -o c2 -- \
  python3 bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --no-extras > "$O/tr.jsonl" 2> "$O/tr.err"
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras > $O/bench.jsonl 2> $O/bench.err
echo ok
