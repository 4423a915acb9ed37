# round-5 (session 2): VALU rates of the packed-u16 forms; the packed anchor
# state (two 16-bit streams) -- anchor model test, full GPU suite, bench
set -e
export TMPDIR=/tmp
O=gpurun_out/r5u
mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_rate tools/ubench/valu_rate.hip
timeout -k 10 60 /tmp/valu_rate > $O/valu_rate.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_anchors.py -x -v --timeout 120 --timeout-method thread > $O/pytest_anchors.txt 2>&1
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras > $O/bench.jsonl 2> $O/bench.err
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
echo ok
