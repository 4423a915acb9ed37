# round-5 (session 2): two ring slots per wave A/B (and the contiguous-round
# staging probe); parity subset after the wait-count rework
set -e
export TMPDIR=/tmp
O=gpurun_out/r5ad
mkdir -p $O
timeout -k 10 180 tools/ubench/scan_geom_ab > $O/scan_geom_ab.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_anchors.py tests/test_gpu_parity.py -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
echo ok
