# round-5 (session 2): 256-byte rounds A/B; parity after the read-out rework
set -e
export TMPDIR=/tmp
O=gpurun_out/r5z
mkdir -p $O
timeout -k 10 180 tools/ubench/scan_geom_ab > $O/scan_geom_ab.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_anchors.py tests/test_gpu_parity.py -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
echo ok
