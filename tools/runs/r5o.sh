# scan occupancy (reordered, repeats) + full GPU suite on the pinned read-back build
set -e
export TMPDIR=/tmp
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 150 ./tools/ubench/scan_occ > $O/scan_occ.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
echo ok
