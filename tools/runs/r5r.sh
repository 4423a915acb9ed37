# historic grid-window keys from the epoch batch: chain/parity/fullsize tests, incremental timing
set -e
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.txt 2>&1
timeout -k 10 200 python tools/inc_ab.py plain > $O/ab.txt 2>&1
timeout -k 10 200 python tools/inc_steps.py 4 > $O/inc_steps.txt 2>&1
echo ok
