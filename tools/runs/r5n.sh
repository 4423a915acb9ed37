# pinned candidate read-back + persistent resolver lists: chain/parity tests, incremental timing
set -e
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
for m in plain records; do timeout -k 10 200 python tools/inc_ab.py $m >> $O/ab.txt 2>&1; done
timeout -k 10 200 python tools/inc_steps.py 4 > $O/inc_steps.txt 2>&1
echo ok
