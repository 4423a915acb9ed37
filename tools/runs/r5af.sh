# round-5 (session 2): the grid SHA-1 beside the scan (ZC_AB_SHA_EARLY) vs
# behind the batch, now that the scan leaves 45 % of the VALU idle
set -e
export TMPDIR=/tmp
O=gpurun_out/r5af
mkdir -p $O
timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps_behind.txt 2>&1
ZC_AB_SHA_EARLY=1 timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps_early.txt 2>&1
timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps_behind2.txt 2>&1
ZC_AB_SHA_EARLY=1 timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps_early2.txt 2>&1
ZC_AB_SHA_EARLY=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_fullsize.py -x -q --timeout 400 --timeout-method thread > $O/pytest_early.txt 2>&1
echo ok
