# round-5 final candidate (session 2): static scale, full GPU suite, profile
# set, SHA-1 and incremental steps
set -e
export TMPDIR=/tmp
O=gpurun_out/r5ae
mkdir -p $O
timeout -k 10 200 python tools/static_scale.py 1 3000 300000 1000000 2000000 4000000 > $O/static_scale.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
bash tools/profile_round.sh $O/prof
timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps.txt 2>&1
timeout -k 10 200 python tools/inc_steps.py 4 > $O/inc_steps.txt 2>&1
echo ok
