# the full GPU suite, then the round-5 profile set of this build (tools/profile_round.sh)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r5e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r5e/pytest_gpu.txt 2>&1
bash tools/profile_round.sh gpurun_out/r5e/prof
echo ok
