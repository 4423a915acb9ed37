set -e
export TMPDIR=/tmp
O=gpurun_out/r5l
mkdir -p $O
for m in 0 1 2; do ZC_NULL_MODE=$m ZC_PHASES=1 timeout -k 10 200 python tools/inc_steps.py 4 > $O/inc_$m.txt 2>&1; done
echo ok
