set -e
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
for i in 1 2; do
timeout -k 10 200 python tools/inc_steps.py 4 > $O/gk_$i.txt 2>&1
ZC_AB_NOGK=1 timeout -k 10 200 python tools/inc_steps.py 4 > $O/nogk_$i.txt 2>&1
done
echo ok
