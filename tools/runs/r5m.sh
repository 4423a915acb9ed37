set -e
export TMPDIR=/tmp
O=gpurun_out/r5m
mkdir -p $O
for m in plain sleep records; do timeout -k 10 200 python tools/inc_ab.py $m >> $O/ab.txt 2>&1; done
echo ok
