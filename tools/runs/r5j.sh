# incremental phases traced (temporary tracer build)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
ZC_PHASES=1 timeout -k 10 200 python tools/inc_steps.py 3 > $O/inc_steps.txt 2>&1
echo ok
