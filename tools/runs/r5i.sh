# scan occupancy variants (round 2) + incremental phases traced (temporary tracer build)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 150 ./tools/ubench/scan_occ > $O/scan_occ.txt 2>&1
ZC_PHASES=1 timeout -k 10 200 python tools/inc_steps.py 3 > $O/inc_steps.txt 2>&1
echo ok
