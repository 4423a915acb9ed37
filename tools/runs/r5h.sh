# scan occupancy experiment (ubench, outputs compared) + incremental step phases
set -e
export TMPDIR=/tmp
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 120 ./tools/ubench/scan_occ > $O/scan_occ.txt 2>&1
timeout -k 10 200 python tools/inc_steps.py 5 > $O/inc_steps.txt 2>&1
echo ok
