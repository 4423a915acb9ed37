# round-5 (session 2): host phases of verify_candidates in an incremental
# backup (A/B-only timers, ZC_AB_VCTIME)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5ah
mkdir -p $O
ZC_AB_VCTIME=1 timeout -k 10 200 python tools/inc_steps.py 4 > $O/inc_steps.txt 2> $O/vc_times.txt
echo ok
