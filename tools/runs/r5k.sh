# CPU share of the box + incremental / SHA-1 steps with and without the spinning helpers (temporary switch)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
( nproc; python -c "import os; print(len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true; cat /proc/self/status | grep -i cpus_allowed_list ) > $O/cpu.txt 2>&1
ZC_PHASES=1 timeout -k 10 200 python tools/inc_steps.py 4 > $O/inc_spin.txt 2>&1
ZC_NO_SPIN=1 ZC_PHASES=1 timeout -k 10 200 python tools/inc_steps.py 4 > $O/inc_nospin.txt 2>&1
timeout -k 10 200 python tools/sha_steps.py 3 > $O/sha_spin.txt 2>&1
ZC_NO_SPIN=1 timeout -k 10 200 python tools/sha_steps.py 3 > $O/sha_nospin.txt 2>&1
echo ok
