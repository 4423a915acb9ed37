# static index at 2 M ids on 1 GiB: kernel trace + FETCH / WRITE passes
set -e
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_static -o st -- python3 tools/static_scale.py 1 300000 2000000 > $O/trace_static.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o f -- python3 tools/static_scale.py 1 2000000 > $O/pmc_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o w -- python3 tools/static_scale.py 1 2000000 > $O/pmc_write.log 2>&1
echo ok
