# SHA-1 mode after the fill / digest-store changes (+ pytest of the touched suites); scan prototype
# load patterns; static index at 2 M ids (trace + FETCH/WRITE)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_window.py tests/test_gpu_static_scale.py > $O/pytest.txt 2>&1
timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps.txt 2>&1
ZC_DEBUG_FILL=1 timeout -k 10 200 python bench.py --sha1 --steps 5 --no-cpu-baseline --no-extras > $O/fill.txt 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_headline.txt 2>&1
rc=0; timeout -k 10 120 tools/ubench/scan_regstage $((8<<30)) 12 > $O/scan_regstage.txt 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 tools/ubench/scan_ablate > $O/scan_ablate.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_static -o st -- python3 tools/static_scale.py 1 300000 2000000 > $O/trace_static.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o f -- python3 tools/static_scale.py 1 2000000 > $O/pmc_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o w -- python3 tools/static_scale.py 1 2000000 > $O/pmc_write.log 2>&1
echo ok
