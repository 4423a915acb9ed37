# SHA-1 mode: arithmetic classification of grid runs, fill team armed early (A/B: records cached vs
# streamed); parity incl. the 8 GiB every-record tests; scan ablation A/B; static index profile
set -e
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_fullsize.py > $O/pytest.txt 2>&1
ZC_DEBUG_FILL=1 timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps.txt 2>&1
ZC_REC_CACHED=1 ZC_DEBUG_FILL=1 timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps_cached.txt 2>&1
timeout -k 10 120 tools/ubench/scan_ablate > $O/scan_ablate.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_static -o st -- python3 tools/static_scale.py 1 300000 2000000 > $O/trace_static.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o f -- python3 tools/static_scale.py 1 2000000 > $O/pmc_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o w -- python3 tools/static_scale.py 1 2000000 > $O/pmc_write.log 2>&1
echo ok
