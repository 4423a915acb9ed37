# SHA-1 finalize (parallel pair checks, pre-wait anchorless scan); key64 run filter a wave per run
set -e
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_screen.py tests/test_gpu_static_scale.py tests/test_gpu_fullsize.py > $O/pytest.txt 2>&1
ZC_DEBUG_FILL=1 timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps.txt 2>&1
timeout -k 10 200 python tools/static_scale.py 1 300000 1000000 2000000 4000000 > $O/static_scale.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_static -o st -- python3 tools/static_scale.py 1 2000000 > $O/trace_static.log 2>&1
echo ok
