# rk_acc edge folding + hybrid key64 filter: the suites that use them, static scale, SHA-1 steps
set -e
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_screen.py tests/test_gpu_static_scale.py tests/test_gpu_fuzz.py tests/test_gpu_window.py tests/test_gpu_chain.py > $O/pytest.txt 2>&1
timeout -k 10 200 python tools/static_scale.py 1 3000 300000 1000000 2000000 4000000 > $O/static_scale.txt 2>&1
timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_static -o st -- python3 tools/static_scale.py 1 300000 2000000 > $O/trace_static.log 2>&1
echo ok
