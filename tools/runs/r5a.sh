set -e
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "all_duplicate or index_persists or grid_sha1_many" tests/test_gpu_chain.py > $O/pytest.txt 2>&1
ZC_SHA_AT=0 timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps_at0.txt 2>&1
ZC_SHA_AT=1 timeout -k 10 200 python tools/sha_steps.py 4 > $O/sha_steps_at1.txt 2>&1
ZC_SHA_AT=0 ZC_DEBUG_FILL=1 timeout -k 10 200 python bench.py --sha1 --steps 5 --no-cpu-baseline --no-extras > $O/fill_at0.txt 2>&1
ZC_SHA_AT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_c2sha_at1 -o c2sha -- python3 bench.py --sha1 --steps 10 --no-cpu-baseline --no-extras > $O/trace_c2sha_at1.log 2>&1
ZC_SHA_AT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_c2sha_at0 -o c2sha -- python3 bench.py --sha1 --steps 10 --no-cpu-baseline --no-extras > $O/trace_c2sha_at0.log 2>&1
rc=0; timeout -k 10 120 tools/ubench/scan_regstage $((8<<30)) 15 > $O/scan_regstage.txt 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc  # 1 = outputs differ (reported); anything else ends the call
python -c "from tests.lzo_inputs import payload; payload('text', 128 << 20, 21).tofile('/tmp/text.bin')"
timeout -k 10 300 tools/ubench/lzo_dict_bench /tmp/text.bin 4 5 > $O/lzo_dict.txt 2>&1
echo ok
