set -o pipefail
OUT=gpurun_out/r3sha
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 && \
timeout -k 10 240 python3 bench.py --sha1 --no-cpu-baseline --no-extras > $OUT/b_sha1_c2.json 2> $OUT/b.err && \
timeout -k 10 240 python3 bench.py --sha1 --config c3 --no-cpu-baseline --no-extras > $OUT/b_sha1_c3.json 2>> $OUT/b.err && \
timeout -k 10 240 python3 bench.py --sha1 --config c5 --no-cpu-baseline --no-extras > $OUT/b_sha1_c5.json 2>> $OUT/b.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace_sha1 -o c2 -- python3 bench.py --sha1 --steps 10 --no-cpu-baseline --no-extras > $OUT/trace_sha1.log 2>&1
echo rc=$?
