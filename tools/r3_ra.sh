set -o pipefail
OUT=gpurun_out/r3ra
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
echo "pytest rc=$?" >> $OUT/pytest.txt
timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras > $OUT/b_c2.json 2> $OUT/b.err && \
timeout -k 10 240 python3 bench.py --sha1 --no-cpu-baseline --no-extras > $OUT/b_sha1_c2.json 2>> $OUT/b.err && \
timeout -k 10 240 python3 bench.py --sha1 --config c3 --no-cpu-baseline --no-extras > $OUT/b_sha1_c3.json 2>> $OUT/b.err && \
timeout -k 10 240 python3 bench.py --sha1 --config c5 --no-cpu-baseline --no-extras > $OUT/b_sha1_c5.json 2>> $OUT/b.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace_c2 -o c2 -- python3 bench.py --steps 10 --no-cpu-baseline --no-extras > $OUT/trace_c2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace_sha1 -o c2 -- python3 bench.py --sha1 --steps 10 --no-cpu-baseline --no-extras > $OUT/trace_sha1.log 2>&1
echo rc=$?
