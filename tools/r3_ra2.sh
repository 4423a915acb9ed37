set -o pipefail
OUT=gpurun_out/r3ra2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 ./tools/ubench/overlap_bench > $OUT/overlap.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_window.py tests/test_gpu_chain.py tests/test_gpu_fuzz.py tests/test_gpu_screen.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 && \
timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras > $OUT/b_c2.json 2> $OUT/b.err && \
timeout -k 10 240 python3 bench.py --sha1 --no-cpu-baseline --no-extras > $OUT/b_sha1_c2.json 2>> $OUT/b.err
echo rc=$?
