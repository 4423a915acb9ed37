set -o pipefail
mkdir -p gpurun_out/r3base
export TMPDIR=/tmp
timeout -k 10 120 ./tools/ubench/valu_rate > gpurun_out/r3base/valu_rate.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3base/pytest.txt 2>&1
echo pytest_rc=$? >> gpurun_out/r3base/pytest.txt
timeout -k 10 240 python3 bench.py --sha1 --no-cpu-baseline --no-extras > gpurun_out/r3base/b_sha1_c2.json 2> gpurun_out/r3base/b.err && \
timeout -k 10 240 python3 bench.py --sha1 --config c3 --no-cpu-baseline --no-extras > gpurun_out/r3base/b_sha1_c3.json 2>> gpurun_out/r3base/b.err && \
timeout -k 10 240 python3 bench.py --sha1 --config c5 --no-cpu-baseline --no-extras > gpurun_out/r3base/b_sha1_c5.json 2>> gpurun_out/r3base/b.err && \
timeout -k 10 400 python3 bench.py > gpurun_out/r3base/b_full.json 2>> gpurun_out/r3base/b.err
echo rc=$?
