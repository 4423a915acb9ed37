set -e
mkdir -p gpurun_out/r4n
export TMPDIR=/tmp
for c in c2 c5; do
ZC_SHA_MODE=5 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4n/t5$c -o t -- python3 bench.py --sha1 --config $c --steps 4 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r4n/t5$c.log 2>&1
done
echo done
