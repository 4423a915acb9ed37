set -e
mkdir -p gpurun_out/r4e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused or multi_tile or long_grid" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4e/pytest.txt 2>&1
for m in 0 1 2; do for c in c2 c3 c5; do
  ZC_SHA_MODE=$m timeout -k 10 120 python bench.py --sha1 --config $c --steps 10 --no-cpu-baseline --no-extras > gpurun_out/r4e/b_${m}_${c}.json 2> gpurun_out/r4e/b_${m}_${c}.err
done; done
echo done
