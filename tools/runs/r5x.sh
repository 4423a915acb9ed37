# round-5 (session 2): post-scan A/B -- anchor/class table size (ZC_AB_TBITS),
# scan workgroups per CU (ZC_AB_SCANWG); probe loads per ref in one level
set -e
export TMPDIR=/tmp
O=gpurun_out/r5x
mkdir -p $O
for cfg in "0 3" "1 3" "2 3" "0 2" "1 2"; do
  set -- $cfg
  export ZC_AB_TBITS=$1 ZC_AB_SCANWG=$2
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$O/tr_$1_$2" -o c2 -- \
    python3 bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --no-extras > "$O/tr_$1_$2.jsonl" 2> "$O/tr_$1_$2.err"
  timeout -k 10 200 python3 bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --no-extras > "$O/b_$1_$2.jsonl" 2> "$O/b_$1_$2.err"
done
unset ZC_AB_TBITS ZC_AB_SCANWG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
echo ok
