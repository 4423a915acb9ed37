set -o pipefail
OUT=gpurun_out/r3ub2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 ./tools/ubench/overlap_bench > $OUT/overlap.txt 2>&1
echo rc=$?
