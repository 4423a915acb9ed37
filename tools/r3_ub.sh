set -o pipefail
OUT=gpurun_out/r3ub
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 ./tools/ubench/scan_ablate > $OUT/scan_ablate.txt 2>&1 && \
timeout -k 10 300 ./tools/ubench/overlap_bench > $OUT/overlap.txt 2>&1
echo rc=$?
