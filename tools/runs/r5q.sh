# scan with 64-byte rounds (4 waves per SIMD) vs 128-byte rounds (3 per SIMD)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 150 ./tools/ubench/scan_occ > $O/scan_occ128.txt 2>&1
timeout -k 10 150 ./tools/ubench/scan_occ64 > $O/scan_occ64.txt 2>&1
timeout -k 10 150 ./tools/ubench/scan_occ > $O/scan_occ128b.txt 2>&1
echo ok
