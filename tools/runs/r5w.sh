# round-5 (session 2): scan geometry A/B with the packed anchor state
set -e
export TMPDIR=/tmp
O=gpurun_out/r5w
mkdir -p $O
timeout -k 10 180 tools/ubench/scan_geom_ab > $O/scan_geom_ab.txt 2>&1
echo ok
