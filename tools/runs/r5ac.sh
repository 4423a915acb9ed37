# round-5 (session 2): staging shapes -- strided rows vs a contiguous wave-round
set -e
export TMPDIR=/tmp
O=gpurun_out/r5ac
mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -o /tmp/stage_bench2 tools/ubench/stage_bench2.hip
hipcc --offload-arch=gfx950 -O3 -o /tmp/stage_bench3 tools/ubench/stage_bench3.hip
timeout -k 10 120 /tmp/stage_bench2 > $O/stage_bench2.txt 2>&1
timeout -k 10 120 /tmp/stage_bench3 > $O/stage_bench3.txt 2>&1
echo ok
