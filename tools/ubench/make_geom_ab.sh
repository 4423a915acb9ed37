#!/bin/bash
# builds scan_geom_ab: the product scan in several geometries (one object each)
set -e
cd "$(dirname "$0")"
out=$(realpath -m "${1:-/tmp/scan_geom_ab}")
b() { hipcc --offload-arch=gfx950 -O3 -std=c++17 -Dzc=zc_$1 -DSCAN_ENTRY=scan_v_$1 $2 -c scan_variant.hip -o /tmp/sv_$1.o; }
b prod "" & b wg4_l64 "-DZC_SCAN_WG_PER_CU_CFG=4 -DZC_WLIST_CFG=64" & b wg4_l48 "-DZC_SCAN_WG_PER_CU_CFG=4 -DZC_WLIST_CFG=48" &
b wg2 "-DZC_SCAN_WG_PER_CU_CFG=2" & wait
hipcc --offload-arch=gfx950 -O3 -std=c++17 -c scan_geom_ab.hip -o /tmp/scan_geom_ab.o
hipcc --offload-arch=gfx950 -o $out /tmp/scan_geom_ab.o /tmp/sv_prod.o /tmp/sv_wg4_l64.o /tmp/sv_wg4_l48.o /tmp/sv_wg2.o
