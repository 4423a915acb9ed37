#!/bin/bash
# builds scan_geom_ab: the product scan in several geometries (one object each)
set -e
out=$(realpath -m "${1:-/tmp/scan_geom_ab}")
cd "$(dirname "$0")"
b() { hipcc --offload-arch=gfx950 -O3 -std=c++17 -Dzc=zc_$1 -DSCAN_ENTRY=scan_v_$1 $2 -c scan_variant.hip -o /tmp/sv_$1.o; }
# (round 5 also measured 4 x 4 waves with lists of 64 / 48 entries: r05_scan_geom_ab.txt)
# and 2 x 4 waves with 256-byte rounds (-DZC_ROUND_CFG=256): r05_scan_geom_ab2.txt
# and 2 KiB lane spans (-DZC_LSPAN_CFG=2048): r05_scan_geom_ab3/4.txt
# and 3 x 4 waves (-DZC_SCAN_WG_PER_CU_CFG=3): r05_scan_geom_ab4.txt
# and two ring slots / one workgroup with two / the contiguous probe (-DZC_SCAN_SLOTS_CFG=2,
# -DZC_SCAN_WG_PER_CU_CFG=1, -DZC_CONTIG_PROBE_CFG=1): r05_scan_geom_ab5.txt
# and the round-6 hand-off priority variants below: r06_scan_prio_ab.txt (no gain; default 0)
b prod "" & b prio1 "-DZC_SCAN_PRIO_CFG=1" & b prio2 "-DZC_SCAN_PRIO_CFG=2" & b prio3 "-DZC_SCAN_PRIO_CFG=3" & wait
hipcc --offload-arch=gfx950 -O3 -std=c++17 -c scan_geom_ab.hip -o /tmp/scan_geom_ab.o
hipcc --offload-arch=gfx950 -o $out /tmp/scan_geom_ab.o /tmp/sv_prod.o /tmp/sv_prio1.o /tmp/sv_prio2.o /tmp/sv_prio3.o
