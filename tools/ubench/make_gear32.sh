#!/bin/bash
# builds tools/ubench/scan_gear_ab (the packed-anchor scan vs the 32-bit-gear
# scan of 1d39f89).  gear32/ is generated here from git (untracked); on a box
# without .git it must already be in the tree.
set -e
cd "$(dirname "$0")"
if git rev-parse 2>/dev/null; then
  mkdir -p gear32
  git show 1d39f89:zbackup_amd/csrc/zc_kernels.hip > gear32/zc_kernels.hip
  git show 1d39f89:zbackup_amd/csrc/zc_device.h > gear32/zc_device.h
fi
hipcc --offload-arch=gfx950 -O3 -std=c++17 -Dzc=zc_gear32 -c scan_gear_ab_old.hip -o /tmp/scan_gear_ab_old.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../zbackup_amd/csrc -c scan_gear_ab.hip -o /tmp/scan_gear_ab.o
hipcc --offload-arch=gfx950 -o ${1:-/tmp/scan_gear_ab} /tmp/scan_gear_ab.o /tmp/scan_gear_ab_old.o
