// One geometry variant of the product scan (zc_kernels.hip built with the
// -D ZC_*_CFG switches of zc_device.h and -Dzc=<namespace>), exported as the C
// entry SCAN_ENTRY for scan_geom_ab.hip.  Tooling only.
#include "../../zbackup_amd/csrc/zc_kernels.hip"
extern "C" hipError_t SCAN_ENTRY(const uint8_t* d, uint64_t n, uint64_t ntiles, uint64_t* blk, uint32_t* base,
                                 uint32_t* cnt, uint32_t* rel, uint32_t* g, uint32_t wcap,
                                 unsigned long long* counters) {
  // this variant's own tile geometry (the lane span sets the tile size)
  (void)ntiles;
  (void)wcap;
  const zc::PoolOut po{base, cnt, rel, g, zc::wave_tile_cap(65536), 0};
  return zc::launch_scan_tiles(d, n, 0, n / zc::ZC_STILE, zc::anchor_lo_for(65536), blk, po, counters, 0);
}
