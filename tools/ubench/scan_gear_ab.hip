// A/B, interleaved in one process: the scan with the packed 16-bit anchor state
// (the product zc_scan_kernel) against the same kernel with the 32-bit gear
// (scan_gear_ab_old.hip), 8 GiB of seeded random bytes.  Span digests are
// compared (the same definition on both sides); anchor counts are printed
// (different anchor definitions, the same rate).  Tooling only.
// Build: tools/ubench/make_gear32.sh
#include "../../zbackup_amd/csrc/zc_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

extern "C" hipError_t gear32_scan(const uint8_t* d, uint64_t n, uint64_t ntiles, uint64_t* blk, uint32_t* base,
                                  uint32_t* cnt, uint32_t* rel, uint32_t* g, uint32_t wcap,
                                  unsigned long long* counters);
using namespace zc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
  const int rounds = argc > 2 ? atoi(argv[2]) : 25;
  uint8_t* d; CK(hipMalloc(&d, n));
  CK(launch_fill_splitmix64(d, n, 2024, 0));
  const uint64_t ntiles = n / ZC_STILE, nwt = wave_tiles(n), nblk = n / ZC_SPAN;
  const uint32_t wcap = wave_tile_cap(65536);
  uint64_t *blk[2]; uint32_t *dbase, *dcnt, *prel, *pg; unsigned long long* cnt[2];
  for (int v = 0; v < 2; ++v) { CK(hipMalloc(&blk[v], nblk * 8)); CK(hipMalloc(&cnt[v], 64)); }
  CK(hipMalloc(&dbase, nwt * 4)); CK(hipMalloc(&dcnt, nwt * 4));
  CK(hipMalloc(&prel, nwt * wcap * 4)); CK(hipMalloc(&pg, nwt * wcap * 4));
  const PoolOut po{dbase, dcnt, prel, pg, wcap, 0};
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::vector<float> t[2];
  unsigned long long pool[2] = {0, 0};
  for (int round = 0; round < rounds; ++round)
    for (int v = 0; v < 2; ++v) {
      CK(hipMemset(cnt[v], 0, 64));
      CK(hipEventRecord(a));
      if (v == 0) CK(launch_scan_tiles(d, n, 0, ntiles, anchor_lo_for(65536), blk[0], po, cnt[0], 0));
      else CK(gear32_scan(d, n, ntiles, blk[1], dbase, dcnt, prel, pg, wcap, cnt[1]));
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (round) t[v].push_back(ms);
      CK(hipMemcpy(&pool[v], cnt[v] + CNT_POOL, 8, hipMemcpyDeviceToHost));
    }
  std::vector<uint64_t> h0(nblk), h1(nblk);
  CK(hipMemcpy(h0.data(), blk[0], nblk * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h1.data(), blk[1], nblk * 8, hipMemcpyDeviceToHost));
  const char* names[2] = {"packed 16-bit anchor state (product)", "32-bit gear (1d39f89)"};
  for (int v = 0; v < 2; ++v) {
    std::sort(t[v].begin(), t[v].end());
    printf("%-40s median %7.3f ms  min %7.3f ms  %7.1f GB/s (min)  anchors %llu\n", names[v], t[v][t[v].size() / 2],
           t[v][0], n / (t[v][0] * 1e6), pool[v]);
  }
  const bool same = h0 == h1;
  printf(same ? "span digests identical\n" : "SPAN DIGESTS DIFFER\n");
  return same ? 0 : 2;
}
