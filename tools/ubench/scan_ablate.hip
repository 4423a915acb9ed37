// Ablation timing of scan variants (the ABL_* bits of scan_ablate_kernel.hip)
// against the product zc_scan_kernel, interleaved rounds in one process
// (cdna_hip_programming.md §5.4 rule 24).  Tooling only.
// Build: hipcc -O3 --offload-arch=gfx950 -I../../zbackup_amd/csrc scan_ablate.hip
#include "../../zbackup_amd/csrc/zc_kernels.hip"
#include "scan_ablate_kernel.hip"

#include <cstdio>
#include <vector>
#include <algorithm>

using namespace zc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
  uint8_t* d; CK(hipMalloc(&d, n));
  CK(launch_fill_splitmix64(d, n, 2024, 0));
  uint64_t ntiles = n / ZC_STILE, nwt = wave_tiles(n);
  const uint32_t wcap = wave_tile_cap(65536);
  int cus = cu_count();
  uint64_t* blk; uint32_t *dbase, *dcnt, *prel, *pg; unsigned long long* cnt;
  CK(hipMalloc(&blk, n / ZC_SPAN * 8)); CK(hipMalloc(&dbase, nwt * 4)); CK(hipMalloc(&dcnt, nwt * 4));
  CK(hipMalloc(&prel, nwt * wcap * 4)); CK(hipMalloc(&pg, nwt * wcap * 4)); CK(hipMalloc(&cnt, 64));
  const PoolOut po{dbase, dcnt, prel, pg, wcap, 0};
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  struct V { const char* name; void (*k)(const uint8_t*, uint64_t, uint64_t, uint64_t, int32_t, uint64_t*, PoolOut, unsigned long long*); std::vector<float> t; };
  // k == nullptr: the product kernel through its launcher (its own geometry)
  constexpr int P = kAblProduct;
  std::vector<V> vs = {
    {"product zc_scan_kernel", nullptr, {}},
    {"ablation copy, product bits", abl_scan_kernel<P>, {}},
    {"no_atomic", abl_scan_kernel<P | ABL_NO_ATOMIC>, {}},
    {"te_no_anchor_store", abl_scan_kernel<P | ABL_TE_NO_ANCHOR_STORE>, {}},
    {"te_digest_only", abl_scan_kernel<P | ABL_TE_DIGEST_ONLY>, {}},
    {"te_no_store", abl_scan_kernel<P | ABL_TE_NO_STORE>, {}},
  };
  for (int round = 0; round < 25; ++round)
    for (auto& v : vs) {
      CK(hipMemset(cnt, 0, 64));
      CK(hipEventRecord(a));
      if (!v.k) CK(launch_scan_tiles(d, n, 0, ntiles, anchor_lo_for(65536), blk, po, cnt, 0));
      else hipLaunchKernelGGL(v.k, dim3(std::min<uint64_t>(ntiles, cus)), dim3(ZC_SCAN_TPB), 0, 0, d, n, (uint64_t)0, ntiles, anchor_lo_for(65536), blk, po, cnt);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (round) v.t.push_back(ms);
    }
  for (auto& v : vs) {
    std::sort(v.t.begin(), v.t.end());
    printf("%-22s median %7.3f ms  min %7.3f ms  %7.1f GB/s\n", v.name, v.t[v.t.size() / 2], v.t[0], n / (v.t[0] * 1e6));
  }
  return 0;
}
