// The grid SHA-1 fused into the scan (zc_scan_sha_kernel) against the scan
// alone, the SHA-1 kernel alone and the two as concurrent kernels (the
// ZC_FLAG_SHA1 pipeline before the fusion).  Interleaved rounds in one
// process; prints the median of each arm and checks the fused digests against
// the SHA-1 kernel's.  Tooling only.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include fuse_bench.hip -o fuse_bench
#include "../../zbackup_amd/csrc/zc_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace zc;
#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);          \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
  const uint32_t W = argc > 2 ? (uint32_t)strtoul(argv[2], 0, 0) : 65536u;
  const int rounds = argc > 3 ? atoi(argv[3]) : 8;
  const uint64_t nr = n / W;
  uint8_t* d;
  CK(hipMalloc(&d, n));
  CK(launch_fill_splitmix64(d, n, 2024, 0));
  const uint64_t ntiles = n / ZC_STILE, nwt = wave_tiles(n);
  const uint32_t wcap = wave_tile_cap(W);
  uint64_t* blk;
  uint32_t *dbase, *dcnt, *prel, *pg;
  unsigned long long* cnt;
  uint8_t *o1, *o2;
  CK(hipMalloc(&blk, n / ZC_SPAN * 8));
  CK(hipMalloc(&dbase, nwt * 4));
  CK(hipMalloc(&dcnt, nwt * 4));
  CK(hipMalloc(&prel, nwt * wcap * 4));
  CK(hipMalloc(&pg, nwt * wcap * 4));
  CK(hipMalloc(&cnt, 64));
  CK(hipMalloc(&o1, nr * 20));
  CK(hipMalloc(&o2, nr * 20));
  const PoolOut po{dbase, dcnt, prel, pg, wcap, 0};
  const int32_t lo = anchor_lo_for(W);
  if (!sha_fusable(n, W, ntiles)) {
    printf("not fusable: n %llu W %u\n", (unsigned long long)n, W);
    return 1;
  }
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a, b, e2;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventCreate(&e2));
  const unsigned grid = (unsigned)std::min<uint64_t>(ntiles, (uint64_t)cu_count());
  const ShaFuse sf{o1, nr, W};
  enum { SCAN, FUSED_T, FUSED_NT, SHA, SCAN_SHA };
  struct Arm {
    const char* name;
    int kind;
    std::vector<float> t;
  };
  std::vector<Arm> arms = {{"scan alone", SCAN, {}},
                           {"fused, temporal SHA-1 loads", FUSED_T, {}},
                           {"fused, nt SHA-1 loads", FUSED_NT, {}},
                           {"sha1 grid kernel alone", SHA, {}},
                           {"scan v128 + sha1 kernel beside", SCAN_SHA, {}}};
  for (int round = 0; round < rounds; ++round)
    for (auto& v : arms) {
      CK(hipMemsetAsync(cnt, 0, 64, s1));
      CK(hipStreamSynchronize(s1));
      CK(hipEventRecord(a, s1));
      CK(hipStreamWaitEvent(s2, a, 0));
      switch (v.kind) {
        case SCAN:
          hipLaunchKernelGGL(zc_scan_kernel<kScanProduct>, dim3(grid), dim3(ZC_SCAN_TPB), 0, s1, d, n, (uint64_t)0,
                             ntiles, lo, blk, po, cnt);
          break;
        case FUSED_T:
          hipLaunchKernelGGL((zc_scan_sha_kernel<kScanProduct, 1>), dim3(grid), dim3(ZC_SCAN_TPB), 0, s1, d, n,
                             (uint64_t)0, ntiles, lo, blk, po, cnt, sf);
          break;
        case FUSED_NT:
          hipLaunchKernelGGL((zc_scan_sha_kernel<kScanProduct, 2>), dim3(grid), dim3(ZC_SCAN_TPB), 0, s1, d, n,
                             (uint64_t)0, ntiles, lo, blk, po, cnt, sf);
          break;
        case SHA:
          CK(launch_sha1_grid(d, n, W, (uint32_t)nr, o2, s2));
          break;
        case SCAN_SHA:
          hipLaunchKernelGGL(zc_scan_kernel_v128<kScanProduct>, dim3(grid), dim3(ZC_SCAN_TPB), sizeof(ScanLds), s1, d,
                             n, (uint64_t)0, ntiles, lo, blk, po, cnt);
          CK(launch_sha1_grid(d, n, W, (uint32_t)nr, o2, s2));
          break;
      }
      CK(hipGetLastError());
      CK(hipEventRecord(e2, s2));
      CK(hipStreamWaitEvent(s1, e2, 0));
      CK(hipEventRecord(b, s1));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (round) v.t.push_back(ms);
    }
  for (auto& v : arms) {
    std::sort(v.t.begin(), v.t.end());
    printf("%-36s median %7.3f ms  min %7.3f ms\n", v.name, v.t[v.t.size() / 2], v.t[0]);
  }
  std::vector<uint8_t> h1(nr * 20), h2(nr * 20);
  CK(hipMemcpy(h1.data(), o1, nr * 20, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2.data(), o2, nr * 20, hipMemcpyDeviceToHost));
  printf("fused digests %s the SHA-1 kernel's (%llu chunks)\n", memcmp(h1.data(), h2.data(), nr * 20) ? "DIFFER from" : "equal",
         (unsigned long long)nr);
  return 0;
}
