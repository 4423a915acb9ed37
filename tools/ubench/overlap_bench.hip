// zc_scan_kernel beside zc_sha1_grid_kernel (the ZC_FLAG_SHA1 pipeline: the grid
// chunks' SHA-1 on a side stream while the scan runs), with variants of both
// kernels' register budgets and of the SHA-1 prefetch depth.  Interleaved rounds
// in one process; prints the median of each arm.  Tooling only.
// Build: hipcc -O3 --offload-arch=gfx950 -I../../zbackup_amd/csrc overlap_bench.hip
#include "../../zbackup_amd/csrc/zc_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace zc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

namespace {
// SHA-1 of whole W-byte grid chunks (n a multiple of W), kAhead blocks
// prefetched per lane, an optional register cap (waves per EU)
template <int kAhead>
__device__ __forceinline__ void sha1_chunk(const uint8_t* __restrict__ data, uint64_t base, uint32_t L, uint32_t i,
                                           uint8_t* __restrict__ out) {
  uint32_t st[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  uint32_t w[16];
  const uint32_t full = L / 64;
  const uint4* p = (const uint4*)(data + base);
  uint4 nx[kAhead][4];
#pragma unroll
  for (uint32_t j = 0; j < kAhead; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) nx[j][k] = p[4 * j + k];
  for (uint32_t b0 = 0; b0 < full; b0 += kAhead) {
#pragma unroll
    for (uint32_t j = 0; j < kAhead; ++j) {
      const uint4 cur[4] = {nx[j][0], nx[j][1], nx[j][2], nx[j][3]};
      if (b0 + j + kAhead < full) {
#pragma unroll
        for (int k = 0; k < 4; ++k) nx[j][k] = p[4 * (b0 + j + kAhead) + k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        w[4 * k] = bswap32(cur[k].x);
        w[4 * k + 1] = bswap32(cur[k].y);
        w[4 * k + 2] = bswap32(cur[k].z);
        w[4 * k + 3] = bswap32(cur[k].w);
      }
      sha1_block(st, w);
    }
  }
  for (int k = 0; k < 16; ++k) w[k] = 0;
  w[0] = 0x80000000u;
  w[15] = L * 8;
  sha1_block(st, w);
  for (int k = 0; k < 5; ++k) ((uint32_t*)out)[i * 5 + k] = st[k];
}

template <int kAhead, int kWpe>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kWpe))) void sha_v(const uint8_t* __restrict__ data,
                                                                                         uint32_t W, uint32_t nr,
                                                                                         uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nr) sha1_chunk<kAhead>(data, (uint64_t)i * W, W, i, out);
}
}  // namespace

int main(int argc, char** argv) {
  uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
  const uint32_t W = 65536, nr = (uint32_t)(n / W);
  uint8_t* d; CK(hipMalloc(&d, n));
  CK(launch_fill_splitmix64(d, n, 2024, 0));
  uint64_t ntiles = n / ZC_STILE, nwt = wave_tiles(n);
  const uint32_t wcap = wave_tile_cap(W);
  int cus = cu_count();
  uint64_t* blk; uint32_t *dbase, *dcnt, *prel, *pg; unsigned long long* cnt; uint8_t* out;
  CK(hipMalloc(&blk, n / ZC_SPAN * 8)); CK(hipMalloc(&dbase, nwt * 4)); CK(hipMalloc(&dcnt, nwt * 4));
  CK(hipMalloc(&prel, nwt * wcap * 4)); CK(hipMalloc(&pg, nwt * wcap * 4)); CK(hipMalloc(&cnt, 64));
  CK(hipMalloc(&out, (size_t)nr * 20));
  const PoolOut po{dbase, dcnt, prel, pg, wcap, 0};
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a, b, e1, e2; CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
  using ScanK = void (*)(const uint8_t*, uint64_t, uint64_t, uint64_t, int32_t, uint64_t*, PoolOut, unsigned long long*);
  using ShaK = void (*)(const uint8_t*, uint32_t, uint32_t, uint8_t*);
  constexpr int P = kScanProduct;
  struct Arm { const char* name; ScanK scan; ShaK sha; int sha_first; std::vector<float> t; };
  std::vector<Arm> arms = {
    {"scan alone", zc_scan_kernel<P>, nullptr, 0, {}},
    {"scan<=128 alone", zc_scan_kernel_v128<P>, nullptr, 0, {}},
    {"sha a4 alone", nullptr, sha_v<4, 1>, 0, {}},
    {"sha a2 alone", nullptr, sha_v<2, 1>, 0, {}},
    {"sha a2<=128 alone", nullptr, sha_v<2, 4>, 0, {}},
    {"sha a1<=96 alone", nullptr, sha_v<1, 5>, 0, {}},
    {"scan + sha a4", zc_scan_kernel<P>, sha_v<4, 1>, 0, {}},
    {"scan + sha a2", zc_scan_kernel<P>, sha_v<2, 1>, 0, {}},
    {"scan<=128 + sha a2<=128", zc_scan_kernel_v128<P>, sha_v<2, 4>, 0, {}},
    {"scan<=128 + sha a4<=128", zc_scan_kernel_v128<P>, sha_v<4, 4>, 0, {}},
    {"scan<=128 + sha a1<=96", zc_scan_kernel_v128<P>, sha_v<1, 5>, 0, {}},
    {"sha a2<=128 first, scan<=128", zc_scan_kernel_v128<P>, sha_v<2, 4>, 1, {}},
    {"scan then sha a4 (serial)", zc_scan_kernel<P>, sha_v<4, 1>, 2, {}},
  };
  const unsigned sgrid = (unsigned)std::min<uint64_t>(ntiles, cus);
  for (int round = 0; round < 12; ++round)
    for (auto& v : arms) {
      CK(hipMemsetAsync(cnt, 0, 64, s1));
      CK(hipStreamSynchronize(s1));
      CK(hipEventRecord(a, s1));
      CK(hipStreamWaitEvent(s2, a, 0));
      const size_t dyn = v.scan == (ScanK)zc_scan_kernel_v128<P> ? sizeof(ScanLds) : 0;
      auto scan = [&] { hipLaunchKernelGGL(v.scan, dim3(sgrid), dim3(ZC_SCAN_TPB), dyn, s1, d, n, (uint64_t)0, ntiles, anchor_lo_for(W), blk, po, cnt); };
      auto sha = [&](hipStream_t s) { hipLaunchKernelGGL(v.sha, dim3((nr + 63) / 64), dim3(64), 0, s, d, W, nr, out); };
      if (v.sha_first == 2) {
        scan();
        sha(s1);
      } else if (v.sha_first == 1) {
        sha(s2);
        if (v.scan) scan();
      } else {
        if (v.scan) scan();
        if (v.sha) sha(s2);
      }
      CK(hipEventRecord(e2, s2));
      CK(hipStreamWaitEvent(s1, e2, 0));
      CK(hipEventRecord(b, s1)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (round) v.t.push_back(ms);
    }
  for (auto& v : arms) {
    std::sort(v.t.begin(), v.t.end());
    printf("%-32s median %7.3f ms  min %7.3f ms\n", v.name, v.t[v.t.size() / 2], v.t[0]);
  }
  return 0;
}
