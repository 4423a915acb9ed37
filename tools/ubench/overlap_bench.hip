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
  constexpr int P = kScanProduct;
  uint32_t *hanc, *hg; uint64_t* hfp;
  CK(hipMalloc(&hanc, (size_t)nr * 16)); CK(hipMalloc(&hg, (size_t)nr * 16)); CK(hipMalloc(&hfp, (size_t)nr * 32));
  // arms: scan variant (or none), SHA (product lean grid kernel), heads (product)
  struct Arm { const char* name; ScanK scan; bool v128; bool sha; bool heads; std::vector<float> t; };
  std::vector<Arm> arms = {
    {"scan alone", zc_scan_kernel<P>, false, false, false, {}},
    {"scan perbyte alone", zc_scan_kernel<P | ABL_PERBYTE>, false, false, false, {}},
    {"scan perbyte + sha", zc_scan_kernel<P | ABL_PERBYTE>, false, true, false, {}},
    {"scan prio alone", zc_scan_kernel<P | ABL_PRIO>, false, false, false, {}},
    {"sha grid16 alone", nullptr, false, true, false, {}},
    {"heads alone", nullptr, false, false, true, {}},
    {"scan + heads", zc_scan_kernel<P>, false, false, true, {}},
    {"scan prio + heads", zc_scan_kernel<P | ABL_PRIO>, false, false, true, {}},
    {"scan + sha", zc_scan_kernel<P>, false, true, false, {}},
    {"scan prio + sha", zc_scan_kernel<P | ABL_PRIO>, false, true, false, {}},
    {"scan v128 + sha", zc_scan_kernel_v128<P>, true, true, false, {}},
    {"scan v128 prio + sha", zc_scan_kernel_v128<P | ABL_PRIO>, true, true, false, {}},
    {"scan + sha + heads", zc_scan_kernel<P>, false, true, true, {}},
    {"scan prio + sha + heads", zc_scan_kernel<P | ABL_PRIO>, false, true, true, {}},
  };
  const unsigned sgrid = (unsigned)std::min<uint64_t>(ntiles, cus);
  hipStream_t s3;
  CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
  hipEvent_t e3; CK(hipEventCreate(&e3));
  for (int round = 0; round < 12; ++round)
    for (auto& v : arms) {
      CK(hipMemsetAsync(cnt, 0, 64, s1));
      CK(hipStreamSynchronize(s1));
      CK(hipEventRecord(a, s1));
      CK(hipStreamWaitEvent(s2, a, 0));
      CK(hipStreamWaitEvent(s3, a, 0));
      if (v.scan)
        hipLaunchKernelGGL(v.scan, dim3(sgrid), dim3(ZC_SCAN_TPB), v.v128 ? sizeof(ScanLds) : 0, s1, d, n, (uint64_t)0,
                           ntiles, anchor_lo_for(W), blk, po, cnt);
      if (v.sha) CK(launch_sha1_grid(d, n, W, nr, out, s2));
      if (v.heads) CK(launch_grid_heads(d, n, 0, nr - 1, W, anchor_lo_for(W), hanc, hg, hfp, s3));
      CK(hipEventRecord(e2, s2));
      CK(hipEventRecord(e3, s3));
      CK(hipStreamWaitEvent(s1, e2, 0));
      CK(hipStreamWaitEvent(s1, e3, 0));
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
