// Staging microbenchmark 3 (tooling only): register loads for a lane-owns-
// contiguous-bytes scan with no LDS ring.  A wave walks 256 KiB wave-tiles in
// groups of 64 * LS bytes; lane i owns bytes [i * LS, (i + 1) * LS) of a group
// and reads them with LS / 16 dwordx4 loads (instruction k: offset i * LS +
// 16 k).  LS = 16 is fully coalesced (one 1 KiB instruction per group); larger
// LS spreads an instruction over LS / 16 times as many cache lines, each
// line's remaining bytes read by the next instructions.  DEPTH groups in
// flight per wave; MINB workgroups per CU (occupancy).
//
//   hipcc --offload-arch=gfx950 -O3 stage_bench3.hip -o stage_bench3
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);              \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr uint64_t kWT = 256 << 10;
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int TPB, int MINB, int LS, int DEPTH, int EXTRA>
__global__ void __launch_bounds__(TPB, MINB) lane_kernel(const uint8_t* __restrict__ data, uint64_t nwt, uint32_t* out) {
  constexpr int NI = LS / 16;
  constexpr uint64_t GB = 64ull * LS;
  constexpr uint64_t GPT = kWT / GB;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (TPB / 64);
  const uint64_t ntw = nwt > gw ? (nwt - 1 - gw) / nw + 1 : 0;
  const uint64_t nR = ntw * GPT;
  uint32_t acc = 0;
  uint4 buf[DEPTH][NI];
  auto ld = [&](uint64_t R, uint4 (&b)[NI]) {
    const uint64_t wt = gw + (R / GPT) * nw;
    const uint4* p = (const uint4*)(data + wt * kWT + (R % GPT) * GB + (uint64_t)lane * LS);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const v4u t = __builtin_nontemporal_load((const v4u*)p + k);
      b[k] = make_uint4(t[0], t[1], t[2], t[3]);
    }
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if ((uint64_t)d < nR) ld(d, buf[d]);
  for (uint64_t R = 0; R < nR; R += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      if (R + d >= nR) break;
      uint4 v[NI];
#pragma unroll
      for (int k = 0; k < NI; ++k) v[k] = buf[d][k];
      if (R + d + DEPTH < nR) ld(R + d + DEPTH, buf[d]);
#pragma unroll
      for (int k = 0; k < NI; ++k) {
        uint32_t xs[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t x = xs[q];
#pragma unroll
          for (int e = 0; e < EXTRA; ++e) x = (x << 1) + (x >> 3);
          acc ^= x;
        }
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// the same with plain (temporal) loads
template <int TPB, int MINB, int LS, int DEPTH, int EXTRA>
__global__ void __launch_bounds__(TPB, MINB) lane_kernel_t(const uint8_t* __restrict__ data, uint64_t nwt, uint32_t* out) {
  constexpr int NI = LS / 16;
  constexpr uint64_t GB = 64ull * LS;
  constexpr uint64_t GPT = kWT / GB;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (TPB / 64);
  const uint64_t ntw = nwt > gw ? (nwt - 1 - gw) / nw + 1 : 0;
  const uint64_t nR = ntw * GPT;
  uint32_t acc = 0;
  uint4 buf[DEPTH][NI];
  auto ld = [&](uint64_t R, uint4 (&b)[NI]) {
    const uint64_t wt = gw + (R / GPT) * nw;
    const uint4* p = (const uint4*)(data + wt * kWT + (R % GPT) * GB + (uint64_t)lane * LS);
#pragma unroll
    for (int k = 0; k < NI; ++k) b[k] = p[k];
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if ((uint64_t)d < nR) ld(d, buf[d]);
  for (uint64_t R = 0; R < nR; R += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      if (R + d >= nR) break;
      uint4 v[NI];
#pragma unroll
      for (int k = 0; k < NI; ++k) v[k] = buf[d][k];
      if (R + d + DEPTH < nR) ld(R + d + DEPTH, buf[d]);
#pragma unroll
      for (int k = 0; k < NI; ++k) {
        uint32_t xs[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t x = xs[q];
#pragma unroll
          for (int e = 0; e < EXTRA; ++e) x = (x << 1) + (x >> 3);
          acc ^= x;
        }
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void coalesced4(const uint4* p, uint64_t n16, uint32_t* out) {
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x * 4 + threadIdx.x, st = (uint64_t)gridDim.x * blockDim.x * 4;
  uint32_t acc = 0;
  for (; i + 3 * blockDim.x < n16; i += st) {
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = p[i + k * blockDim.x];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t n = 8ull << 30;
  uint8_t* d;
  CK(hipMalloc(&d, n));
  CK(hipMemset(d, 1, n));
  uint32_t* out;
  CK(hipMalloc(&out, 64));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct V {
    const char* name;
    std::function<void()> f;
    std::vector<float> t;
  };
  std::vector<V> vs;
  const uint64_t nwt = n / kWT;
#define LK(K, TPB, MINB, LS, DEPTH, EXTRA)                                                                    \
  vs.push_back({#K " tpb=" #TPB " wg/cu=" #MINB " ls=" #LS " depth=" #DEPTH " extra=" #EXTRA, [=] {            \
                  hipLaunchKernelGGL((K<TPB, MINB, LS, DEPTH, EXTRA>), dim3(cus * MINB), dim3(TPB), 0, 0, d, nwt, \
                                     out);                                                                    \
                },                                                                                            \
                {}});
  LK(lane_kernel_t, 256, 2, 16, 8, 0)
  LK(lane_kernel_t, 256, 2, 16, 16, 0)
  LK(lane_kernel_t, 256, 4, 16, 8, 0)
  LK(lane_kernel_t, 256, 2, 32, 4, 0)
  LK(lane_kernel_t, 256, 2, 32, 8, 0)
  LK(lane_kernel_t, 256, 4, 32, 4, 0)
  LK(lane_kernel_t, 256, 2, 64, 2, 0)
  LK(lane_kernel_t, 256, 2, 64, 4, 0)
  LK(lane_kernel_t, 256, 4, 64, 2, 0)
  LK(lane_kernel_t, 256, 4, 64, 3, 0)
  LK(lane_kernel_t, 512, 1, 64, 4, 0)
  LK(lane_kernel_t, 256, 2, 128, 2, 0)
  LK(lane_kernel_t, 256, 4, 128, 1, 0)
  LK(lane_kernel, 256, 2, 64, 4, 0)
  LK(lane_kernel, 256, 4, 64, 2, 0)
  LK(lane_kernel, 256, 2, 16, 16, 0)
  LK(lane_kernel, 256, 2, 16, 8, 0)
  LK(lane_kernel, 256, 4, 16, 8, 0)
  LK(lane_kernel, 256, 4, 16, 4, 0)
  LK(lane_kernel, 512, 1, 16, 16, 0)
  LK(lane_kernel, 256, 2, 32, 8, 0)
  LK(lane_kernel, 256, 2, 16, 16, 8)
  LK(lane_kernel, 256, 4, 16, 8, 8)
  LK(lane_kernel, 256, 4, 16, 8, 16)
  LK(lane_kernel_t, 256, 2, 64, 4, 8)
  LK(lane_kernel_t, 256, 4, 64, 2, 8)
  LK(lane_kernel_t, 256, 4, 64, 3, 8)
  LK(lane_kernel_t, 256, 2, 16, 16, 8)
  LK(lane_kernel_t, 256, 4, 16, 8, 8)
  LK(lane_kernel_t, 256, 4, 32, 4, 8)
  vs.push_back({"coalesced4 8192x256", [=] { hipLaunchKernelGGL(coalesced4, dim3(8192), dim3(256), 0, 0, (const uint4*)d, n / 16, out); }, {}});
  for (int round = 0; round < 6; ++round)
    for (auto& v : vs) {
      CK(hipEventRecord(a));
      v.f();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (round) v.t.push_back(ms);
    }
  for (auto& v : vs) {
    std::sort(v.t.begin(), v.t.end());
    printf("%-60s %7.3f ms %7.1f GB/s (median %7.3f)\n", v.name, v.t[0], n / (v.t[0] * 1e6), v.t[v.t.size() / 2]);
  }
  return 0;
}
