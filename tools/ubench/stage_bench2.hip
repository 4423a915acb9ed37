// Staging microbenchmark 2 (tooling only): does the 4 KiB row stride of the
// scan's LDS-DMA staging cost bandwidth compared with rows that sit next to
// each other (a wave-round = one contiguous 8 KiB block)?  And what do plain
// coalesced register loads reach with a persistent grid?
//
//   A  rows 4 KiB apart (the product's lane spans), 512 thr, 128 B rounds, 2 slots
//   B  rows ROWB apart (contiguous wave-round), same schedule
//   C  persistent coalesced register loads, 8 x dwordx4 per lane per round,
//      one round in flight ahead
//   D  grid-stride coalesced (non-persistent), 4 loads in flight
//   E  4 KiB rows, each row's rounds rotated by (row % ROT) * 4096 / ROT bytes
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <functional>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

template <int N> __device__ __forceinline__ void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// ROWSTRIDE: byte distance of consecutive rows (lanes); SPAN: bytes per row per tile
template <int TPB, int ROWB, int SLOTS, int EXTRA, bool CONTIG, int S = 4096, int ROT = 1>
__global__ void __launch_bounds__(TPB, 1) stage_kernel(const uint8_t* __restrict__ data, uint64_t ntiles, uint32_t* out) {
  constexpr int RPI = 1024 / ROWB;
  constexpr int NI = 64 / RPI;
  constexpr int PIECES = ROWB / 16;
  constexpr int ROUNDS = S / ROWB;
  __shared__ __attribute__((aligned(16))) uint8_t ring[TPB / 64][SLOTS][64 * ROWB];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t acc = 0;
  const uint64_t ntk = ntiles > blockIdx.x ? (ntiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const uint64_t nR = ntk * ROUNDS;
  auto swz = [](uint32_t row) { return PIECES == 16 ? (row & 15) : PIECES == 8 ? ((row >> 1) & 7) : ((row >> 2) & 3); };
  auto issue = [&](uint64_t R) {
    const uint64_t tile = blockIdx.x + (R / ROUNDS) * gridDim.x;
    const uint32_t r = R % ROUNDS;
    uint8_t* slot = ring[wave][R % SLOTS];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const uint32_t row = j * RPI + lane / PIECES;
      const uint32_t p = (lane % PIECES) ^ swz(row);
      const uint64_t wbase = tile * (uint64_t)(TPB * S) + (uint64_t)wave * 64 * S;
      const uint64_t off = CONTIG ? (uint64_t)r * 64 * ROWB + (uint64_t)row * ROWB : (uint64_t)row * S + ((r * ROWB + ((wave * 64 + row) % ROT) * (S / ROT)) % S);
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(data + wbase + off + p * 16), (lds_void_t*)(slot + j * 1024), 16, 0, 2);  // nt, as the product
    }
  };
  for (uint64_t R = 0; R < nR && R < SLOTS; ++R) issue(R);
  for (uint64_t R = 0; R < nR; ++R) {
    if (R + SLOTS - 1 < nR) wait_vmcnt<NI * (SLOTS - 1)>();
    else wait_vmcnt<0>();
    const uint8_t* row = ring[wave][R % SLOTS] + lane * ROWB;
    uint4 v[PIECES];
#pragma unroll
    for (int p = 0; p < PIECES; ++p) v[p] = *(const uint4*)(row + ((p ^ swz(lane)) << 4));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (R + SLOTS < nR) issue(R + SLOTS);
#pragma unroll
    for (int p = 0; p < PIECES; ++p) {
      uint32_t xs[4] = {v[p].x, v[p].y, v[p].z, v[p].w};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint32_t x = xs[d];
#pragma unroll
        for (int e = 0; e < EXTRA; ++e) x = (x << 1) + (x >> 3);
        acc ^= x;
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// persistent, coalesced register loads: a wave-round is 8 KiB contiguous,
// instruction k of lane i reads bytes k*1024 + 16*i; DEPTH rounds in flight
template <int TPB, int DEPTH, int EXTRA>
__global__ void __launch_bounds__(TPB, 1) reg_kernel(const uint8_t* __restrict__ data, uint64_t nrounds, uint32_t* out) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * (TPB / 64) + wave, nw = (uint64_t)gridDim.x * (TPB / 64);
  uint32_t acc = 0;
  uint4 buf[DEPTH][8];
  auto ld = [&](uint64_t R, uint4 (&b)[8]) {
    const uint4* p = (const uint4*)(data + R * 8192) + lane;
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = p[64 * k];
  };
  uint64_t R = gw;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (R + d * nw < nrounds) ld(R + d * nw, buf[d]);
  for (; R < nrounds; R += DEPTH * nw) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const uint64_t Rd = R + d * nw;
      if (Rd >= nrounds) break;
      uint4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = buf[d][k];
      if (Rd + DEPTH * nw < nrounds) ld(Rd + DEPTH * nw, buf[d]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
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
  uint64_t n = 8ull << 30;
  uint8_t* d; CK(hipMalloc(&d, n)); CK(hipMemset(d, 1, n));
  uint32_t* out; CK(hipMalloc(&out, 64));
  int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  struct V { const char* name; std::function<void()> f; std::vector<float> t; };
  std::vector<V> vs;
#define STG(TPB, ROWB, SLOTS, EXTRA, CONTIG) vs.push_back({"stage tpb=" #TPB " rowb=" #ROWB " slots=" #SLOTS " extra=" #EXTRA " contig=" #CONTIG, [=] { \
    uint64_t nt = n / (TPB * 4096ull); hipLaunchKernelGGL((stage_kernel<TPB, ROWB, SLOTS, EXTRA, CONTIG>), dim3(std::min<uint64_t>(nt, (uint64_t)cus)), dim3(TPB), 0, 0, d, nt, out); }, {}});
  STG(512, 128, 2, 0, false) STG(512, 128, 2, 0, true) STG(512, 128, 2, 8, false) STG(512, 128, 2, 8, true)
#define STS(S) vs.push_back({"stage tpb=512 rowb=128 slots=2 stride=" #S, [=] { \
    uint64_t nt = n / (512 * (uint64_t)S); hipLaunchKernelGGL((stage_kernel<512, 128, 2, 0, false, S>), dim3(std::min<uint64_t>(nt, (uint64_t)cus)), dim3(512), 0, 0, d, nt, out); }, {}});
  STS(256) STS(512) STS(1024) STS(2048) STS(4096) STS(8192)
#define STR(ROT) vs.push_back({"stage tpb=512 rowb=128 slots=2 stride=4096 rot=" #ROT, [=] { \
    uint64_t nt = n / (512 * 4096ull); hipLaunchKernelGGL((stage_kernel<512, 128, 2, 0, false, 4096, ROT>), dim3(std::min<uint64_t>(nt, (uint64_t)cus)), dim3(512), 0, 0, d, nt, out); }, {}});
  STR(2) STR(4) STR(8) STR(32)
#define STV(ROWB, SLOTS, EXTRA) vs.push_back({"stage rot=2 rowb=" #ROWB " slots=" #SLOTS " extra=" #EXTRA, [=] { \
    uint64_t nt = n / (512 * 4096ull); hipLaunchKernelGGL((stage_kernel<512, ROWB, SLOTS, EXTRA, false, 4096, 2>), dim3(std::min<uint64_t>(nt, (uint64_t)cus)), dim3(512), 0, 0, d, nt, out); }, {}});
  STV(128, 2, 0) STV(128, 2, 8) STV(128, 2, 10) STV(64, 4, 0) STV(64, 4, 8) STV(64, 4, 10) STV(64, 3, 8) STV(256, 1, 8)
#define REG(TPB, DEPTH, EXTRA, WPC) vs.push_back({"reg tpb=" #TPB " depth=" #DEPTH " extra=" #EXTRA " wg/cu=" #WPC, [=] { \
    hipLaunchKernelGGL((reg_kernel<TPB, DEPTH, EXTRA>), dim3(cus * WPC), dim3(TPB), 0, 0, d, n / 8192, out); }, {}});
  REG(512, 2, 0, 1)

  vs.push_back({"coalesced4 2048x256", [=] { hipLaunchKernelGGL(coalesced4, dim3(2048), dim3(256), 0, 0, (const uint4*)d, n / 16, out); }, {}});
  vs.push_back({"coalesced4 8192x256", [=] { hipLaunchKernelGGL(coalesced4, dim3(8192), dim3(256), 0, 0, (const uint4*)d, n / 16, out); }, {}});
  vs.push_back({"coalesced4 1024x1024", [=] { hipLaunchKernelGGL(coalesced4, dim3(1024), dim3(1024), 0, 0, (const uint4*)d, n / 16, out); }, {}});
  for (int round = 0; round < 6; ++round)
    for (auto& v : vs) {
      CK(hipEventRecord(a)); v.f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b)); if (round) v.t.push_back(ms);
    }
  for (auto& v : vs) { std::sort(v.t.begin(), v.t.end()); printf("%-52s %7.3f ms %7.1f GB/s (median %7.3f)\n", v.name, v.t[0], n / (v.t[0] * 1e6), v.t[v.t.size() / 2]); }
  return 0;
}
