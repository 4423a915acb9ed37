// Staging-only microbenchmark: how fast can lane-contiguous 4 KiB spans be
// streamed HBM -> LDS (global_load_lds_dwordx4, swizzled source) -> per-lane
// ds_read_b128, as a function of row bytes per round (ROWB), ring slots
// (SLOTS) and workgroup size (TPB)?  Also plain per-lane register loads.
// Tooling only.
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
constexpr int S = 4096;

template <int N> __device__ __forceinline__ void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// per wave: 64 rows (lanes) x ROWB bytes per round; one DMA instruction = 1 KiB
// = RPI rows; the wave's ring has SLOTS slots
template <int TPB, int ROWB, int SLOTS>
__global__ void __launch_bounds__(TPB) stage_kernel(const uint8_t* __restrict__ data, uint64_t ntiles, uint32_t* out) {
  constexpr int RPI = 1024 / ROWB;          // rows per DMA instruction
  constexpr int NI = 64 / RPI;              // instructions per wave-round
  constexpr int PIECES = ROWB / 16;
  constexpr int ROUNDS = S / ROWB;
  __shared__ __attribute__((aligned(16))) uint8_t ring[TPB / 64][SLOTS][64 * ROWB];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t acc = 0;
  const uint64_t ntk = ntiles > blockIdx.x ? (ntiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const uint64_t nR = ntk * ROUNDS;
  auto issue = [&](uint64_t R) {
    const uint64_t tile = blockIdx.x + (R / ROUNDS) * gridDim.x;
    const uint32_t r = R % ROUNDS;
    uint8_t* slot = ring[wave][R % SLOTS];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const uint32_t row = j * RPI + lane / PIECES;
      const uint32_t p = (lane % PIECES) ^ ((row / (64 / PIECES >= 1 ? 1 : 1)) % PIECES);
      const uint8_t* src = data + tile * (uint64_t)(TPB * S) + (uint64_t)(wave * 64 + row) * S + r * ROWB + p * 16;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(slot + j * 1024), 16, 0, 0);
    }
  };
  for (uint64_t R = 0; R < nR && R < SLOTS - 1; ++R) issue(R);
  for (uint64_t R = 0; R < nR; ++R) {
    if (R + SLOTS - 1 < nR) { issue(R + SLOTS - 1); wait_vmcnt<NI * (SLOTS - 1)>(); }
    else wait_vmcnt<0>();
    const uint8_t* row = ring[wave][R % SLOTS] + lane * ROWB;
#pragma unroll
    for (int p = 0; p < PIECES; ++p) {
      uint4 v = *(const uint4*)(row + ((p ^ (lane % PIECES)) << 4));
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    asm volatile("" ::: "memory");
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// the scan kernel's schedule: wait for round R, read the lane's row into
// registers, refill the slot with round R + SLOTS, then "compute" (an xor per
// dword plus EXTRA dependent VALU ops per dword, to mimic hashing work)
template <int TPB, int ROWB, int SLOTS, int EXTRA>
__global__ void __launch_bounds__(TPB, 1) stage2_kernel(const uint8_t* __restrict__ data, uint64_t ntiles, uint32_t* out) {
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
      const uint8_t* src = data + tile * (uint64_t)(TPB * S) + (uint64_t)(wave * 64 + row) * S + r * ROWB + p * 16;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(slot + j * 1024), 16, 0, 0);
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

// per-lane register loads of the lane's own span, BATCH bytes per lane in flight x 2
template <int TPB, int BATCH>
__global__ void __launch_bounds__(TPB) reg_kernel(const uint8_t* __restrict__ data, uint64_t ntiles, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint4* p = (const uint4*)(data + t * (uint64_t)(TPB * S) + (uint64_t)threadIdx.x * S);
    uint4 cur[BATCH / 16], nxt[BATCH / 16];
#pragma unroll
    for (int k = 0; k < BATCH / 16; ++k) cur[k] = p[k];
    for (int b = 0; b < S / BATCH; ++b) {
      if (b + 1 < S / BATCH) {
#pragma unroll
        for (int k = 0; k < BATCH / 16; ++k) nxt[k] = p[(b + 1) * (BATCH / 16) + k];
      }
#pragma unroll
      for (int k = 0; k < BATCH / 16; ++k) acc ^= cur[k].x ^ cur[k].y ^ cur[k].z ^ cur[k].w;
#pragma unroll
      for (int k = 0; k < BATCH / 16; ++k) cur[k] = nxt[k];
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void coalesced(const uint4* p, uint64_t n16, uint32_t* out) {
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, st = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (; i < n16; i += st) { uint4 v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
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
#define STG(TPB, ROWB, SLOTS, WPC) vs.push_back({"stage tpb=" #TPB " rowb=" #ROWB " slots=" #SLOTS " wg/cu=" #WPC, [=] { \
    uint64_t nt = n / (TPB * (uint64_t)S); hipLaunchKernelGGL((stage_kernel<TPB, ROWB, SLOTS>), dim3(std::min<uint64_t>(nt, (uint64_t)cus * WPC)), dim3(TPB), 0, 0, d, nt, out); }, {}});
  STG(512, 64, 4, 1) STG(512, 128, 2, 1) STG(256, 128, 2, 2) STG(256, 128, 4, 1) STG(256, 256, 2, 1)
  STG(256, 64, 4, 2) STG(128, 256, 2, 2) STG(512, 64, 2, 2) STG(256, 64, 2, 4) STG(256, 128, 3, 1)
  STG(128, 128, 4, 2) STG(64, 256, 4, 4)
#define ST2(TPB, ROWB, SLOTS, EXTRA) vs.push_back({"stage2 tpb=" #TPB " rowb=" #ROWB " slots=" #SLOTS " extra=" #EXTRA, [=] { \
    uint64_t nt = n / (TPB * (uint64_t)S); hipLaunchKernelGGL((stage2_kernel<TPB, ROWB, SLOTS, EXTRA>), dim3(std::min<uint64_t>(nt, (uint64_t)cus)), dim3(TPB), 0, 0, d, nt, out); }, {}});
  ST2(512, 128, 2, 0) ST2(512, 256, 1, 0) ST2(256, 256, 2, 0) ST2(512, 128, 2, 8) ST2(512, 256, 1, 8)
  ST2(256, 256, 2, 8) ST2(512, 128, 2, 16) ST2(512, 256, 1, 16) ST2(256, 256, 2, 16)
  ST2(512, 64, 4, 0) ST2(512, 64, 4, 8) ST2(512, 64, 4, 16)
#define REG(TPB, BATCH, WPC) vs.push_back({"reg tpb=" #TPB " batch=" #BATCH " wg/cu=" #WPC, [=] { \
    uint64_t nt = n / (TPB * (uint64_t)S); hipLaunchKernelGGL((reg_kernel<TPB, BATCH>), dim3(std::min<uint64_t>(nt, (uint64_t)cus * WPC)), dim3(TPB), 0, 0, d, nt, out); }, {}});
  REG(256, 128, 8) REG(256, 256, 4) REG(256, 64, 8) REG(512, 128, 4)
  vs.push_back({"coalesced", [=] { hipLaunchKernelGGL(coalesced, dim3(2048), dim3(256), 0, 0, (const uint4*)d, n / 16, out); }, {}});
  for (int round = 0; round < 5; ++round)
    for (auto& v : vs) {
      CK(hipEventRecord(a)); v.f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b)); if (round) v.t.push_back(ms);
    }
  for (auto& v : vs) { std::sort(v.t.begin(), v.t.end()); printf("%-44s %7.3f ms %7.1f GB/s\n", v.name, v.t[0], n / (v.t[0] * 1e6)); }
  return 0;
}
