// VALU issue-rate microbenchmark (tooling only): lane-ops per clock per CU of
// the instructions the scan's per-byte loop is made of, 8 independent chains
// per lane, all CUs busy.  Prints G lane-ops/s per instruction form.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int ITERS = 4096;

#define KERNEL32(NAME, ASM)                                                               \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {             \
    uint32_t a[8], b = seed ^ threadIdx.x, c = seed * 3u + 1u;                            \
    for (int i = 0; i < 8; ++i) a[i] = seed + i * 77u + threadIdx.x;                      \
    for (int it = 0; it < ITERS; ++it) {                                                  \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(a[i]) : "v"(b), "v"(c)); \
    }                                                                                     \
    uint32_t x = 0;                                                                       \
    for (int i = 0; i < 8; ++i) x ^= a[i];                                                \
    if (x == 0x9u) out[0] = x;                                                            \
  }

KERNEL32(k_add, "v_add_u32 %0, %0, %1")
KERNEL32(k_lshl_add, "v_lshl_add_u32 %0, %0, 1, %1")
KERNEL32(k_perm, "v_perm_b32 %0, %0, %1, %2")
KERNEL32(k_alignbit, "v_alignbit_b32 %0, %0, %1, 24")
KERNEL32(k_dot4, "v_dot4_u32_u8 %0, %0, %1, %2")
KERNEL32(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
KERNEL32(k_mul24, "v_mul_u32_u24 %0, %0, %1")
KERNEL32(k_mad24, "v_mad_u32_u24 %0, %0, %1, %2")
KERNEL32(k_max3, "v_max3_i32 %0, %0, %1, %2")
KERNEL32(k_bfe, "v_bfe_u32 %0, %0, 8, 8")
KERNEL32(k_pk_add, "v_pk_add_u16 %0, %0, %1")
KERNEL32(k_sad, "v_sad_u8 %0, %0, %1, %2")
KERNEL32(k_lerp, "v_lerp_u8 %0, %0, %1, %2")
KERNEL32(k_and, "v_and_b32 %0, %0, %1")
KERNEL32(k_or, "v_or_b32 %0, %0, %1")
KERNEL32(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL32(k_max, "v_max_i32 %0, %0, %1")
KERNEL32(k_lshlrev, "v_lshlrev_b32 %0, 3, %0")
KERNEL32(k_add_sdwa, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2")
KERNEL32(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL32(k_or3, "v_or3_b32 %0, %0, %1, %2")
KERNEL32(k_lshl_or, "v_lshl_or_b32 %0, %0, 2, %1")
KERNEL32(k_add_e64, "v_add_u32_e64 %0, %0, %1")
KERNEL32(k_mad_u16, "v_mad_u32_u16 %0, %0, %1, %2")
KERNEL32(k_dot2, "v_dot2_u32_u16 %0, %0, %1, %2")
KERNEL32(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
KERNEL32(k_pk_mad, "v_pk_mad_u16 %0, %0, %1, %2")
KERNEL32(k_pk_fma, "v_pk_fma_f16 %0, %0, %1, %2")
KERNEL32(k_fma, "v_fma_f32 %0, %0, %1, %2")
KERNEL32(k_cvt_pk, "v_cvt_pk_u8_f32 %0, %1, 1, %0")
KERNEL32(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca")

#define KERNEL64(NAME, ASM)                                                               \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {             \
    uint64_t a[8], b = seed ^ threadIdx.x;                                                \
    for (int i = 0; i < 8; ++i) a[i] = seed + i * 77u + threadIdx.x;                      \
    for (int it = 0; it < ITERS; ++it) {                                                  \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(a[i]) : "v"(b)); \
    }                                                                                     \
    uint64_t x = 0;                                                                       \
    for (int i = 0; i < 8; ++i) x ^= a[i];                                                \
    if (x == 0x9u) out[0] = (uint32_t)x;                                                  \
  }

KERNEL64(k_lshl_add64, "v_lshl_add_u64 %0, %0, 0, %1")
__global__ void __launch_bounds__(256) k_mad64(uint32_t* out, uint32_t seed) {
  uint64_t a[8];
  const uint32_t b = seed ^ threadIdx.x;
  for (int i = 0; i < 8; ++i) a[i] = seed + i * 77u + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] = (uint64_t)(uint32_t)a[i] * b + a[i];
      asm volatile("" : "+v"(a[i]));
    }
  }
  uint64_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a[i];
  if (x == 0x9u) out[0] = (uint32_t)x;
}

int main() {
  int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int clk = 0; CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
  uint32_t* out; CK(hipMalloc(&out, 64));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  struct K { const char* name; void (*f)(uint32_t*, uint32_t); int ops_per; };
  K ks[] = {{"v_add_u32", k_add, 1}, {"v_lshl_add_u32", k_lshl_add, 1}, {"v_perm_b32", k_perm, 1},
            {"v_alignbit_b32", k_alignbit, 1}, {"v_dot4_u32_u8", k_dot4, 1}, {"v_mul_lo_u32", k_mul_lo, 1},
            {"v_mul_u32_u24", k_mul24, 1}, {"v_mad_u32_u24", k_mad24, 1}, {"v_max3_i32", k_max3, 1},
            {"v_bfe_u32", k_bfe, 1}, {"v_pk_add_u16", k_pk_add, 1}, {"v_sad_u8", k_sad, 1}, {"v_lerp_u8", k_lerp, 1},
            {"v_and_b32", k_and, 1}, {"v_or_b32", k_or, 1}, {"v_xor_b32", k_xor, 1}, {"v_max_i32", k_max, 1},
            {"v_lshlrev_b32", k_lshlrev, 1}, {"v_add_u32_sdwa", k_add_sdwa, 1}, {"v_add3_u32", k_add3, 1},
            {"v_or3_b32", k_or3, 1}, {"v_lshl_or_b32", k_lshl_or, 1}, {"v_add_u32_e64", k_add_e64, 1},
            {"v_mad_u32_u16", k_mad_u16, 1}, {"v_dot2_u32_u16", k_dot2, 1}, {"v_mul_hi_u32", k_mul_hi, 1},
            {"v_pk_mad_u16", k_pk_mad, 1}, {"v_pk_fma_f16", k_pk_fma, 1}, {"v_fma_f32", k_fma, 1},
            {"v_cvt_pk_u8_f32", k_cvt_pk, 1}, {"v_bitop3_b32", k_bitop3, 1},
            {"v_lshl_add_u64", k_lshl_add64, 1},
            {"v_mad_u64_u32", k_mad64, 1}};
  const int blocks = cus * 8, tpb = 256;
  printf("CUs %d, clock attr %d kHz\n", cus, clk);
  for (auto& k : ks) {
    float best = 1e9;
    for (int r = 0; r < 4; ++r) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(tpb), 0, 0, out, 12345u + r);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (r && ms < best) best = ms;
    }
    const double lane_ops = (double)blocks * tpb * ITERS * 8 * k.ops_per;
    printf("%-28s %8.3f ms  %8.1f G lane-instr/s  %6.1f lane-instr/clk/CU (at %d MHz)\n", k.name, best,
           lane_ops / best / 1e6, lane_ops / (best * 1e-3) / cus / (clk * 1e3), clk / 1000);
  }
  return 0;
}
