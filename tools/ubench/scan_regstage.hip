// Register-staged scan prototype vs the shipped zc_scan_kernel (VERDICT r04
// item 2; DESIGN 4.1 names the variant).  Tooling only: interleaved rounds in
// one process, medians, and the outputs compared.
//
// The shipped kernel stages the stream through a per-wave LDS ring
// (buffer_load ... lds, then ds_read_b128) so that each lane reads a
// contiguous 4 KiB lane span.  Here the stream goes straight to registers with
// non-temporal global loads and no LDS: a wave walks its 256 KiB wave-tile row
// by row, a row is 4 KiB, lane l owns bytes [64 l, 64 l + 64) of every row
// (four 16-byte loads per lane per row, three rows in flight).  What that costs
// in VALU is the work a contiguous lane span does not need:
//   * the gear of a lane's first 31 positions needs the 32 bytes before them,
//     which belong to lane l - 1 (lane 0: the previous row's lane 63): every
//     lane first folds the gear of its own last 32 bytes (8 v_dot4 + 8
//     shift-adds), the values move one lane up (a DPP shift), and the lane's
//     full gear chain starts from its neighbour's value;
//   * a 1 KiB span digest is 16 lanes' 64-byte Horner accumulators, each
//     multiplied by 257^(64 (15 - l % 16)) and summed across the 16 lanes
//     (four 64-bit shuffle-add levels).
// Outputs: the span digests (must equal the shipped kernel's bit for bit) and
// the anchors (position, gear) of each wave-tile, appended in discovery order
// (the shipped kernel stores them sorted by position: the prototype does less
// work there, which only favours it); the totals are compared.
//
//   hipcc -O3 --offload-arch=gfx950 -I../../zbackup_amd/csrc -o scan_regstage scan_regstage.hip
//   ./scan_regstage [bytes] [rounds]
#include "../../zbackup_amd/csrc/zc_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace zc;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("HIP %s at line %d\n", hipGetErrorString(e_), __LINE__);           \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

namespace rs {

constexpr int kRow = 4096;                       // bytes per wave-row
constexpr int kLaneBytes = kRow / 64;            // 64 per lane
constexpr int kRowsPerWt = (64 * ZC_LSPAN) / kRow;  // rows of a 256 KiB wave-tile (64)
constexpr int kDepth = 3;                        // rows in flight ahead of the one hashed
constexpr uint32_t kPoolCap = 4096;              // anchors per wave-tile (prototype pool)

typedef unsigned v4u32 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4u32 ldnt(const uint8_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(p));
}

__device__ __forceinline__ uint64_t pow257(uint64_t e) {
  uint64_t r = 1, b = 257;
  while (e) {
    if (e & 1) r *= b;
    b *= b;
    e >>= 1;
  }
  return r;
}

struct Row {
  v4u32 v[4];
};

__device__ __forceinline__ void load_row(Row& r, const uint8_t* __restrict__ p) {
#pragma unroll
  for (int j = 0; j < 4; ++j) r.v[j] = ldnt(p + 16 * j);
}

// gear of the 32 bytes ending at the lane's last byte: sum b[63 - j] 2^j
__device__ __forceinline__ uint32_t tail_gear(const uint32_t (&x)[16]) {
  uint32_t g = 0;
#pragma unroll
  for (int d = 8; d < 16; ++d) g = (g << 4) + __builtin_amdgcn_udot4(x[d], 0x01020408u, 0u, false);
  return g;
}

// one wave-tile per wave (grid-stride over wave-tiles)
__global__ void __launch_bounds__(512, 1) rs_scan_kernel(const uint8_t* __restrict__ data, uint64_t nwt, int32_t lo_thr,
                                                         uint64_t* __restrict__ blk, uint32_t* __restrict__ pool_rel,
                                                         uint32_t* __restrict__ pool_g, uint32_t* __restrict__ pool_cnt) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t waves = gridDim.x * (blockDim.x >> 6);
  __shared__ uint32_t s_cnt[8];
  // this lane's multiplier into its 1 KiB span: 257^(64 (15 - l % 16))
  const uint64_t mul = pow257((uint64_t)kLaneBytes * (15 - (lane & 15)));
  for (uint64_t wt = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave; wt < nwt; wt += waves) {
    const uint8_t* base = data + (wt << ZC_WT_SHIFT);
    if (lane == 0) s_cnt[wave] = 0;
    // the gear before the wave-tile: its 32 preceding bytes (none for the first)
    uint32_t carry = 0;
    if (wt > 0) {
      const v4u32 a = ldnt(base - 32), b = ldnt(base - 16);
      const uint32_t x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
      uint32_t g = 0;
#pragma unroll
      for (int d = 0; d < 8; ++d) g = (g << 4) + __builtin_amdgcn_udot4(x[d], 0x01020408u, 0u, false);
      carry = __builtin_amdgcn_readfirstlane(g);
    }
    Row buf[kDepth + 1];
#pragma unroll
    for (int k = 0; k < kDepth; ++k) load_row(buf[k], base + (uint64_t)k * kRow + lane * kLaneBytes);
    uint32_t nanch = 0;  // this lane's anchors in the wave-tile (pool offsets come from the LDS counter)
#pragma unroll 1
    for (int r0 = 0; r0 < kRowsPerWt; r0 += kDepth + 1) {
#pragma unroll
      for (int u = 0; u <= kDepth; ++u) {
        const int r = r0 + u;
        if (r >= kRowsPerWt) break;
        // keep kDepth rows in flight: issue row r + kDepth into the free buffer
        if (r + kDepth < kRowsPerWt)
          load_row(buf[(u + kDepth) % (kDepth + 1)], base + (uint64_t)(r + kDepth) * kRow + lane * kLaneBytes);
        const Row& R = buf[u];
        const uint32_t x[16] = {R.v[0][0], R.v[0][1], R.v[0][2], R.v[0][3], R.v[1][0], R.v[1][1],
                                R.v[1][2], R.v[1][3], R.v[2][0], R.v[2][1], R.v[2][2], R.v[2][3],
                                R.v[3][0], R.v[3][1], R.v[3][2], R.v[3][3]};
        // the neighbour's tail gear starts this lane's chain
        const uint32_t tg = tail_gear(x);
        uint32_t up = __shfl_up(tg, 1, 64);
        up = lane == 0 ? carry : up;
        carry = __builtin_amdgcn_readlane(tg, 63);
        uint32_t glo = up;
        uint32_t hlo = 0, hhi = 0;
        const uint32_t rel0 = (uint32_t)(r * kRow + lane * kLaneBytes);
#pragma unroll
        for (int pc = 0; pc < 4; ++pc) {  // 16-byte pieces
          uint32_t g[4][4];
          int32_t mx = (int32_t)0x80000000;
          const uint32_t g0 = glo;
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const uint32_t w = x[4 * pc + d];
            const uint32_t dd[4] = {w & 0xFFu, __builtin_amdgcn_udot4(w, 0x00000102u, 0u, false),
                                    __builtin_amdgcn_udot4(w, 0x00010204u, 0u, false),
                                    __builtin_amdgcn_udot4(w, 0x01020408u, 0u, false)};
#pragma unroll
            for (int k = 0; k < 4; ++k) g[d][k] = (glo << (k + 1)) + dd[k];
            glo = g[d][3];
            mx = max(max(mx, (int32_t)g[d][0]), (int32_t)g[d][1]);
            mx = max(max(mx, (int32_t)g[d][2]), (int32_t)g[d][3]);
            // digest: two bytes per Horner step, as the shipped kernel
            const uint32_t sp = __builtin_amdgcn_perm(0u, w, 0x02030001u);
            const uint32_t t[2] = {(sp & 0xFFFFu) + (w & 0xFFu), (sp >> 16) + ((w >> 16) & 0xFFu)};
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              const uint64_t R64 = (uint64_t)hlo * 66049u + ((uint64_t)(hhi * 66049u) << 32 | t[k]);
              hhi = (uint32_t)(R64 >> 32);
              hlo = (uint32_t)R64;
            }
          }
          const uint64_t any = __ballot(mx >= lo_thr);
          if (__builtin_expect(any != 0, 0)) {
            if (mx >= lo_thr) {
              // this piece's anchors, in position order, appended to the wave-tile's pool
              uint32_t gg = g0;
              const uint64_t span_pos = (wt << ZC_WT_SHIFT) + rel0 + 16 * pc;
#pragma unroll
              for (int d = 0; d < 4; ++d) {
                const uint32_t w = x[4 * pc + d];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                  gg = (gg << 1) + ((w >> (8 * k)) & 0xFFu);
                  const uint64_t p = span_pos + 4 * d + k;
                  if ((int32_t)gg >= lo_thr && p >= ZC_ANCHOR_MIN_OFF) {
                    const uint32_t o = atomicAdd(&s_cnt[wave], 1u);
                    if (o < kPoolCap) {
                      pool_rel[wt * kPoolCap + o] = rel0 + 16 * pc + 4 * d + k;
                      pool_g[wt * kPoolCap + o] = gg;
                    }
                    ++nanch;
                  }
                }
              }
            }
          }
        }
        // the 1 KiB span digest: 16 lanes' 64-byte accumulators, weighted and summed
        uint64_t y = (((uint64_t)hhi << 32) | hlo) * mul;
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) y += (uint64_t)__shfl_xor((long long)y, m, 64);
        if ((lane & 15) == 0) blk[((wt << ZC_WT_SHIFT) + (uint64_t)r * kRow) / ZC_SPAN + (lane >> 4)] = y;
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) pool_cnt[wt] = s_cnt[wave];
    (void)nanch;
  }
}

// reads only (no hashing): the prototype's load pattern (lane: 64 bytes of
// each 4 KiB row, four 16-byte loads) against fully coalesced rows (lane: 16
// bytes of each 1 KiB row), same depth, the XOR of everything kept live
template <int kLaneB>
__global__ void __launch_bounds__(512, 1) rs_loads_kernel(const uint8_t* __restrict__ data, uint64_t nwt,
                                                          uint32_t* __restrict__ sink) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t waves = gridDim.x * (blockDim.x >> 6);
  constexpr int kRowB = 64 * kLaneB, kLoads = kLaneB / 16, kRows = (64 * ZC_LSPAN) / kRowB;
  uint32_t acc = 0;
  for (uint64_t wt = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave; wt < nwt; wt += waves) {
    const uint8_t* base = data + (wt << ZC_WT_SHIFT) + lane * kLaneB;
#pragma unroll 1
    for (int r = 0; r < kRows; r += 4) {
      v4u32 v[4][kLoads];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < kLoads; ++j) v[u][j] = ldnt(base + (uint64_t)(r + u) * kRowB + 16 * j);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < kLoads; ++j) acc ^= v[u][j][0] ^ v[u][j][1] ^ v[u][j][2] ^ v[u][j][3];
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

}  // namespace rs

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
  const int rounds = argc > 2 ? atoi(argv[2]) : 15;
  if (n % ZC_STILE) {
    printf("n must be a multiple of %llu\n", (unsigned long long)ZC_STILE);
    return 2;
  }
  uint8_t* d;
  CK(hipMalloc(&d, n));
  CK(launch_fill_splitmix64(d, n, 2024, 0));
  const uint64_t ntiles = n / ZC_STILE, nwt = wave_tiles(n);
  const uint32_t wcap = wave_tile_cap(65536);
  const int32_t lo = anchor_lo_for(65536);
  const int cus = cu_count();
  uint64_t *blkA, *blkB;
  uint32_t *dbase, *dcnt, *prel, *pg, *rrel, *rg, *rcnt;
  unsigned long long* cnt;
  CK(hipMalloc(&blkA, n / ZC_SPAN * 8));
  CK(hipMalloc(&blkB, n / ZC_SPAN * 8));
  CK(hipMalloc(&dbase, nwt * 4));
  CK(hipMalloc(&dcnt, nwt * 4));
  CK(hipMalloc(&prel, nwt * wcap * 4));
  CK(hipMalloc(&pg, nwt * wcap * 4));
  CK(hipMalloc(&rrel, nwt * rs::kPoolCap * 4));
  CK(hipMalloc(&rg, nwt * rs::kPoolCap * 4));
  CK(hipMalloc(&rcnt, nwt * 4));
  CK(hipMalloc(&cnt, 64));
  const PoolOut po{dbase, dcnt, prel, pg, wcap, 0};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto runA = [&]() {
    hipMemsetAsync(cnt, 0, 64, 0);
    (void)launch_scan_tiles(d, n, 0, ntiles, lo, blkA, po, cnt, 0);
  };
  // wpc: workgroups of 8 waves per CU (no LDS ring: up to 4 waves per SIMD fit 119 VGPRs)
  auto runB = [&](int wpc) {
    hipLaunchKernelGGL(rs::rs_scan_kernel, dim3(cus * wpc), dim3(512), 0, 0, d, nwt, lo, blkB, rrel, rg, rcnt);
  };
  // outputs: span digests equal, anchor totals equal (per wave-tile)
  runA();
  runB(1);
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> ha(n / ZC_SPAN), hb(n / ZC_SPAN);
  CK(hipMemcpy(ha.data(), blkA, ha.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb.data(), blkB, hb.size() * 8, hipMemcpyDeviceToHost));
  std::vector<uint32_t> ca(nwt), cb(nwt);
  CK(hipMemcpy(ca.data(), dcnt, nwt * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(cb.data(), rcnt, nwt * 4, hipMemcpyDeviceToHost));
  uint64_t dig_diff = 0, cnt_diff = 0, anc = 0;
  for (size_t i = 0; i < ha.size(); ++i) dig_diff += ha[i] != hb[i];
  for (size_t i = 0; i < nwt; ++i) {
    cnt_diff += ca[i] != cb[i];
    anc += cb[i];
  }
  printf("span digests differing: %llu of %zu; wave-tiles with other anchor counts: %llu of %llu (%llu anchors)\n",
         (unsigned long long)dig_diff, ha.size(), (unsigned long long)cnt_diff, (unsigned long long)nwt,
         (unsigned long long)anc);
  std::vector<float> t[5];
  for (int r = 0; r < rounds; ++r)
    for (int v = 0; v < 3; ++v) {
      float ms;
      CK(hipEventRecord(a));
      if (v == 0) runA();
      else runB(v);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      if (r) t[v].push_back(ms);
    }
  const char* names[5] = {"shipped zc_scan_kernel (LDS ring)", "register-staged, 2 waves/SIMD",
                          "register-staged, 4 waves/SIMD", "loads only, 64 B per lane per row",
                          "loads only, 16 B per lane per row"};
  for (int r = 0; r < rounds; ++r)
    for (int v = 3; v < 5; ++v) {
      float ms;
      CK(hipEventRecord(a));
      if (v == 3) hipLaunchKernelGGL(rs::rs_loads_kernel<64>, dim3(cus), dim3(512), 0, 0, d, nwt, rcnt);
      else hipLaunchKernelGGL(rs::rs_loads_kernel<16>, dim3(cus), dim3(512), 0, 0, d, nwt, rcnt);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      if (r) t[v].push_back(ms);
    }
  for (int v = 0; v < 5; ++v) {
    std::sort(t[v].begin(), t[v].end());
    printf("%-36s median %.3f ms  min %.3f ms  %.1f GB/s\n", names[v], t[v][t[v].size() / 2], t[v][0],
           n / (t[v][t[v].size() / 2] * 1e6));
  }
  return dig_diff || cnt_diff ? 1 : 0;
}
