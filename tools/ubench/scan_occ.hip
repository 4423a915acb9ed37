// Occupancy experiment for the scan (tooling only, DESIGN 4.1 experiment 18).
// The product kernel runs 8 waves per CU (2 per SIMD): its 2-slot LDS ring
// (16 KiB per wave) plus the anchor list fill the CU's 160 KiB.  Here every
// wave walks whole 256 KiB wave-tiles on its own (the product's per-wave work,
// helpers shared: stage_round, scan_piece, scan_tile_end), so the workgroup
// size and the ring depth are free parameters:
//   RING = 2: the product's pipeline (two rounds in flight per wave);
//   RING = 1: the round is read from its slot into registers, the slot is
//             refilled with the next round, then the round is hashed (one round
//             in flight per wave, 12 KiB of LDS per wave: 12 waves = 3 per SIMD).
// Outputs (span digests, anchor pool) are compared with the product kernel's.
// Build: hipcc -O3 --offload-arch=gfx950 -I../../zbackup_amd/csrc scan_occ.hip -o scan_occ
#include "../../zbackup_amd/csrc/zc_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

namespace zc {
namespace {

template <int WAVES, int RING>
struct OccLds {
  uint8_t ring[WAVES][RING * 64 * ZC_ROUND];
  uint4 wdata[WAVES][ZC_WLIST];
  uint32_t wlist[WAVES][ZC_WLIST * 3];
};

template <int WAVES, int RING, int WPE>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(WPE)))
occ_scan_kernel(const uint8_t* __restrict__ data, uint64_t n, uint64_t nwt, int32_t lo_thr,
                uint64_t* __restrict__ blk, PoolOut po, unsigned long long* __restrict__ counters) {
  __shared__ OccLds<WAVES, RING> L;
  constexpr uint32_t kRpt = kRounds;
  constexpr uint32_t kWpt = ZC_SCAN_TPB / 64;  // wave-tiles per product tile
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t gw = blockIdx.x * WAVES + wave, nw = gridDim.x * WAVES;
  uint8_t* myring = L.ring[wave];
  WaveList wl{L.wlist[wave], L.wdata[wave], 0};
  const uint32_t ntk = nwt > gw ? (uint32_t)((nwt - 1 - gw) / nw + 1) : 0;
  const uint32_t nR = ntk * kRpt;
  uint32_t lane_off[kDmaRound];
#pragma unroll
  for (int j = 0; j < kDmaRound; ++j) {
    const uint32_t row = j * (1024 / ZC_ROUND) + lane / kPieces;
    lane_off[j] = row * ZC_LSPAN + (row & 1) * kHalfSpan + ((lane % kPieces) ^ row_swizzle(row)) * 16;
  }
  const uint32_t sw = row_swizzle(lane);
  const uint32_t hs = (lane & 1) * kHalfRounds;
  v4u32 warm[2] = {};
  auto issue = [&](uint32_t Rx) {
    const uint32_t k = Rx / kRpt, r = Rx - k * kRpt;
    const uint64_t wt = gw + (uint64_t)k * nw;
    stage_round<kScanDmaAux>(data, myring, (uint32_t)(wt % kWpt), lane_off, wt / kWpt, (int)r,
                             RING == 1 ? 0u : (Rx & 1));
    if (r % kHalfRounds == 0) {
      const uint64_t at = (wt << ZC_WT_SHIFT) + (uint64_t)lane * ZC_LSPAN + (uint64_t)(r ^ hs) * ZC_ROUND;
      const uint8_t* src = at >= 32 ? data + at - 32 : data + at;
      warm[0] = global_read16(src);
      warm[1] = global_read16(src + 16);
    }
  };
  if (nR > 0) issue(0);
  if (RING == 2 && nR > 1) issue(1);
  ScanLane s{0, 0, 0};
  uint64_t bk[kDigests];
#pragma unroll
  for (int t = 0; t < kDigests; ++t) bk[t] = 0;
  uint64_t span0 = 0;
  uint32_t tail_stores = 0, last = kNoEntry, acc_pool = 0, acc_over = 0;
#pragma unroll 1
  for (uint32_t R = 0; R < nR; ++R) {
    const uint32_t k = R / kRpt;
    const int r = (int)(R - k * kRpt);
    if constexpr (RING == 2) {
      if (R + 1 >= nR) wait_vmcnt<0>();
      else if ((r + 1) % kHalfRounds == 0) wait_vmcnt<kDmaRound + 2>();
      else if (r == 0) wait_vmcnt_dyn(kDmaRound + tail_stores);
      else wait_vmcnt<kDmaRound>();
    } else {
      // only round R (and its warm-up loads) was issued before the last
      // tile end's stores
      if (r == 0) wait_vmcnt_dyn(tail_stores);
      else wait_vmcnt<0>();
    }
    const uint8_t* row = myring + (RING == 1 ? 0u : (R & 1) * (64 * ZC_ROUND));
    const uint32_t pr = (uint32_t)r ^ hs;
    if (r == 0) {
      span0 = ((gw + (uint64_t)k * nw) << ZC_WT_SHIFT) + (uint64_t)lane * ZC_LSPAN;
      s = ScanLane{0, 0, 0};
      wl.n = 0;
      last = kNoEntry;
    }
    if (r % kHalfRounds == 0) {
      s.glo = 0;
      ties(warm);
      if (span0 + pr * ZC_ROUND >= 64) {
        const uint32_t xs[8] = {warm[0][0], warm[0][1], warm[0][2], warm[0][3],
                                warm[1][0], warm[1][1], warm[1][2], warm[1][3]};
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) gear_step((xs[j] >> (8 * q)) & 0xFFu, s);
      }
    }
    v4u32 va[4], vb[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) va[p] = lds_read16(row + lane * ZC_ROUND + ((p ^ sw) << 4));
    if constexpr (kPieces == 8) {
#pragma unroll
      for (int p = 0; p < 4; ++p) vb[p] = lds_read16(row + lane * ZC_ROUND + (((p + 4) ^ sw) << 4));
    }
    if constexpr (RING == 1) {
      wait_lgkmcnt<0>();  // the slot is read out: refill it with the next round
      ties(va);
      if constexpr (kPieces == 8) ties(vb);
      if (R + 1 < nR) issue(R + 1);
#pragma unroll
      for (int p = 0; p < 4; ++p) scan_piece(to_uint4(va[p]), pr * ZC_ROUND + p * 16, lo_thr, s, wl, last);
    } else if constexpr (kPieces == 8) {
      wait_lgkmcnt<4>();
      ties(va);
#pragma unroll
      for (int p = 0; p < 4; ++p) scan_piece(to_uint4(va[p]), pr * ZC_ROUND + p * 16, lo_thr, s, wl, last);
      wait_lgkmcnt<0>();
      ties(vb);
      if (R + 2 < nR) issue(R + 2);
    } else {
      wait_lgkmcnt<0>();
      ties(va);
      if (R + 2 < nR) issue(R + 2);
#pragma unroll
      for (int p = 0; p < 4; ++p) scan_piece(to_uint4(va[p]), pr * ZC_ROUND + p * 16, lo_thr, s, wl, last);
    }
    if constexpr (kPieces == 8) {
#pragma unroll
      for (int p = 0; p < 4; ++p) scan_piece(to_uint4(vb[p]), pr * ZC_ROUND + (p + 4) * 16, lo_thr, s, wl, last);
    }
    if ((r + 1) % (ZC_SPAN / ZC_ROUND) == 0) {
      const uint64_t h = ((uint64_t)s.hhi << 32) | s.hlo;
      const uint32_t q = pr / (ZC_SPAN / ZC_ROUND);
#pragma unroll
      for (int t = 0; t < kDigests; ++t) bk[t] = q == (uint32_t)t ? h : bk[t];
      s.hlo = s.hhi = 0;
    }
    if (r == kRounds - 1) tail_stores = scan_tile_end(span0, lane, lo_thr, bk, wl, last, blk, po, acc_pool, acc_over);
  }
  if (lane == 0) {
    if (acc_pool) atomicAdd(&counters[CNT_POOL], (unsigned long long)acc_pool);
    if (acc_over) atomicAdd(&counters[CNT_OVERFLOW], (unsigned long long)acc_over);
  }
}

}  // namespace
}  // namespace zc

using namespace zc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef void (*OccK)(const uint8_t*, uint64_t, uint64_t, int32_t, uint64_t*, PoolOut, unsigned long long*);

static uint64_t fnv(const std::vector<uint32_t>& v) {
  uint64_t h = 1469598103934665603ull;
  for (uint32_t x : v) h = (h ^ x) * 1099511628211ull;
  return h;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
  const int rounds = argc > 2 ? atoi(argv[2]) : 15;
  if (n % ZC_STILE) { printf("n must be a multiple of %llu\n", (unsigned long long)ZC_STILE); return 1; }
  uint8_t* d; CK(hipMalloc(&d, n));
  CK(launch_fill_splitmix64(d, n, 2024, 0));
  const uint64_t ntiles = n / ZC_STILE, nwt = wave_tiles(n);
  const uint32_t wcap = wave_tile_cap(65536);
  const int cus = cu_count();
  const int32_t lo = anchor_lo_for(65536);
  uint64_t* blk; uint32_t *dbase, *dcnt, *prel, *pg; unsigned long long* cnt;
  CK(hipMalloc(&blk, n / ZC_SPAN * 8)); CK(hipMalloc(&dbase, nwt * 4)); CK(hipMalloc(&dcnt, nwt * 4));
  CK(hipMalloc(&prel, nwt * wcap * 4)); CK(hipMalloc(&pg, nwt * wcap * 4)); CK(hipMalloc(&cnt, 128));
  const PoolOut po{dbase, dcnt, prel, pg, wcap, 0};
  struct V { const char* name; OccK k; int tpb; int wg_per_cu; std::vector<float> t; uint64_t sig; unsigned long long pool; };
  std::vector<V> vs = {
    {"product zc_scan_kernel", nullptr, 0, 0, {}, 0, 0},
#if ZC_ROUND_CFG == 64
    {"per-wave tiles, 4 waves x4, ring 1, wpe4", occ_scan_kernel<4, 1, 4>, 256, 4, {}, 0, 0},
    {"per-wave tiles, 4 waves x3, ring 2, wpe3", occ_scan_kernel<4, 2, 3>, 256, 3, {}, 0, 0},
    {"per-wave tiles, 4 waves x3, ring 1, wpe3", occ_scan_kernel<4, 1, 3>, 256, 3, {}, 0, 0},
    {"per-wave tiles, 4 waves x4, ring 1, wpe4 (again)", occ_scan_kernel<4, 1, 4>, 256, 4, {}, 0, 0},
#else
    {"per-wave tiles, 4 waves x3, ring 1, wpe3", occ_scan_kernel<4, 1, 3>, 256, 3, {}, 0, 0},
    {"per-wave tiles, 2 waves x6, ring 1, wpe3", occ_scan_kernel<2, 1, 3>, 128, 6, {}, 0, 0},
#endif
  };
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::vector<uint32_t> h32(n / ZC_SPAN * 2), hc(nwt);
  for (int round = 0; round <= rounds; ++round)
    for (auto& v : vs) {
      CK(hipMemset(cnt, 0, 128));
      CK(hipEventRecord(a));
      if (!v.k)
        CK(launch_scan_tiles(d, n, 0, ntiles, lo, blk, po, cnt, 0));
      else
        hipLaunchKernelGGL(v.k, dim3(cus * v.wg_per_cu), dim3(v.tpb), 0, 0, d, n, nwt, lo, blk, po, cnt);
      if (hipError_t e = hipGetLastError(); e != hipSuccess) {
        printf("%s: launch %s\n", v.name, hipGetErrorString(e));
        return 1;
      }
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (round) v.t.push_back(ms);
      if (round == 0) {  // outputs: span digests + directory counts + pool total
        CK(hipMemcpy(h32.data(), blk, h32.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hc.data(), dcnt, hc.size() * 4, hipMemcpyDeviceToHost));
        unsigned long long c[CNT_LAST];
        CK(hipMemcpy(c, cnt, sizeof(c), hipMemcpyDeviceToHost));
        v.sig = fnv(h32) ^ (fnv(hc) * 3);
        v.pool = c[CNT_POOL];
        CK(hipMemset(blk, 0, n / ZC_SPAN * 8));
        CK(hipMemset(dcnt, 0, nwt * 4));
      }
    }
  bool same = true;
  for (auto& v : vs) {
    std::sort(v.t.begin(), v.t.end());
    same = same && v.sig == vs[0].sig && v.pool == vs[0].pool;
    printf("%-42s median %7.3f ms  min %7.3f ms  %7.1f GB/s  outputs %016llx pool %llu%s\n", v.name,
           v.t[v.t.size() / 2], v.t[0], n / (v.t[0] * 1e6), (unsigned long long)v.sig, v.pool,
           v.sig == vs[0].sig && v.pool == vs[0].pool ? "" : "  DIFFERS");
  }
  printf(same ? "all outputs identical\n" : "OUTPUTS DIFFER\n");
  return same ? 0 : 2;
}
