// The scan kernel with its ablation switches (tooling only): the round-4
// state of zc_scan_kernel's body as a template over ABL_* bits, moved out of
// the product source.  Each bit removes or alters one
// part of the work, for interleaved timing against the product kernel in
// tools/ubench/scan_ablate.hip (DESIGN 4.1's ablation numbers).  ABL = ABL_DMA_NT
// is the product kernel's work.  Included after zc_kernels.hip (it uses the
// product's helpers: stage_round, the ring reads, piece_hits, ...; the
// round-4 LDS layout -- a two-slot ring per wave, 8 waves -- is AblScanLds).
namespace zc {
namespace {

// Ablation bits (tools/ubench/scan_ablate.hip only; the product uses 0):
// 1 = no digest, 2 = no gear/anchors, 4 = anchors counted but not recorded,
// 8 = skip the per-byte work entirely (staging + reads only),
// 16 = gear + max computed but folded into the state without a ballot/branch,
// 32 = anchor threshold raised so the recording block is (almost) never taken,
// 64 = no tile-end work (span digests, anchors to the pool), 128 = no
// counter atomic, 256 = the tile end stores the span digests only
enum { ABL_NO_DIGEST = 1, ABL_NO_GEAR = 2, ABL_NO_RECORD = 4, ABL_NO_BYTES = 8, ABL_NO_BRANCH = 16,
       ABL_NEVER = 32, ABL_NO_TILE_END = 64, ABL_NO_ATOMIC = 128, ABL_TE_DIGEST_ONLY = 256,
       ABL_DMA_NT = 512, ABL_DMA_SC1 = 1024, ABL_STAGGER_HALF = 2048, ABL_STAGGER_QUARTER = 4096,
       ABL_NO_WARM = 8192, ABL_TE_NO_STORE = 16384, ABL_TE_NO_ANCHOR_STORE = 32768,
       ABL_TE_DIGEST_NT = 65536, ABL_TE_DIGEST_SAME = 131072, ABL_PRIO = 262144,
       ABL_DWORD_SAMPLED = 524288 /* timing only: anchors tested at dword ends only (experiment 16) */ };
// the product's scan: the staging DMA is non-temporal (the stream is read
// once; tools/ubench/scan_ablate.hip: 1.675 -> 1.560 ms per 8 GiB)
constexpr int kAblProduct = ABL_DMA_NT;

// One 16-byte piece of the scan (four dwords).  Gear: position k of a dword is
// g_k = (g << (k+1)) + sum_{j<=k} b_j 2^(k-j), the byte-weighted sums coming
// from v_dot4_u32_u8, so the four positions are independent of each other.
// Digest: two bytes per step, acc*257^2 + (257 b_0 + b_1) (v_perm + SDWA
// add for the pair, two v_mad_u64_u32 for the 64-bit multiply-add).  Anchor
// test: the max of the piece's sixteen gears (two v_max3 per dword), one
// compare and one ballot per piece.  The recording block is wave-uniform (the
// list count stays scalar) and entered for ~22 % of pieces at the 1/4096
// anchor rate: each lane with a hit appends the piece (its bytes, the gear
// before it and a link to the lane's previous entry) to the wave's LDS list,
// and the tile end re-derives the exact anchors from those 16 bytes.
// (ABL_DWORD_SAMPLED, timing only: the gear tested at dword ends alone -- a
// quarter of the positions -- saves 6 % of the kernel, but windows at other
// alignments then need every chunk's anchors in four residues, whose search
// costs more than that: DESIGN 4.1, experiment 16.)
template <int ABL>
__device__ __forceinline__ void abl_scan_piece(uint4 v, uint32_t rel, int32_t lo_thr, ScanLane& s, WaveList& wl,
                                           uint32_t& last) {
  const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
  if (ABL & ABL_NO_BYTES) {
    s.hlo ^= xs[0] ^ xs[1] ^ xs[2] ^ xs[3];
    return;
  }
  const uint32_t g0 = s.glo;  // gear before the piece
  uint32_t g[4][4];
  int32_t mx[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t x = xs[d];
    if ((ABL & ABL_DWORD_SAMPLED) && !(ABL & ABL_NO_GEAR)) {
      s.glo = (s.glo << 4) + __builtin_amdgcn_udot4(x, 0x01020408u, 0u, false);
      mx[d] = d == 0 ? (int32_t)s.glo : max(mx[d - 1], (int32_t)s.glo);
      g[d][3] = s.glo;
    } else if (!(ABL & ABL_NO_GEAR)) {
      const uint32_t dd[4] = {x & 0xFFu, __builtin_amdgcn_udot4(x, 0x00000102u, 0u, false),
                              __builtin_amdgcn_udot4(x, 0x00010204u, 0u, false),
                              __builtin_amdgcn_udot4(x, 0x01020408u, 0u, false)};
#pragma unroll
      for (int k = 0; k < 4; ++k) g[d][k] = (s.glo << (k + 1)) + dd[k];
      s.glo = g[d][3];
      // one max3 chain over the piece's 16 gears (8 v_max3_i32 per piece)
      mx[d] = d == 0 ? max(max((int32_t)g[0][0], (int32_t)g[0][1]), (int32_t)g[0][2])
                     : max(max(mx[d - 1], (int32_t)g[d - 1][3]), (int32_t)g[d][0]);
      if (d > 0) mx[d] = max(max(mx[d], (int32_t)g[d][1]), (int32_t)g[d][2]);
    }
    if (!(ABL & ABL_NO_DIGEST)) {
      // two bytes per Horner step: acc*257^2 + (257 b_0 + b_1).  One v_perm
      // swaps the bytes of each half (b_1 | b_0 << 8), an SDWA add adds b_0;
      // acc*66049 + t is a v_mad_u64_u32 on the low word and one on the
      // high word: 9 lane-ops per dword instead of 12
      const uint32_t sp = __builtin_amdgcn_perm(0u, x, 0x02030001u);
      const uint32_t t[2] = {(sp & 0xFFFFu) + (x & 0xFFu), (sp >> 16) + ((x >> 16) & 0xFFu)};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        // acc*66049 + t = lo*66049 + {t, hi*66049}: a v_mul_lo_u32 for the
        // high word feeds the 64-bit addend of ONE v_mad_u64_u32
        const v2u32 addend = {t[k], s.hhi * 66049u};
        const uint64_t R = (uint64_t)s.hlo * 66049u + __builtin_bit_cast(uint64_t, addend);
        s.hhi = (uint32_t)(R >> 32);
        s.hlo = (uint32_t)R;
      }
    }
  }
  if (ABL & ABL_NO_GEAR) return;
  const int32_t m = (ABL & ABL_DWORD_SAMPLED) ? mx[3] : max(mx[3], (int32_t)g[3][3]);
  if (ABL & ABL_NO_BRANCH) {
    s.hhi ^= (uint32_t)m;
    return;
  }
  if (ABL & ABL_NEVER) lo_thr = 0x7FFFFFFF;
  const uint64_t any = __ballot(m >= lo_thr);
  if (__builtin_expect(any != 0, 0)) {
    if (ABL & ABL_NO_RECORD) {
      wl.n += __popcll(any);
      return;
    }
    const uint32_t idx = wl.n + lane_prefix(any);
    if (m >= lo_thr && idx < ZC_WLIST) {
      wl.e[3 * idx] = ((rel >> 4) << 8) | last | (__lane_id() << 16);
      wl.e[3 * idx + 1] = g0;
      wl.x[idx] = v;
      last = idx;
    }
    wl.n += __popcll(any);
  }
}

// End of a tile: the lane's span digests; the wave's anchors, from its LDS
// piece list, to the wave-tile's pool share in position order; the directory
// entry and the anchor count.  Every lane walks only its own entries (a chain
// through the list, newest first, `last` = its newest): once to count --
// re-deriving each piece's anchor mask, kept in the entry's high half -- and
// once to store, visiting only the set bits (each anchor's gear from the gear
// before its dword and one v_dot4), so the list costs O(entries + anchors per
// lane).  Returns a lower bound of the global stores it leaves in flight, so
// the next round's wait can leave them be.  A wave-tile whose list or pool
// share overflowed is marked for the exact rescan (zc_anchor_rescan) and
// stores no anchors.
template <int ABL>
__device__ __forceinline__ uint32_t abl_scan_tile_end(uint64_t span0, uint32_t lane, int32_t lo_thr,
                                                  const uint64_t (&bk)[kDigests], const WaveList& wl,
                                                  uint32_t last, uint64_t* __restrict__ blk, PoolOut po,
                                                  uint32_t& acc_pool, uint32_t& acc_over) {
  uint4* bo = (uint4*)(blk + span0 / ZC_SPAN);
  if (ABL & ABL_TE_NO_STORE) {
    uint32_t x = 0;
#pragma unroll
    for (int t = 0; t < kDigests; ++t) x ^= (uint32_t)bk[t] ^ (uint32_t)(bk[t] >> 32);
    asm volatile("" ::"v"(x));
    return 0;
  }
  if (ABL & ABL_TE_DIGEST_SAME) bo = (uint4*)(blk + (span0 % ZC_STILE) / ZC_SPAN);  // timing only: L2-hot
#pragma unroll
  for (int t = 0; t < kDigests / 2; ++t) {
    const uint4 v = make_uint4((uint32_t)bk[2 * t], (uint32_t)(bk[2 * t] >> 32), (uint32_t)bk[2 * t + 1],
                               (uint32_t)(bk[2 * t + 1] >> 32));
    if (ABL & ABL_TE_DIGEST_NT)
      __builtin_nontemporal_store(*(const v4u32*)&v, (v4u32*)(bo + t));
    else
      bo[t] = v;
  }
  if (ABL & ABL_TE_DIGEST_ONLY) return kDigests / 2;
  const uint64_t wt = span0 >> ZC_WT_SHIFT;
  const uint32_t base = (uint32_t)(wt - po.wt0) * po.wcap;
  uint32_t tot = 0, excl = 0, nst = 0;
  bool over = wl.n > ZC_WLIST;
  if (!over) {
    const uint32_t ne = wl.n;  // <= ZC_WLIST
    const uint64_t tspan0 = span0 - (uint64_t)lane * ZC_LSPAN;  // the wave-tile's first byte
    // pass 1, over the entries (one per lane per step): each piece's anchor
    // mask, re-derived from its bytes and the gear before it
    for (uint32_t i = lane; i < ne; i += 64) {
      const uint32_t L = (wl.e[3 * i] >> 16) & 63u;
      wl.e[3 * i + 2] = piece_hits(wl, i, tspan0 + (uint64_t)L * ZC_LSPAN, lo_thr).mask;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // pass 2, along each lane's own chain (newest entry first): its counts,
    // the wave's prefix sum, then each entry's pool offset -- within each half
    // (either half may be the one taken first), so the wave-tile's anchors
    // land in position order
    uint32_t cnt = 0, cnt_lo = 0;  // cnt_lo: anchors in the span's first half
    for (uint32_t i = last; i != kNoEntry; i = wl.e[3 * i] & 0xFFu) {
      const uint32_t c = __popc(wl.e[3 * i + 2]);
      cnt += c;
      if ((((wl.e[3 * i] >> 8) & 0xFFu) << 4) < kHalfSpan) cnt_lo += c;
    }
    excl = wave_excl_scan(cnt, lane, &tot);
    over = tot > po.wcap;
    if (!over) {
      uint32_t k_lo = excl + cnt_lo, k_hi = excl + cnt;
      for (uint32_t i = last; i != kNoEntry; i = wl.e[3 * i] & 0xFFu) {
        const uint32_t m = wl.e[3 * i + 2];
        uint32_t& k = ((((wl.e[3 * i] >> 8) & 0xFFu) << 4) < kHalfSpan) ? k_lo : k_hi;
        k -= __popc(m);
        wl.e[3 * i + 2] = m | (k << 16);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      // pass 3, over the entries again: the stores, in one wave-uniform loop
      // (one anchor per lane per pass) whose store instructions are counted
      // exactly (nst): the next tile's first wait then leaves exactly them in
      // flight instead of draining the round prefetched behind them
      uint32_t i = lane, mask = 0, w = 0, sb = 0;
      uint32_t xs[4] = {0, 0, 0, 0}, gd[4] = {0, 0, 0, 0};
      for (;;) {
        // a lane whose entry is used up takes its next one (an entry's mask
        // may be empty: the stream's first positions are no anchors)
        while (!mask && i < ne) {
          const uint32_t e0 = wl.e[3 * i], e2 = wl.e[3 * i + 2];
          mask = e2 & 0xFFFFu;
          w = e2 >> 16;
          sb = ((e0 >> 16) & 63u) * ZC_LSPAN + (((e0 >> 8) & 0xFFu) << 4);  // in the wave-tile
          const uint4 v = wl.x[i];
          xs[0] = v.x;
          xs[1] = v.y;
          xs[2] = v.z;
          xs[3] = v.w;
          // the gear before each dword of the piece
          gd[0] = wl.e[3 * i + 1];
#pragma unroll
          for (int d = 0; d < 3; ++d) gd[d + 1] = (gd[d] << 4) + __builtin_amdgcn_udot4(xs[d], 0x01020408u, 0u, false);
          i += 64;
        }
        if (__ballot(mask != 0) == 0) break;
        if (ABL & ABL_TE_NO_ANCHOR_STORE) {
          mask = 0;
          continue;
        }
        if (mask) {
          const uint32_t t = __builtin_ctz(mask), d = t >> 2, q = t & 3u;
          const uint32_t gdd = d == 0 ? gd[0] : d == 1 ? gd[1] : d == 2 ? gd[2] : gd[3];
          const uint32_t xd = d == 0 ? xs[0] : d == 1 ? xs[1] : d == 2 ? xs[2] : xs[3];
          // g at position t: the dword's gear shifted q + 1, plus its first q + 1
          // bytes weighted 2^(q - j)
          const uint32_t g = (gdd << (q + 1)) + __builtin_amdgcn_udot4(xd, 0x01020408u >> (8 * (3 - q)), 0u, false);
          po.rel[base + w] = sb + t;
          po.g[base + w] = g;
          mask &= mask - 1;
          ++w;
        }
        nst += 2;
      }
    }
  }
  if (lane == 0) {
    po.base[wt] = base;
    po.cnt[wt] = over ? ZC_WT_OVERFLOW : tot;
  }
  // the pool / overflow counters are added once per wave at the kernel's end
  // (one same-address atomic per wave-tile serialised in L2: 1.5 % of the scan)
  acc_pool += over ? 0u : tot;
  acc_over += over ? 1u : 0u;
  return kDigests / 2 + __builtin_amdgcn_readfirstlane(nst) + 2;
}

struct AblScanLds {
  uint8_t ring[ZC_SCAN_TPB / 64][2 * 64 * ZC_ROUND];
  uint4 wdata[ZC_SCAN_TPB / 64][ZC_WLIST];
  uint32_t wlist[ZC_SCAN_TPB / 64][ZC_WLIST * 3];
};
template <int ABL>
__device__ __forceinline__ void abl_scan_body(
    const uint8_t* __restrict__ data, uint64_t n, uint64_t tile0, uint64_t ntiles, int32_t lo_thr,
    uint64_t* __restrict__ blk, PoolOut po, unsigned long long* __restrict__ counters, AblScanLds& L) {
  auto& ring = L.ring;
  auto& wlist = L.wlist;
  auto& wdata = L.wdata;
  constexpr uint32_t kRpt = kRounds;  // rounds per tile
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t grid = gridDim.x;
  uint8_t* myring = ring[wave];
  WaveList wl{wlist[wave], wdata[wave], 0};
  if (ABL & ABL_PRIO) __builtin_amdgcn_s_setprio(3);  // ablation: issue ahead of co-resident kernels' waves
  const uint32_t ntk = ntiles > blockIdx.x ? (uint32_t)((ntiles - 1 - blockIdx.x) / grid + 1) : 0;
  const uint32_t nR = ntk * kRpt;
  // this lane's share of DMA instruction j: row j * (1024 / ZC_ROUND) + lane /
  // kPieces of the wave, the source piece that lands at position lane % kPieces
  uint32_t lane_off[kDmaRound];
#pragma unroll
  for (int j = 0; j < kDmaRound; ++j) {
    const uint32_t row = j * (1024 / ZC_ROUND) + lane / kPieces;
    lane_off[j] = row * ZC_LSPAN + (row & 1) * kHalfSpan + ((lane % kPieces) ^ row_swizzle(row)) * 16;
  }
  const uint32_t sw = row_swizzle(lane);  // read-side swizzle of this lane's row
  const uint32_t hs = (lane & 1) * kHalfRounds;  // logical round r is physical round r ^ hs
  v4u32 warm[2] = {};                       // the 32 bytes before the next half span
  auto issue = [&](uint32_t Rx) {
    const uint32_t k = Rx / kRpt, r = Rx - k * kRpt;
    const uint64_t tile = tile0 + blockIdx.x + (uint64_t)k * grid;
    stage_round<((ABL & ABL_DMA_NT) ? 2 : 0) | ((ABL & ABL_DMA_SC1) ? 16 : 0)>(data, myring, wave, lane_off, tile,
                                                                                  (int)r, Rx & 1);
    if (!(ABL & ABL_NO_WARM) && r % kHalfRounds == 0) {
      // span 0 of the stream has no bytes before it: it reads itself (unused)
      const uint64_t at = tile * ZC_STILE + (uint64_t)tid * ZC_LSPAN + (uint64_t)(r ^ hs) * ZC_ROUND;
      const uint8_t* src = at >= 32 ? data + at - 32 : data + at;
      warm[0] = global_read16(src);
      warm[1] = global_read16(src + 16);
    }
  };
  if (ABL & (ABL_STAGGER_HALF | ABL_STAGGER_QUARTER)) {
    // ablation: odd waves start later, so a SIMD's two waves reach their
    // tile ends at different times
    if (wave & 1)
      for (int i = 0; i < ((ABL & ABL_STAGGER_HALF) ? 14 : 7); ++i) __builtin_amdgcn_s_sleep(127);
  }
  if (nR > 0) issue(0);
  if (nR > 1) issue(1);
  ScanLane s{0, 0, 0};
  uint64_t bk[kDigests];
#pragma unroll
  for (int t = 0; t < kDigests; ++t) bk[t] = 0;
  uint64_t span0 = 0;
  uint32_t tail_stores = 0;  // global stores the last tile end left in flight
  uint32_t last = kNoEntry;  // this lane's newest entry in the wave's list
  uint32_t acc_pool = 0, acc_over = 0;  // wave-uniform: anchors stored, wave-tiles overflowed

#pragma unroll 1
  for (uint32_t R = 0; R < nR; ++R) {
    const uint32_t k = R / kRpt;
    const int r = (int)(R - k * kRpt);
    // round R (and, for a half's first round, its warm-up loads) has landed
    // once only what was issued after it is outstanding: round R + 1's DMA,
    // plus the next half's warm-up loads before a half's first round, plus
    // the tile end's stores before round 0
    if (R + 1 >= nR) wait_vmcnt<0>();
    else if ((r + 1) % kHalfRounds == 0) wait_vmcnt<(ABL & ABL_NO_WARM) ? kDmaRound : kDmaRound + 2>();
    else if (r == 0) wait_vmcnt_dyn(kDmaRound + tail_stores);
    else wait_vmcnt<kDmaRound>();
    const uint8_t* row = myring + (R & 1) * (64 * ZC_ROUND);
    const uint32_t pr = (uint32_t)r ^ hs;  // the physical round in the lane span
    if (r == 0) {
      // a new tile
      span0 = (tile0 + blockIdx.x + (uint64_t)k * grid) * ZC_STILE + (uint64_t)tid * ZC_LSPAN;
      s = ScanLane{0, 0, 0};
      wl.n = 0;
      last = kNoEntry;
    }
    if (r % kHalfRounds == 0) {
      // a new half: the warm-up bytes prime the gear (its value depends on the
      // 32 bytes before only, so this equals the gear rolled on continuously)
      s.glo = 0;
      ties(warm);  // landed: the wait above covers them
      if (!(ABL & ABL_NO_WARM) && span0 + pr * ZC_ROUND >= 64) {
        const uint32_t xs[8] = {warm[0][0], warm[0][1], warm[0][2], warm[0][3],
                                warm[1][0], warm[1][1], warm[1][2], warm[1][3]};
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) gear_step((xs[j] >> (8 * q)) & 0xFFu, s);
      }
    }
    static_assert(kPieces == 8, "the round is read in two halves of four pieces");
    v4u32 va[4], vb[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) va[p] = lds_read16(row + lane * ZC_ROUND + ((p ^ sw) << 4));
#pragma unroll
    for (int p = 0; p < 4; ++p) vb[p] = lds_read16(row + lane * ZC_ROUND + (((p + 4) ^ sw) << 4));
    // the first four pieces are hashed while the last four are still in flight
    wait_lgkmcnt<4>();
    ties(va);
    const bool tile_end = r == kRounds - 1 && !(ABL & ABL_NO_TILE_END);
#pragma unroll
    for (int p = 0; p < 4; ++p) abl_scan_piece<ABL>(to_uint4(va[p]), pr * ZC_ROUND + p * 16, lo_thr, s, wl, last);
    wait_lgkmcnt<0>();  // the slot is free
    ties(vb);
    if (R + 2 < nR) issue(R + 2);
#pragma unroll
    for (int p = 0; p < 4; ++p)
      abl_scan_piece<ABL>(to_uint4(vb[p]), pr * ZC_ROUND + (p + 4) * 16, lo_thr, s, wl, last);
    if ((r + 1) % (ZC_SPAN / ZC_ROUND) == 0) {
      const uint64_t h = ((uint64_t)s.hhi << 32) | s.hlo;
      const uint32_t q = pr / (ZC_SPAN / ZC_ROUND);  // per lane: the halves are rotated
#pragma unroll
      for (int t = 0; t < kDigests; ++t) bk[t] = q == (uint32_t)t ? h : bk[t];
      s.hlo = s.hhi = 0;
    }
    if (tile_end) tail_stores = abl_scan_tile_end<ABL>(span0, lane, lo_thr, bk, wl, last, blk, po, acc_pool, acc_over);
  }
  if (!(ABL & ABL_NO_ATOMIC) && lane == 0) {
    if (acc_pool) atomicAdd(&counters[CNT_POOL], (unsigned long long)acc_pool);
    if (acc_over) atomicAdd(&counters[CNT_OVERFLOW], (unsigned long long)acc_over);
  }
}

template <int ABL>
__global__ void __launch_bounds__(ZC_SCAN_TPB, 1) abl_scan_kernel(
    const uint8_t* __restrict__ data, uint64_t n, uint64_t tile0, uint64_t ntiles, int32_t lo_thr,
    uint64_t* __restrict__ blk, PoolOut po, unsigned long long* __restrict__ counters) {
  __shared__ AblScanLds lds;
  abl_scan_body<ABL>(data, n, tile0, ntiles, lo_thr, blk, po, counters, lds);
}

}  // namespace
}  // namespace zc
