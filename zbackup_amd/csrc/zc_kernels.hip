// zc_kernels.hip -- CDNA4 (gfx950) kernels of the rolling-hash chunking engine.
//
// The reference runs its 64-bit Rabin-Karp hash one byte at a time on one core
// and probes a hash map at every byte (backup_creator.cc:85-107,
// chunk_index.cc:119-143).  Here the stream is device resident and processed by
// lanes that each own a contiguous 1 KiB span:
//
//   zc_scan        ONE pass over the stream (the HBM-bound kernel): per byte it
//                  advances the 64-bit Rabin-Karp digest of the lane's span
//                  (base 257, mod 2^64 -- rolling_hash.hh:54-61 Horner form) and
//                  a content-defined gear hash whose rare hits ("anchors") are
//                  compacted with a per-lane LDS stage + block prefix sum.
//   zc_chunk_meta  64-bit keys of candidate grid chunks (Horner fold of span
//                  digests) + the first anchor inside each chunk.
//   zc_table_*     device hash table: anchor fingerprint -> chunk.
//   zc_probe       every anchor of the stream probes the table; a hit names a
//                  window that may equal an indexed chunk.
//   zc_verify      byte-exact check of candidate windows (one wave per window).
//   zc_range_digest  RollingHash::digest(buf, size) of arbitrary byte ranges
//                  (rolling_hash.cc:19-29) from span digests.
//   zc_fscan       per-byte 32-bit screen of the exact window hash H(p) against
//                  keys that have no anchor (static index entries, low-entropy
//                  chunks such as all-zero ones); maximal hit runs are emitted.
//   zc_sha1        SHA-1 of byte ranges (chunk ids, backup_creator.cc:130-131).
//
// No MFMA: this is integer/byte work bound by HBM reads.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "zc_device.h"

namespace zc {

namespace {

constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;
typedef unsigned v2u32 __attribute__((ext_vector_type(2)));

// Wave issue priority for the short, latency-bound kernels (chunk metadata,
// index inserts, probe, class joins, historic registration, range digests).
// With ZC_FLAG_SHA1 they run while the grid SHA-1 kernel holds every SIMD
// (VALU-bound, 96 % busy): a SIMD issues to the highest-priority ready wave,
// oldest first among equals, so without this a kernel dispatched after the
// SHA-1 waves only got their stall cycles (chunk metadata 1.2 ms instead of
// 25 us, zc_ref_meta 21-412 us).  s_setprio only changes the
// arbitration order of this wave's instructions; it has no other effect.
#define ZC_URGENT() __builtin_amdgcn_s_setprio(3)

__host__ __device__ inline uint64_t pow257_dev(uint64_t e) {
  uint64_t r = 1, b = 257;
  while (e) {
    if (e & 1) r *= b;
    b *= b;
    e >>= 1;
  }
  return r;
}

// 257^ZC_SPAN mod 2^64, the multiplier that appends one whole span digest
__device__ __forceinline__ uint64_t span_mul() { return pow257_dev(ZC_SPAN); }

// Exclusive prefix sum over the threads of a block (at most 1024).
__device__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_tmp, uint32_t& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_tmp[wid] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
  for (int w = 0; w < nw; ++w) {
    uint32_t t = s_tmp[w];
    pre += (w < wid) ? t : 0u;
    tot += t;
  }
  total = tot;
  __syncthreads();
  return pre + x - v;
}

// Rabin-Karp accumulator (no leading 257^len term) of bytes [a, b):
// sum_i data[i] * 257^(b-1-i) mod 2^64, folding whole spans from blk[].
// acc * 257^(b - a) + the bytes [a, b) Horner-folded (mod 2^64): bytes up to a
// 16-byte boundary one at a time, then 16-byte loads folded two bytes per
// step (acc * 257^2 + 257 b_0 + b_1), then the rest one at a time.  (The
// stream base is 16-byte aligned, so absolute offsets give the alignment.)
template <bool kVec = true>
__device__ __forceinline__ uint64_t rk_bytes(const uint8_t* __restrict__ data, uint64_t acc, uint64_t a, uint64_t b) {
  if (!kVec) {
    for (; a < b; ++a) acc = acc * 257u + data[a];
    return acc;
  }
  for (; a < b && (a & 15); ++a) acc = acc * 257u + data[a];
  for (; a + 16 <= b; a += 16) {
    const uint4 v = *(const uint4*)(data + a);
    const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t x = xs[d];
      acc = acc * 66049u + ((x & 0xFFu) * 257u + ((x >> 8) & 0xFFu));
      acc = acc * 66049u + (((x >> 16) & 0xFFu) * 257u + (x >> 24));
    }
  }
  for (; a < b; ++a) acc = acc * 257u + data[a];
  return acc;
}

// (kVec = false: the edges one byte at a time -- for the screen kernels, whose
// lane start states need no edges at W = 0 mod 1 KiB and whose register
// allocation the vector edge loop disturbed: the two-level screen ran 2.5 ->
// 3.7 ms per GiB with it inlined, round 5)
template <bool kVec = true>
__device__ uint64_t rk_acc(const uint8_t* __restrict__ data, const uint64_t* __restrict__ blk,
                           uint64_t a, uint64_t b) {
  uint64_t acc = 0;
  uint64_t a_up = (a + ZC_SPAN - 1) / ZC_SPAN * ZC_SPAN;
  if (a_up >= b) return rk_bytes<kVec>(data, 0, a, b);
  acc = rk_bytes<kVec>(data, 0, a, a_up);
  uint64_t b_dn = b / ZC_SPAN * ZC_SPAN;
  const uint64_t m = span_mul();
  uint64_t k = a_up / ZC_SPAN;
  const uint64_t k1 = b_dn / ZC_SPAN;
  // span digests sixteen loads at a time (the fold is a dependent chain; the
  // loads need not be)
  for (; k + 16 <= k1; k += 16) {
    uint64_t v[16];
    if ((k & 1) == 0) {  // 16-byte loads, two digests each
      const uint4* q = (const uint4*)(blk + k);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint4 t = q[i];
        v[2 * i] = ((uint64_t)t.y << 32) | t.x;
        v[2 * i + 1] = ((uint64_t)t.w << 32) | t.z;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = blk[k + i];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) acc = acc * m + v[i];
  }
  if (k + 8 <= k1) {
    uint64_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = blk[k + i];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc = acc * m + v[i];
    k += 8;
  }
  for (; k < k1; ++k) acc = acc * m + blk[k];
  return rk_bytes<kVec>(data, acc, b_dn, b);
}

__device__ uint32_t rk_acc32(const uint8_t* __restrict__ data, const uint64_t* __restrict__ blk,
                             uint64_t a, uint64_t b) {
  // the same fold in 32-bit arithmetic (reduction mod 2^32 commutes)
  uint32_t acc = 0;
  uint64_t a_up = (a + ZC_SPAN - 1) / ZC_SPAN * ZC_SPAN;
  if (a_up >= b) {
    for (uint64_t i = a; i < b; ++i) acc = acc * 257u + data[i];
    return acc;
  }
  for (uint64_t i = a; i < a_up; ++i) acc = acc * 257u + data[i];
  uint64_t b_dn = b / ZC_SPAN * ZC_SPAN;
  const uint32_t m = (uint32_t)span_mul();
  for (uint64_t k = a_up / ZC_SPAN; k < b_dn / ZC_SPAN; ++k) acc = acc * m + (uint32_t)blk[k];
  for (uint64_t i = b_dn; i < b; ++i) acc = acc * 257u + data[i];
  return acc;
}

// 4 bytes at an arbitrary byte address with aligned dword loads (the second
// word is only touched when the address is unaligned, and then it holds a byte
// we need, so no read leaves the granule of a valid byte).
__device__ __forceinline__ uint32_t load4_any(const uint8_t* base, uint64_t addr) {
  const uint32_t* w = (const uint32_t*)(base + (addr & ~3ull));
  uint32_t mis = (uint32_t)(addr & 3);
  uint32_t lo = w[0];
  if (mis == 0) return lo;
  uint32_t hi = w[1];
  return __builtin_amdgcn_alignbyte(hi, lo, mis);
}

// ---------------------------------------------------------------------------
// zc_scan (the HBM-bound pass)
//
// Persistent workgroups of 4 waves (one per SIMD), two workgroups per CU (two
// waves per SIMD); each lane owns a 4 KiB span, a wave's 64 spans are a
// 256 KiB wave-tile, and every wave walks wave-tiles on its own (2 MiB tiles of
// 8 wave-tiles remain the unit of launch_scan_tiles).  Every wave streams its
// own 64 rows through a private ONE-slot LDS ring of 128-byte rounds with
// buffer_load ... lds (non-temporal): a round is read out of the slot, the slot
// is refilled with the next round, then the round is hashed, so one round is
// in flight per wave while it computes.  One DMA instruction fills 8 rows x
// 128 B (whole cache lines); the LDS image is linear and the global source is
// swizzled (piece p of row i sits at piece p ^ ((i >> 1) & 7)), so the per-lane
// ds_read_b128 of a row is bank-conflict free (MI355X_MICROARCH.md §LDS lane
// groups); odd lanes take the two halves of their span in the other order (a
// row stride of 4 KiB alone cost the staging 12 %).  The 32 bytes before each
// half span (the anchor state's warm-up) are two register loads issued with
// the DMA of the half's first round.  Waves never touch each other's LDS: no
// barriers.  (DESIGN 4.1 has the measured geometry experiments 1-22.)
//
// Anchors are appended to a per-wave LDS list (one ballot per 16-byte piece; a
// wave-uniform block in the ~22 % of pieces where any lane hits) and moved to
// the wave-tile's pool share once per wave-tile, in position order, with their
// store instructions counted so the next round's wait leaves them in flight.
struct ScanLane {
  uint32_t glo;       // anchor state {st(q - 1), st(q)} after position q (zc_device.h)
  uint32_t hlo, hhi;  // 64-bit Rabin-Karp accumulator of the current 1 KiB span
};

// One byte of the anchor state: st(q + 1) = 2 st(q - 1) + b[q + 1] (mod 2^16)
// joins as the high half, st(q) moves down.  The scalar form (tail, rescan).
__device__ __forceinline__ void gear_step(uint32_t b, ScanLane& s) {
  s.glo = (s.glo >> 16) | (((s.glo << 1) + b) << 16);
}

// The packed form: the two halves of the state are the even- and odd-position
// streams, so v_pk_mad_u16 advances both by one byte each.  A dword at an even
// position 4t: {b0, b1} and {b2, b3} as u16 pairs (one v_perm each), two
// steps; the state after the first is {st(4t), st(4t + 1)}, after the second
// {st(4t + 2), st(4t + 3)}.  `two` is 0x00020002 (an SGPR operand keeps the
// compiler from splitting the multiply into a shift and an add).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_step(uint32_t S, uint32_t P, uint32_t two) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, S) * __builtin_bit_cast(u16x2, two) +
                                          __builtin_bit_cast(u16x2, P));
}
__device__ __forceinline__ uint32_t pk_max16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(i16x2, a),
                                                                __builtin_bit_cast(i16x2, b)));
}
__device__ __forceinline__ uint32_t bytes01(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0C010C00u); }
__device__ __forceinline__ uint32_t bytes23(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0C030C02u); }
// the larger signed half of a packed pair
__device__ __forceinline__ int32_t hmax16(uint32_t m) { return max((int32_t)(int16_t)m, (int32_t)m >> 16); }
__device__ __forceinline__ uint32_t pk_two() {
  uint32_t t;
  asm volatile("s_mov_b32 %0, 0x20002" : "=s"(t));
  return t;
}
// The anchor key at each position of a dword, from the state before it (S)
// and after its two steps (S1, S2): {st(q - 1), st(q)} for q = 4t .. 4t + 3
__device__ __forceinline__ uint32_t dword_key(uint32_t S, uint32_t S1, uint32_t S2, uint32_t k) {
  return k == 0 ? __builtin_amdgcn_alignbit(S1, S, 16) : k == 1 ? S1 : k == 2 ? __builtin_amdgcn_alignbit(S2, S1, 16) : S2;
}

__device__ __forceinline__ void digest_step(uint32_t b, ScanLane& s) {
  // acc*257 + b  (mod 2^64)
  uint64_t h = (((uint64_t)s.hhi << 32) | s.hlo) * 257u + b;
  s.hlo = (uint32_t)h;
  s.hhi = (uint32_t)(h >> 32);
}

// 64-bit fingerprint of anchor position q (q >= 63).
// Computed lazily from HBM -- only for chunk first-anchors and for stream
// anchors whose gear value hits the table -- so the scan keeps no per-byte
// fingerprint state.  Any fixed function of those bytes works: both sides
// (chunks and stream windows) use this one.
__device__ __forceinline__ uint32_t load4_any(const uint8_t* base, uint64_t addr);
__device__ uint64_t anchor_fp(const uint8_t* __restrict__ data, uint64_t q) {
  // the 8 bytes ending at q (the anchor key adds the 32 before; a key has
  // only ~20 free bits, these 64 make a false match rare)
  return ((uint64_t)load4_any(data, q - 3) << 32) | load4_any(data, q - 7);
}

// The staging DMA's cache policy: non-temporal (the stream is read once;
// interleaved A/B in tools/ubench/scan_ablate.hip: 1.675 -> 1.560 ms per 8 GiB).
// The ablation switches the round-4 scan carried (DESIGN 4.1's experiments)
// live in tools/ubench/scan_ablate_kernel.hip, not in the product.
constexpr int kScanDmaAux = 2;  // buffer_load ... lds, nt

struct WaveList {   // per-wave LDS list of pieces holding anchors
  uint32_t* e;      // {the lane's previous entry | (rel of the piece >> 4) << 8 | lane << 16, gear before
                    //  the piece, tile-end scratch: anchor mask | pool offset << 16}
  uint4* x;         // the piece's 16 bytes
  uint32_t n;       // wave-uniform count (may exceed capacity: then rescan)
};

__device__ __forceinline__ uint32_t lane_prefix(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// One 16-byte piece of the scan (four dwords).  Anchor state: two v_perm give
// a dword's byte pairs {b0, b1}, {b2, b3}; two v_pk_mad_u16 advance the even
// and the odd stream (pk_step).  Digest: two bytes per step, acc*257^2 +
// (257 b_0 + b_1), the addend a v_dot2_u32_u16 of the same byte pair, the
// 64-bit multiply-add a v_mul_lo_u32 + v_mad_u64_u32.  Anchor test: a
// v_pk_max_i16 chain over the piece's sixteen states (two per dword), one
// compare and one ballot per piece: 12 VALU per dword where the 32-bit gear
// took 16.5.  The recording block is wave-uniform (the
// list count stays scalar) and entered for ~22 % of pieces at the 1/4096
// anchor rate: each lane with a hit appends the piece (its bytes, the state
// before it and a link to the lane's previous entry) to the wave's LDS list,
// and the tile end re-derives the exact anchors from those 16 bytes.
// (Anchors tested at dword ends alone -- a quarter of the positions -- save
// 6 % of the kernel, but windows at other alignments then need every chunk's
// anchors in four residues, whose search costs more than that: DESIGN 4.1,
// experiment 16.)
__device__ __forceinline__ void scan_piece(uint4 v, uint32_t rel, int32_t lo_thr, uint32_t two, ScanLane& s,
                                           WaveList& wl, uint32_t& last) {
  const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
  const uint32_t g0 = s.glo;  // anchor state before the piece
  uint32_t m = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t x = xs[d];
    // the byte pairs feed both the anchor state and the digest
    const uint32_t p01 = bytes01(x), p23 = bytes23(x);
    const uint32_t S1 = pk_step(s.glo, p01, two), S2 = pk_step(S1, p23, two);
    s.glo = S2;
    // one v_pk_max_i16 chain over the piece's 16 states (st(q) of every q)
    m = d == 0 ? pk_max16(S1, S2) : pk_max16(pk_max16(m, S1), S2);
    // two bytes per Horner step: acc*257^2 + (257 b_0 + b_1), the addend one
    // v_dot2_u32_u16 of a byte pair; acc*66049 + t is a v_mad_u64_u32 on the
    // low word and a v_mul_lo_u32 on the high one
    const uint32_t t[2] = {__builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, p01), (u16x2){257, 1}, 0u, false),
                           __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, p23), (u16x2){257, 1}, 0u, false)};
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
  const bool hit = hmax16(m) >= lo_thr;
  const uint64_t any = __ballot(hit);
  if (__builtin_expect(any != 0, 0)) {
    const uint32_t idx = wl.n + lane_prefix(any);
    if (hit && idx < ZC_WLIST) {
      wl.e[3 * idx] = ((rel >> 4) << 8) | last | (__lane_id() << 16);
      wl.e[3 * idx + 1] = g0;
      wl.x[idx] = v;
      last = idx;
    }
    wl.n += __popcll(any);
  }
}

// 16 stream bytes at q (16-byte aligned), zero past the end of the stream
__device__ __forceinline__ uint4 load16_clamped(const uint8_t* __restrict__ data, uint64_t n, uint64_t q) {
  if (q + 16 <= n) return *(const uint4*)(data + q);
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint64_t i = q; i < n && i < q + 16; ++i) w[(i - q) >> 2] |= (uint32_t)data[i] << (8 * ((i - q) & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// One 1 KiB sub-span [q0, min(q0 + 1024, n)) (q0 1 KiB aligned) read with
// 16-byte loads, eight in flight: emit(pos, gear) for each anchor in order;
// returns the sub-span's 64-bit Rabin-Karp digest (the block digest).  For
// the partial last tile and the exact rescan of overflowed wave-tiles.
template <class Emit>
__device__ uint64_t subspan_pass(const uint8_t* __restrict__ data, uint64_t n, uint64_t q0, int32_t lo_thr,
                                 Emit&& emit) {
  ScanLane s{0, 0, 0};
  if (q0 >= 32) {
    const uint4 w[2] = {*(const uint4*)(data + q0 - 32), *(const uint4*)(data + q0 - 16)};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t xs[4] = {w[k].x, w[k].y, w[k].z, w[k].w};
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int j = 0; j < 4; ++j) gear_step((xs[d] >> (8 * j)) & 0xFFu, s);
    }
  }
  const uint64_t end = (q0 + ZC_SPAN < n) ? q0 + ZC_SPAN : n;
  for (uint64_t c = q0; c < end; c += 128) {
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = load16_clamped(data, n, c + 16 * k);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t xs[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint64_t p = c + 16 * k + 4 * d + j;
          if (p < end) {
            const uint32_t b = (xs[d] >> (8 * j)) & 0xFFu;
            gear_step(b, s);
            digest_step(b, s);
            if (((int32_t)s.glo >> 16) >= lo_thr && p >= ZC_ANCHOR_MIN_OFF) emit(p, s.glo);
          }
        }
    }
  }
  return ((uint64_t)s.hhi << 32) | s.hlo;
}

// exclusive prefix sum over the 64 lanes of a wave; *total = the sum
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t lane, uint32_t* total) {
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  *total = __shfl(x, 63, 64);
  return x - v;
}

// A whole wave-tile by one 256-thread block, a 1 KiB sub-span per thread:
// count, block prefix, write the anchors in position order at rel/g[base ...]
// (at most cap of them); optionally the block digests.  Returns the total.
__device__ uint32_t wave_tile_block(const uint8_t* __restrict__ data, uint64_t n, uint64_t wt, int32_t lo_thr,
                                    uint64_t* __restrict__ blk, uint32_t* __restrict__ rel,
                                    uint32_t* __restrict__ g, uint32_t base, uint32_t cap, uint32_t* s_tmp) {
  // blockDim.x == ZC_WT_BLOCK: the block covers the wave-tile
  const uint64_t t0 = wt << ZC_WT_SHIFT, q0 = t0 + (uint64_t)threadIdx.x * ZC_SPAN;
  uint32_t cnt = 0;
  if (q0 < n) {
    const uint64_t h = subspan_pass(data, n, q0, lo_thr, [&](uint64_t, uint32_t) { ++cnt; });
    if (blk) blk[q0 / ZC_SPAN] = h;
  }
  uint32_t tot;
  const uint32_t excl = block_excl_scan(cnt, s_tmp, tot);
  if (cnt && excl < cap && rel) {
    uint32_t k = excl;
    subspan_pass(data, n, q0, lo_thr, [&](uint64_t p, uint32_t gv) {
      if (k < cap) {
        rel[base + k] = (uint32_t)(p - t0);
        g[base + k] = gv;
      }
      ++k;
    });
  }
  return tot;
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

constexpr int kRounds = ZC_LSPAN / ZC_ROUND;  // rounds per tile
constexpr int kDmaRound = 64 * ZC_ROUND / 1024;  // DMA instructions per wave-round
constexpr int kDigests = ZC_LSPAN / ZC_SPAN;     // span digests per lane span
// Odd rows (lanes) take their lane span's two halves in the other order
// (round r reads half-span-rotated round r ^ kHalfRounds): the rows of a
// wave-round are then not all 4 KiB apart, a stride that costs the staging
// 12 % (tools/ubench/stage_bench2.hip: 5.5 -> 6.3 TB/s staged).  The gear is
// re-primed from the 32 bytes before each half, so a lane's anchors and gear
// values do not depend on the order.
constexpr int kHalfRounds = kRounds / 2;
// Timing probe for tools/ubench/scan_geom_ab.hip only (never set in the
// product): the DMA reads each wave-round as one contiguous 8 KiB block
// (rows 128 bytes apart) while the lanes hash as if it were their spans --
// wrong digests and anchors, the staging cost of a contiguous layout under
// the real per-byte work (DESIGN 4.1 experiment 22)
#ifndef ZC_CONTIG_PROBE_CFG
#define ZC_CONTIG_PROBE_CFG 0
#endif
constexpr bool kContigProbe = ZC_CONTIG_PROBE_CFG != 0;
constexpr uint32_t kHalfSpan = ZC_LSPAN / 2;
static_assert((kHalfRounds & (kHalfRounds - 1)) == 0 && kHalfRounds % (ZC_SPAN / ZC_ROUND) == 0, "half-span rotation");

// LDS image of a wave-round: row i (lane i's ZC_ROUND bytes) is stored
// linearly, with its 16-byte piece p at position p ^ swz(i); the swizzle makes
// the per-lane ds_read_b128 of a row bank-conflict free (rows within one
// 256-byte bank stripe get distinct piece positions).
constexpr int kPieces = ZC_ROUND / 16;
__host__ __device__ constexpr uint32_t row_swizzle(uint32_t row) { return (row / (256 / ZC_ROUND)) % kPieces; }

// DMA of round r of `tile` into ring slot `slot`: ZC_ROUND bytes of each of
// the wave's 64 rows (an odd row's from the other half of its span); one
// instruction fills 1024 / ZC_ROUND rows (1 KiB).
// Through a buffer descriptor at the wave-round's first byte (wave-uniform,
// built with scalar instructions): the lane's part of every instruction is
// its loop-invariant 32-bit offset lane_off[j], so a round costs no vector
// address arithmetic.  (wave must be wave-uniform: readfirstlane'd.)
template <int AUX>
__device__ __forceinline__ void stage_round(const uint8_t* __restrict__ data, uint8_t* ring, uint32_t wave,
                                            const uint32_t (&lane_off)[kDmaRound], uint64_t tile, int r,
                                            uint32_t slot) {
  uint8_t* dst = ring + slot * (64 * ZC_ROUND);
  const uint64_t at = kContigProbe
                          ? tile * ZC_STILE + (uint64_t)wave * 64 * ZC_LSPAN + (uint64_t)r * 64 * ZC_ROUND
                          : tile * ZC_STILE + (uint64_t)wave * 64 * ZC_LSPAN + (uint64_t)(r % kHalfRounds) * ZC_ROUND;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(data + at), (short)0, 64 * ZC_LSPAN, 0x00020000);
  const uint32_t flip = !kContigProbe && r >= kHalfRounds ? kHalfSpan : 0u;
#pragma unroll
  for (int j = 0; j < kDmaRound; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + j * 1024), 16, (int)(lane_off[j] ^ flip), 0, 0,
                                             AUX);
}

template <int N>
__device__ __forceinline__ void wait_lgkmcnt() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// Loads the hand-counted vmcnt waits order, written as inline asm so the
// compiler's own wait insertion does not track them: it cannot follow the
// counts across loop iterations and would put an s_waitcnt vmcnt(0) before
// every use (draining the prefetched rounds).  LDS reads of a ring slot the
// DMA fills are the same case (any DS read of the ring array may alias an
// outstanding LDS-DMA).  ties(v) pins the values after the wait that covers
// them.
typedef unsigned v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u32 lds_read16(const uint8_t* p) {
  v4u32 v;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ v4u32 global_read16(const uint8_t* p) {
  v4u32 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ uint4 to_uint4(v4u32 v) { return make_uint4(v[0], v[1], v[2], v[3]); }
template <int N>
__device__ __forceinline__ void ties(v4u32 (&v)[N]) {
  static_assert(N == 2 || N == 4 || N == 8, "ties");
  if constexpr (N == 2) {
    asm volatile("" : "+v"(v[0]), "+v"(v[1])::"memory");
  } else if constexpr (N == 4) {
    asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3])::"memory");
  } else {
    asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                 "+v"(v[7])::"memory");
  }
}

// s_waitcnt vmcnt(n) for a wave-uniform n (the tile end's store count is only
// known at run time); n < 8 or n > 63 waits for fewer, which is always safe
__device__ __forceinline__ void wait_vmcnt_dyn(uint32_t n) {
  switch (n) {
#define ZC_W(k) case k: wait_vmcnt<k>(); break;
    ZC_W(8) ZC_W(9) ZC_W(10) ZC_W(11) ZC_W(12) ZC_W(13) ZC_W(14) ZC_W(15) ZC_W(16) ZC_W(17) ZC_W(18)
    ZC_W(19) ZC_W(20) ZC_W(21) ZC_W(22) ZC_W(23) ZC_W(24) ZC_W(25) ZC_W(26) ZC_W(27) ZC_W(28) ZC_W(29)
    ZC_W(30) ZC_W(31) ZC_W(32) ZC_W(33) ZC_W(34) ZC_W(35) ZC_W(36) ZC_W(37) ZC_W(38) ZC_W(39) ZC_W(40)
    ZC_W(41) ZC_W(42) ZC_W(43) ZC_W(44) ZC_W(45) ZC_W(46) ZC_W(47) ZC_W(48) ZC_W(49) ZC_W(50) ZC_W(51)
    ZC_W(52) ZC_W(53) ZC_W(54) ZC_W(55) ZC_W(56) ZC_W(57) ZC_W(58) ZC_W(59) ZC_W(60) ZC_W(61) ZC_W(62)
#undef ZC_W
    default:
      if (n > 62) wait_vmcnt<63>();
      else wait_vmcnt<0>();
  }
}

// directory count of a wave-tile left for the exact rescan
constexpr uint32_t ZC_WT_OVERFLOW = 0xFFFFFFFFu;
// no list entry (end of a lane's chain)
constexpr uint32_t kNoEntry = 0xFFu;
static_assert(ZC_WLIST < kNoEntry, "entry indices fit 8 bits");

// The anchors of list entry i (a 16-byte piece of the lane span at span0):
// hit mask of its 16 positions (offsets below 63 of the stream excluded) and
// the gear value of each position, rolled on from the gear before the piece.
struct PieceHits {
  uint32_t mask, rel;  // rel: offset of the piece in the lane span
  uint32_t g0;         // gear before the piece
  uint32_t xs[4];
};

__device__ __forceinline__ PieceHits piece_hits(const WaveList& wl, uint32_t i, uint64_t span0, int32_t lo_thr) {
  PieceHits h;
  const uint32_t e0 = wl.e[3 * i];
  h.rel = ((e0 >> 8) & 0xFFu) << 4;
  h.g0 = wl.e[3 * i + 1];
  const uint4 v = wl.x[i];
  h.xs[0] = v.x;
  h.xs[1] = v.y;
  h.xs[2] = v.z;
  h.xs[3] = v.w;
  const uint32_t two = 0x00020002u;
  uint32_t S = h.g0, mask = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t S1 = pk_step(S, bytes01(h.xs[d]), two), S2 = pk_step(S1, bytes23(h.xs[d]), two);
    // st(q) of the dword's four positions: the halves of S1, then of S2
    mask |= ((int32_t)(int16_t)S1 >= lo_thr ? 1u : 0u) << (4 * d);
    mask |= (((int32_t)S1 >> 16) >= lo_thr ? 1u : 0u) << (4 * d + 1);
    mask |= ((int32_t)(int16_t)S2 >= lo_thr ? 1u : 0u) << (4 * d + 2);
    mask |= (((int32_t)S2 >> 16) >= lo_thr ? 1u : 0u) << (4 * d + 3);
    S = S2;
  }
  if (span0 + h.rel < ZC_ANCHOR_MIN_OFF)  // the stream's first 63 positions are no anchors
    mask &= ~0u << min(ZC_ANCHOR_MIN_OFF - (uint32_t)(span0 + h.rel), 16u);
  h.mask = mask;
  return h;
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
// (gko.key: also the grid-chunk keys of the wave-tile: each lane folds its
// span digests, weights them by 257^(4 KiB x the lanes after it in its chunk)
// -- lane_w -- and the chunk's lanes add up; the chunk's first lane stores the
// key, always lane 0 among them, so both store instructions always issue and
// are counted)
__device__ __forceinline__ uint32_t scan_tile_end(uint64_t span0, uint32_t lane, int32_t lo_thr,
                                                  const uint64_t (&bk)[kDigests], const WaveList& wl,
                                                  uint32_t last, uint64_t* __restrict__ blk, PoolOut po,
                                                  uint32_t& acc_pool, uint32_t& acc_over, const GridKeysOut& gko,
                                                  uint64_t span_m, uint64_t lane_w) {
  uint4* bo = (uint4*)(blk + span0 / ZC_SPAN);
#pragma unroll
  for (int t = 0; t < kDigests / 2; ++t)
    bo[t] = make_uint4((uint32_t)bk[2 * t], (uint32_t)(bk[2 * t] >> 32), (uint32_t)bk[2 * t + 1],
                       (uint32_t)(bk[2 * t + 1] >> 32));
  uint32_t nkey = 0;
  if (gko.key) {
    uint64_t acc = 0;
#pragma unroll
    for (int t = 0; t < kDigests; ++t) acc = acc * span_m + bk[t];
    acc *= lane_w;
    for (uint32_t d = 1; d < (1u << gko.lshift); d <<= 1) acc += __shfl_xor(acc, (int)d, 64);
    if ((lane & ((1u << gko.lshift) - 1)) == 0) {
      const uint64_t i = (span0 / ZC_LSPAN) >> gko.lshift;  // grid chunk i (the first epoch: r_e = 0)
      gko.key[i] = gko.pw + acc;
      gko.hkey[i] = gko.pw + acc;
    }
    nkey = 2;
  }
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
          // the anchor state before each dword of the piece
          gd[0] = wl.e[3 * i + 1];
#pragma unroll
          for (int d = 0; d < 3; ++d)
            gd[d + 1] = pk_step(pk_step(gd[d], bytes01(xs[d]), 0x00020002u), bytes23(xs[d]), 0x00020002u);
          i += 64;
        }
        if (__ballot(mask != 0) == 0) break;
        if (mask) {
          const uint32_t t = __builtin_ctz(mask), d = t >> 2, q = t & 3u;
          const uint32_t gdd = d == 0 ? gd[0] : d == 1 ? gd[1] : d == 2 ? gd[2] : gd[3];
          const uint32_t xd = d == 0 ? xs[0] : d == 1 ? xs[1] : d == 2 ? xs[2] : xs[3];
          // the key at position t: {st(t - 1), st(t)} from the dword's state
          const uint32_t S1 = pk_step(gdd, bytes01(xd), 0x00020002u), S2 = pk_step(S1, bytes23(xd), 0x00020002u);
          const uint32_t g = dword_key(gdd, S1, S2, q);
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
  return kDigests / 2 + __builtin_amdgcn_readfirstlane(nst) + 2 + nkey;
}

// Every wave walks whole wave-tiles (256 KiB, 64 lane spans) on its own:
// wave-tiles wt0 + g, wt0 + g + G, ... for global wave g of G.  Its rounds form
// one flat sequence over them (32 per wave-tile).  The ring has ONE slot per
// wave: a round is read from the slot into registers, the slot is refilled
// with the next round, then the round is hashed -- one round (8 KiB) in flight
// per wave while it computes; 12 KiB of LDS per wave (slot + anchor list).
// Two 4-wave workgroups per CU (two waves per SIMD): with the 32-bit gear
// (16.5 VALU per dword) a third wave per SIMD paid (1.525 vs 1.564 ms per
// 8 GiB, DESIGN 4.1 experiment 18); with the packed anchor state (12 per
// dword) two are 1.5 % faster than three (tools/ubench/scan_geom_ab.hip, three
// interleaved runs, outputs identical; experiment 21).  The 32 bytes before
// each half of a lane span (they prime the anchor state) are two per-lane
// register loads issued with the DMA of the half's first round, so half and
// wave-tile boundaries cost no extra pipeline round.
constexpr int kScanWaves = ZC_SCAN_WAVES;  // per workgroup (one per SIMD)
#ifndef ZC_SCAN_WG_PER_CU_CFG
#define ZC_SCAN_WG_PER_CU_CFG 2
#endif
constexpr int kScanWgPerCu = ZC_SCAN_WG_PER_CU_CFG;  // workgroups resident per CU
// ring slots per wave: rounds in flight while a wave hashes one
#ifndef ZC_SCAN_SLOTS_CFG
#define ZC_SCAN_SLOTS_CFG 1
#endif
constexpr int kScanSlots = ZC_SCAN_SLOTS_CFG;
// Wave priority around the hand-off (A/B switch, tools/ubench/scan_geom_ab):
// a wave waits for its round, reads the slot out and issues the refill at
// priority kScanPrioHandoff, and hashes at 0, so a wave whose round has landed
// gets the SIMD's issue slots ahead of the other wave's hashing and the ring
// is refilled at once (0: no priority changes)
#ifndef ZC_SCAN_PRIO_CFG
#define ZC_SCAN_PRIO_CFG 0
#endif
constexpr int kScanPrioHandoff = ZC_SCAN_PRIO_CFG;
static_assert(kScanSlots == 1 || kScanSlots == 2, "one or two ring slots");
struct ScanLds {
  uint8_t ring[kScanWaves][kScanSlots * 64 * ZC_ROUND];
  uint4 wdata[kScanWaves][ZC_WLIST];
  uint32_t wlist[kScanWaves][ZC_WLIST * 3];
};
static_assert(kScanWgPerCu * sizeof(ScanLds) <= 160 * 1024, "the scan workgroups of a CU fit its LDS");
__device__ __forceinline__ void scan_body(
    const uint8_t* __restrict__ data, uint64_t n, uint64_t wt0, uint64_t nwt, int32_t lo_thr,
    uint64_t* __restrict__ blk, PoolOut po, unsigned long long* __restrict__ counters, ScanLds& L,
    GridKeysOut gko = GridKeysOut{nullptr, nullptr, 0, 0}) {
  constexpr uint32_t kRpt = kRounds;  // rounds per wave-tile
  constexpr uint32_t kWpt = ZC_SCAN_TPB / 64;  // wave-tiles per 2 MiB tile
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t gw = blockIdx.x * kScanWaves + wave, nw = gridDim.x * kScanWaves;
  uint8_t* myring = L.ring[wave];
  WaveList wl{L.wlist[wave], L.wdata[wave], 0};
  const uint32_t ntk = nwt > gw ? (uint32_t)((nwt - 1 - gw) / nw + 1) : 0;
  const uint32_t nR = ntk * kRpt;
  // this lane's share of DMA instruction j: row j * (1024 / ZC_ROUND) + lane /
  // kPieces of the wave, the source piece that lands at position lane % kPieces
  uint32_t lane_off[kDmaRound];
#pragma unroll
  for (int j = 0; j < kDmaRound; ++j) {
    const uint32_t row = j * (1024 / ZC_ROUND) + lane / kPieces;
    lane_off[j] = kContigProbe ? row * ZC_ROUND + ((lane % kPieces) ^ row_swizzle(row)) * 16
                               : row * ZC_LSPAN + (row & 1) * kHalfSpan + ((lane % kPieces) ^ row_swizzle(row)) * 16;
  }
  const uint32_t sw = row_swizzle(lane);  // read-side swizzle of this lane's row
  const uint32_t two = pk_two();          // the packed state's multiplier, in an SGPR
  const uint32_t hs = (lane & 1) * kHalfRounds;  // logical round r is physical round r ^ hs
  v4u32 warm[2] = {};                       // the 32 bytes before the next half span
  // vector-memory instructions of round Rx's group (its DMA, and for a half's
  // first round the two warm-up loads)
  auto group = [&](uint32_t Rx) -> uint32_t { return kDmaRound + ((Rx % kRpt) % kHalfRounds == 0 ? 2u : 0u); };
  auto issue = [&](uint32_t Rx) {
    const uint32_t k = Rx / kRpt, r = Rx - k * kRpt;
    const uint64_t wt = wt0 + gw + (uint64_t)k * nw;
    stage_round<kScanDmaAux>(data, myring, (uint32_t)(wt % kWpt), lane_off, wt / kWpt, (int)r, Rx % kScanSlots);
    if (r % kHalfRounds == 0) {
      // span 0 of the stream has no bytes before it: it reads itself (unused)
      const uint64_t at = (wt << ZC_WT_SHIFT) + (uint64_t)lane * ZC_LSPAN + (uint64_t)(r ^ hs) * ZC_ROUND;
      const uint8_t* src = at >= 32 ? data + at - 32 : data + at;
      warm[0] = global_read16(src);
      warm[1] = global_read16(src + 16);
    }
  };
  // after[i]: vector-memory instructions issued after the group of round
  // R + i (in flight: rounds R .. R + kScanSlots - 1); the wait for round R is
  // vmcnt(after[0]) -- the counter retires in issue order
  uint32_t after[kScanSlots];
#pragma unroll
  for (int i = 0; i < kScanSlots; ++i) {
    after[i] = 0;
    if ((uint32_t)i < nR) {
#pragma unroll
      for (int j = 0; j < i; ++j) after[j] += group(i);
      issue(i);
    }
  }
  ScanLane s{0, 0, 0};
  uint64_t bk[kDigests];
#pragma unroll
  for (int t = 0; t < kDigests; ++t) bk[t] = 0;
  uint64_t span0 = 0;
  uint32_t last = kNoEntry;  // this lane's newest entry in the wave's list
  uint32_t acc_pool = 0, acc_over = 0;  // wave-uniform: anchors stored, wave-tiles overflowed
  // the grid keys' multipliers: 257^1 KiB, and this lane's weight in its chunk
  const uint64_t span_m = span_mul();
  const uint64_t lane_w =
      gko.key ? pow257_dev((uint64_t)ZC_LSPAN * (((1u << gko.lshift) - 1) - (lane & ((1u << gko.lshift) - 1)))) : 0;

#pragma unroll 1
  for (uint32_t R = 0; R < nR; ++R) {
    const uint32_t k = R / kRpt;
    const int r = (int)(R - k * kRpt);
    if constexpr (kScanPrioHandoff > 0) __builtin_amdgcn_s_setprio(kScanPrioHandoff);
    // round R (and, for a half's first round, its warm-up loads) has landed
    // once only what was issued after it is outstanding: the later rounds in
    // flight and the last tile end's stores
    if (kScanSlots == 1 && r != 0) wait_vmcnt<0>();
    else wait_vmcnt_dyn(after[0]);
    const uint32_t pr = (uint32_t)r ^ hs;  // the physical round in the lane span
    if (r == 0) {
      // a new wave-tile
      span0 = ((wt0 + gw + (uint64_t)k * nw) << ZC_WT_SHIFT) + (uint64_t)lane * ZC_LSPAN;
      s = ScanLane{0, 0, 0};
      wl.n = 0;
      last = kNoEntry;
    }
    if (r % kHalfRounds == 0) {
      // a new half: the warm-up bytes prime the anchor state (it depends on
      // the 32 bytes before only, so this equals the state rolled on
      // continuously)
      s.glo = 0;
      ties(warm);  // landed: the wait above covers them
      if (span0 + pr * ZC_ROUND >= 64) {
        const uint32_t xs[8] = {warm[0][0], warm[0][1], warm[0][2], warm[0][3],
                                warm[1][0], warm[1][1], warm[1][2], warm[1][3]};
#pragma unroll
        for (int j = 0; j < 8; ++j) s.glo = pk_step(pk_step(s.glo, bytes01(xs[j]), two), bytes23(xs[j]), two);
      }
    }
    // the round's pieces, in groups of four (one ties() each)
    static_assert(kPieces % 4 == 0 && kPieces <= 16, "the round is read as 4, 8 or 16 pieces");
    constexpr int kGroups = kPieces / 4;
    v4u32 vg[kGroups][4];
#pragma unroll
    for (int g = 0; g < kGroups; ++g)
#pragma unroll
      for (int p = 0; p < 4; ++p)
        vg[g][p] = lds_read16(myring + (R % kScanSlots) * (64 * ZC_ROUND) + lane * ZC_ROUND + (((4 * g + p) ^ sw) << 4));
    wait_lgkmcnt<0>();  // the slot is read out: refill it with round R + kScanSlots
#pragma unroll
    for (int g = 0; g < kGroups; ++g) ties(vg[g]);
#pragma unroll
    for (int i = 0; i + 1 < kScanSlots; ++i) after[i] = after[i + 1];
    after[kScanSlots - 1] = 0;
    if (R + kScanSlots < nR) {
#pragma unroll
      for (int i = 0; i + 1 < kScanSlots; ++i) after[i] += group(R + kScanSlots);
      issue(R + kScanSlots);
    }
    if constexpr (kScanPrioHandoff > 0) __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int g = 0; g < kGroups; ++g)
#pragma unroll
      for (int p = 0; p < 4; ++p)
        scan_piece(to_uint4(vg[g][p]), pr * ZC_ROUND + (4 * g + p) * 16, lo_thr, two, s, wl, last);
    if ((r + 1) % (ZC_SPAN / ZC_ROUND) == 0) {
      const uint64_t h = ((uint64_t)s.hhi << 32) | s.hlo;
      const uint32_t q = pr / (ZC_SPAN / ZC_ROUND);  // per lane: the halves are rotated
#pragma unroll
      for (int t = 0; t < kDigests; ++t) bk[t] = q == (uint32_t)t ? h : bk[t];
      s.hlo = s.hhi = 0;
    }
    if (r == kRounds - 1) {
      const uint32_t ns =
          scan_tile_end(span0, lane, lo_thr, bk, wl, last, blk, po, acc_pool, acc_over, gko, span_m, lane_w);
#pragma unroll
      for (int i = 0; i < kScanSlots; ++i) after[i] += ns;
    }
  }
  if (lane == 0) {
    if (acc_pool) atomicAdd(&counters[CNT_POOL], (unsigned long long)acc_pool);
    if (acc_over) atomicAdd(&counters[CNT_OVERFLOW], (unsigned long long)acc_over);
  }
}

// (__launch_bounds__' second argument: at least kScanWgPerCu waves per SIMD)
__global__ void __launch_bounds__(64 * kScanWaves, kScanWgPerCu) zc_scan_kernel(
    const uint8_t* __restrict__ data, uint64_t n, uint64_t wt0, uint64_t nwt, int32_t lo_thr,
    uint64_t* __restrict__ blk, PoolOut po, unsigned long long* __restrict__ counters, GridKeysOut gko) {
  __shared__ ScanLds lds;
  scan_body(data, n, wt0, nwt, lo_thr, blk, po, counters, lds, gko);
}
// the stream's last, partial tile: one 256-thread block per wave-tile, a
// 1 KiB sub-span per thread (block digests and anchors)
__global__ void __launch_bounds__(ZC_WT_BLOCK) zc_scan_tail_kernel(const uint8_t* __restrict__ data, uint64_t n,
                                                             uint64_t tile, int32_t lo_thr,
                                                             uint64_t* __restrict__ blk, PoolOut po,
                                                             unsigned long long* __restrict__ counters) {
  __shared__ uint32_t s_tmp[ZC_WT_BLOCK / 64];
  const uint64_t wt = tile * (ZC_SCAN_TPB / 64) + blockIdx.x;
  const uint32_t base = (uint32_t)(wt - po.wt0) * po.wcap;
  const uint32_t tot = wave_tile_block(data, n, wt, lo_thr, blk, po.rel, po.g, base, po.wcap, s_tmp);
  if (threadIdx.x == 0) {
    po.base[wt] = base;
    if (tot > po.wcap) {
      po.cnt[wt] = ZC_WT_OVERFLOW;
      atomicAdd(&counters[CNT_OVERFLOW], 1ull);
    } else {
      po.cnt[wt] = tot;
      if (tot) atomicAdd(&counters[CNT_POOL], (unsigned long long)tot);
    }
  }
}

// Exact rescan of the wave-tiles marked overflowed, one block each: pass 0
// counts (cnt[wt] = exact count), pass 1 writes the anchors into the side
// pool at sbase[i] and points the directory there.
__global__ void __launch_bounds__(ZC_WT_BLOCK) zc_anchor_rescan_kernel(const uint8_t* __restrict__ data, uint64_t n,
                                                                 int32_t lo_thr, const uint32_t* __restrict__ tiles,
                                                                 const uint32_t* __restrict__ sbase, int pass,
                                                                 uint32_t* __restrict__ dbase,
                                                                 uint32_t* __restrict__ dcnt,
                                                                 uint32_t* __restrict__ srel, uint32_t* __restrict__ sg) {
  __shared__ uint32_t s_tmp[ZC_WT_BLOCK / 64];
  const uint64_t wt = tiles[blockIdx.x];
  const uint32_t b = pass ? sbase[blockIdx.x] : 0u;
  const uint32_t tot = wave_tile_block(data, n, wt, lo_thr, nullptr, pass ? srel : nullptr, sg, b, ~0u, s_tmp);
  if (threadIdx.x == 0) {
    dcnt[wt] = tot;
    if (pass) dbase[wt] = b | ZC_SIDE_POOL;
  }
}

// After the feed window slid down by `shift` pool entries: the directory
// entries [0, cnt) that point into the main pool follow their shares
__global__ void zc_slide_dir_kernel(uint32_t* __restrict__ base, const uint32_t* __restrict__ dcnt, uint32_t cnt,
                                    uint32_t shift) {
  ZC_URGENT();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cnt && dcnt[i] != ZC_WT_OVERFLOW && !(base[i] & ZC_SIDE_POOL)) base[i] -= shift;
}

// the anchors of wave-tile wt: entry k at rel[k], g[k], sorted by position
struct TileAnchors {
  const uint32_t* rel;
  const uint32_t* g;
  uint32_t cnt;
};

__device__ __forceinline__ TileAnchors tile_anchors(const AnchorView& av, uint64_t wt) {
  // a wave-tile still marked overflowed (before its exact rescan) reads empty
  const uint32_t b = av.base[wt], c0 = av.cnt[wt], c = c0 == ZC_WT_OVERFLOW ? 0u : c0;
  if (b & ZC_SIDE_POOL) return TileAnchors{av.srel + (b & ~ZC_SIDE_POOL), av.sg + (b & ~ZC_SIDE_POOL), c};
  return TileAnchors{av.rel + b, av.g + b, c};
}

// ---------------------------------------------------------------------------
// the epoch's tables and counters, cleared by the chunk-metadata launch
// The grid chunks' SHA-1 (zc_sha1_grid_kernel: 20 bytes per chunk [q W, (q + 1) W)
// of the stream, q < n_sha), when the side stream computes them (ZC_FLAG_SHA1)
struct ShaGrid {
  const uint8_t* sha;  // null: none
  uint64_t n_sha;
  uint64_t n;
  uint32_t W;
  __device__ __forceinline__ bool has(uint64_t c) const {
    return sha && c % W == 0 && c / W < n_sha && c + W <= n;
  }
  __device__ __forceinline__ uint4 prefix(uint64_t c) const {
    const uint32_t* p = (const uint32_t*)(sha + c / W * 20);  // 4-byte aligned
    return make_uint4(p[0], p[1], p[2], p[3]);
  }
};

struct EpochClear {
  uint64_t* ckeys;  // class table {key high word | lowest ref}: empty
  uint32_t cwords;
  uint64_t* tab;  // anchor table: empty (null: none)
  uint64_t twords;
  uint32_t* gfilt;  // key filter: zero
  uint32_t gwords;
  unsigned long long* counters;
  // the scan's two counters (anchors pooled, wave-tiles overflowed): copied to
  // the host's pinned h_scnt and cleared for the next scan (null: not this batch)
  unsigned long long* scnt;
  unsigned long long* h_scnt;
};

// The first anchor of chunk [c, c + W) at offset >= ZC_ANCHOR_MIN_OFF: its
// offset (ZC_NO_ANCHOR: none), gear value and fingerprint
__device__ __forceinline__ void first_anchor(const uint8_t* __restrict__ data, const AnchorView& av, uint64_t c,
                                             uint32_t W, uint32_t& off, uint32_t& gv, uint64_t& f) {
  off = ZC_NO_ANCHOR;
  gv = 0;
  f = 0;
  if (W > ZC_ANCHOR_MIN_OFF) {
    const uint64_t lo = c + ZC_ANCHOR_MIN_OFF, hi = c + W - 1;  // inclusive
    for (uint64_t wt = lo >> ZC_WT_SHIFT; wt <= (hi >> ZC_WT_SHIFT); ++wt) {
      const TileAnchors ta = tile_anchors(av, wt);
      const uint64_t t0 = wt << ZC_WT_SHIFT;
      const uint32_t lo_rel = lo > t0 ? (uint32_t)(lo - t0) : 0u;
      // first entry with rel >= lo_rel: it lies in [L, R] (R = cnt: none);
      // a 4-way search loads three pivots per step (a quarter of the
      // dependent loads of a binary search), then the last <= 3 at once
      uint32_t L = 0, R = ta.cnt;
      while (R - L > 3) {
        const uint32_t q = (R - L) >> 2, a = L + q, b = L + 2 * q, c = L + 3 * q;
        const uint32_t ra = ta.rel[a], rb = ta.rel[b], rc = ta.rel[c];
        if (rc < lo_rel) {
          L = c + 1;
        } else if (rb < lo_rel) {
          L = b + 1;
          R = c;
        } else if (ra < lo_rel) {
          L = a + 1;
          R = b;
        } else {
          R = a;
        }
      }
      {
        const bool b0 = L < R && ta.rel[L] < lo_rel, b1 = L + 1 < R && ta.rel[L + 1] < lo_rel,
                   b2 = L + 2 < R && ta.rel[L + 2] < lo_rel;
        L += (uint32_t)b0 + (uint32_t)b1 + (uint32_t)b2;  // sorted: a prefix is below
      }
      if (L < ta.cnt) {
        const uint64_t pos = t0 + ta.rel[L];
        if (pos <= hi) {
          off = (uint32_t)(pos - c);
          gv = ta.g[L];
          f = anchor_fp(data, pos);
        }
        break;  // later wave-tiles only hold later anchors
      }
    }
  }
}

// The epoch's table inserts (zc_index_insert_kernel), also done inside the
// metadata kernel when the tables start out empty (FusedInsert, below)
struct FusedInsert {
  uint64_t* ckeys;  // null: not fused
  uint32_t cbits;
  uint64_t* tab;  // null: no anchor table this epoch
  uint32_t tbits;
  uint32_t* gfilt;
};
__device__ __forceinline__ void class_insert(const uint64_t* __restrict__ key, uint32_t i, uint64_t* ckeys,
                                             uint32_t cbits);
__device__ __forceinline__ void anchor_insert(uint32_t i, uint32_t g, uint64_t fp, uint64_t* tab, uint32_t tbits,
                                              uint32_t* __restrict__ gfilt);

// zc_chunk_meta: per grid chunk i of the epoch, start = r_e + i * W: start,
// visibility time, key, first anchor (offset, gear value, 8-byte
// fingerprint); the chunk is not yet consumed by a match (dead = 0).  Two
// threads per chunk, in different waves: thread i folds the key (W / 1 KiB
// span digests), thread split + i searches the first anchor (a chain of
// dependent loads), so the two latency chains overlap instead of adding up
// (split: a multiple of the block size).  The whole grid also clears the
// epoch's tables (no separate fills) -- or, fused (fi.ckeys; the tables are
// empty already and every key was written before the kernel), inserts each
// chunk into them: the key thread into the class table, the anchor thread
// into the anchor table, in place of zc_index_insert_kernel.
__global__ void zc_chunk_meta_kernel(const uint8_t* __restrict__ data, uint64_t n,
                                     const uint64_t* __restrict__ blk, AnchorView av, uint64_t r_e,
                                     uint32_t nchunks, uint32_t split, uint32_t W, uint64_t pw,
                                     uint64_t* __restrict__ start, uint64_t* __restrict__ vis,
                                     uint8_t* __restrict__ dead, uint64_t* __restrict__ key,
                                     uint32_t* __restrict__ cg, uint64_t* __restrict__ cfp,
                                     uint32_t* __restrict__ anc_off, uint64_t* __restrict__ hkey, uint32_t key_from,
                                     EpochClear ec, FusedInsert fi) {
  ZC_URGENT();
  const uint64_t gt = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = gt; j < ec.cwords; j += gs) ec.ckeys[j] = ~0ull;
  if (ec.tab)
    for (uint64_t j = gt; j < ec.twords; j += gs) ec.tab[j] = ~0ull;
  for (uint64_t j = gt; j < ec.gwords; j += gs) ec.gfilt[j] = 0u;
  if (gt < CNT_LAST) ec.counters[gt] = 0ull;
  if (ec.scnt && gt < 2) {
    ec.h_scnt[gt] = ec.scnt[gt];
    ec.scnt[gt] = 0ull;
  }
  if (gt < nchunks) {
    const uint32_t i = (uint32_t)gt;
    const uint64_t c = r_e + (uint64_t)i * W;
    start[i] = c;
    vis[i] = c + 2ull * W - 1;  // cut in the iteration whose probe is at c + 2W - 1
    dead[i] = 0;
    if (i >= key_from) {  // (below: the scan wrote the key and the host's copy)
      const uint64_t k = pw + rk_acc(data, blk, c, c + W);
      key[i] = k;
      // the host's copy (pinned memory, written across PCIe while the kernel
      // runs): no separate copy kernel beside the index build
      if (hkey) hkey[i] = k;
    }
    if (fi.ckeys) class_insert(key, i, fi.ckeys, fi.cbits);  // (fused: key_from == nchunks)
  } else if (gt >= split && gt - split < nchunks) {
    const uint32_t i = (uint32_t)(gt - split);
    uint32_t off, gv;
    uint64_t f;
    first_anchor(data, av, r_e + (uint64_t)i * W, W, off, gv, f);
    anc_off[i] = off;
    cg[i] = gv;
    cfp[i] = f;
    if (fi.ckeys && fi.tab && off != ZC_NO_ANCHOR) anchor_insert(i, gv, f, fi.tab, fi.tbits, fi.gfilt);
  }
}

// zc_ref_meta: per chunk [start[i], start[i] + W) anywhere in the resident
// stream: key, first anchor {offset, gear, fingerprint} (the chunks that
// join the historic index); the key by thread i, the anchor by thread
// split + i, as in zc_chunk_meta
__global__ void zc_ref_meta_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ blk, AnchorView av,
                                   const uint64_t* __restrict__ starts, uint32_t cnt, uint32_t split, uint32_t W,
                                   uint64_t pw, uint64_t* __restrict__ key, uint32_t* __restrict__ anc_off,
                                   uint32_t* __restrict__ cg, uint64_t* __restrict__ cfp) {
  ZC_URGENT();
  const uint64_t gt = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gt < cnt) {
    const uint64_t c = starts[gt];
    key[gt] = pw + rk_acc(data, blk, c, c + W);
  } else if (gt >= split && gt - split < cnt) {
    const uint32_t i = (uint32_t)(gt - split);
    uint32_t off, gv;
    uint64_t f;
    first_anchor(data, av, starts[i], W, off, gv, f);
    anc_off[i] = off;
    cg[i] = gv;
    cfp[i] = f;
  }
}

// zc_ref_gather: historic entry dst[t] (t < cnt) takes ref src[t] of the
// epoch's arrays (its key, first anchor offset, gear and fingerprint) -- the
// stream's saved chunks, whose metadata the epoch computed already
__global__ void zc_ref_gather_kernel(const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst, uint32_t cnt,
                                     const uint64_t* __restrict__ ckey, const uint32_t* __restrict__ canc,
                                     const uint32_t* __restrict__ cgv, const uint64_t* __restrict__ cfpv,
                                     uint64_t* __restrict__ key, uint32_t* __restrict__ anc, uint32_t* __restrict__ g,
                                     uint64_t* __restrict__ fp) {
  ZC_URGENT();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cnt) return;
  const uint32_t r = src[t], e = dst[t];
  key[e] = ckey[r];
  anc[e] = canc[r];
  g[e] = cgv[r];
  fp[e] = cfpv[r];
}

// a ref without an anchor is found by its key (the exact screen)
__device__ __forceinline__ bool anc_missing(const uint32_t* __restrict__ anc_off, uint32_t ref) {
  return anc_off[ref] == ZC_NO_ANCHOR;
}

// ---------------------------------------------------------------------------
// anchor table: open addressing on the anchor's gear value, duplicates kept.
// A slot is 16 bytes, {gear | ref << 32, fingerprint}: one load gives the
// key, the ref and the fingerprint to compare (empty: all ones).
constexpr uint64_t kEmpty = ~0ull;

// The slot mixes the gear with the fingerprint: the gear alone has ~20 free
// bits on random bytes but as few as 4 on content whose bytes of one parity
// are constant (UTF-16 text: every odd byte 0, so st(q - 1) = 0 at every
// anchor, and st(q) keeps only the 4 bits the anchor test leaves free), and
// every chunk's anchor would then share 16 probe chains (quadratic inserts and
// walks).  The 8 fingerprint bytes spread such keys like any others.
__device__ __forceinline__ uint32_t table_slot(uint32_t g, uint64_t fp, uint32_t tbits) {
  return (uint32_t)(((((uint64_t)g << 32) ^ fp) * kGolden) >> (64 - tbits));
}

// the probe's first level: bit (g mod 2^kGFiltBits) of every table key (the
// low bits: an anchor's gear always has its top bits set)
constexpr int kGFiltBits = 20;                               // 2^20 bits = 128 KiB
constexpr uint32_t kGFiltWords = 1u << (kGFiltBits - 5);

// ---------------------------------------------------------------------------
// zc_probe: every anchor of the stream probes the table (key = gear value,
// confirmed by the 8-byte fingerprint).  A wave takes kProbeWT consecutive
// wave-tiles and a lane their slots lane, lane + 64, ... (kProbeSlots per
// wave-tile; slots past that -- dense small-W streams, side-pool wave-tiles --
// in a second loop; the geometry is chosen at the launch).
// The loads are issued level by level -- every slot's gear value, then every
// filter word -- so a lane has all of them in flight at once; an anchor
// tests the table's 2^20-bit key filter (L2 resident, ~1 in 8 pass at
// W = 64 KiB) and only then walks the table.  The passing anchors of the
// wave are compacted into LDS and walked one per lane, so the table walks
// (a few dependent loads each) run side by side instead of one slot after
// another.
constexpr int kProbeTPB = 256;

// the epoch's grid: chunk j starts at r_e + j W (ref nconf + j), j < nspec
struct EpochGrid {
  uint64_t r_e;
  uint32_t nconf, nspec;
};

// The probe's candidates are staged per wave in LDS and appended to the
// global list with one atomic per wave (an incremental backup of unchanged
// data emits a candidate per 64 KiB, 16 per wave: 131,072 same-address
// atomics made the probe 190 us per 8 GiB); a full stage spills to the
// global counter.
constexpr uint32_t kCandStage = 64;
// The probe's per-wave list of anchors that pass the filters: 128 entries
// (random data at W = 64 KiB: ~32 per wave).  The probe's LDS is 12 KiB per
// 4-wave workgroup, so its occupancy is bound by registers, not LDS. With
// 512 entries it was 41 KiB per workgroup, three workgroups per CU, and the
// 2048 workgroups of an 8 GiB stream ran in three rounds.
constexpr uint32_t kPassCap = 128;
struct CandOut {
  Cand* cand;
  uint64_t cap;
  unsigned long long* counters;
  Cand* stage;      // this wave's LDS stage
  uint32_t* nstage; // its fill count (LDS)
};
__device__ __forceinline__ void emit_cand(const CandOut& co, uint64_t p, uint32_t ref, uint32_t pad) {
  const uint32_t k = atomicAdd(co.nstage, 1u);
  if (k < kCandStage) {
    co.stage[k].p = p;
    co.stage[k].ref = ref;
    co.stage[k].pad = pad;
    return;
  }
  const unsigned long long c = atomicAdd(&co.counters[CNT_CAND], 1ull);
  if (c < co.cap) {
    co.cand[c].p = p;
    co.cand[c].ref = ref;
    co.cand[c].pad = pad;
  }
}

__device__ __forceinline__ void probe_anchor(uint64_t pos, uint32_t gk, uint64_t fp,
                                             const uint64_t* __restrict__ tab, uint32_t tbits,
                                             const uint32_t* __restrict__ anc_off, const uint32_t* __restrict__ cls,
                                             const uint64_t* __restrict__ vis, const uint8_t* __restrict__ dead,
                                             uint64_t r, uint64_t n, uint32_t W, const EpochGrid& eg,
                                             const CandOut& co) {
  if (pos < r + ZC_ANCHOR_MIN_OFF || !tab) return;
  const uint32_t mask = (1u << tbits) - 1;
  uint32_t h = table_slot(gk, fp, tbits);
  for (;;) {
    const uint4 slot = *(const uint4*)(tab + 2 * (uint64_t)h);
    if (slot.x == 0xFFFFFFFFu && slot.y == 0xFFFFFFFFu) break;  // empty
    if (slot.x == gk) {
      const uint32_t ref = slot.y;
      // everything indexed by ref in one round of loads (one dependent level
      // after the slot instead of two)
      const uint32_t cr = cls[ref], o32 = anc_off[ref];
      const uint64_t vr = vis[ref];
      const uint8_t dr = dead[ref];
      if (fp == (((uint64_t)slot.w << 32) | slot.z) && cr == ref) {
        const uint64_t o = o32;
        if (pos >= r + o) {
          const uint64_t ws = pos - o, p = ws + W - 1;
          // a window that is a grid chunk of this epoch in ref's class is the
          // walk's (grid shortcut): no candidate.  The common case is the grid
          // chunk's own first anchor (ref = nconf + j, whose class is ref):
          // known without reading cls[nconf + j]
          bool grid_twin = false;
          if (ws >= eg.r_e && (ws - eg.r_e) % W == 0) {
            const uint64_t j = (ws - eg.r_e) / W;
            grid_twin = j < eg.nspec && (eg.nconf + j == ref || cls[eg.nconf + j] == ref);
          }
          if (p < n && p >= vr && !dr && !grid_twin) emit_cand(co, p, ref, 0u);
        }
      }
    }
    h = (h + 1) & mask;
  }
}

// The historic index (chunks whose bytes have left HBM: earlier streams of
// the context, or evicted from a bounded feed window) is a second table of the
// same layout.  Its entries are always visible and never consumed; a
// candidate names the entry (pad = 1) and is confirmed by the window's key and
// SHA-1 (chunk_index.cc:119-143), not by bytes.
__device__ __forceinline__ void probe_hist(uint64_t pos, uint32_t gk, uint64_t fp, const HistTab& ht, uint64_t r,
                                           uint64_t n, uint32_t W, const CandOut& co) {
  if (pos < r + ZC_ANCHOR_MIN_OFF) return;
  const uint32_t mask = (1u << ht.bits) - 1;
  uint32_t h = table_slot(gk, fp, ht.bits);
  for (;;) {
    const uint4 slot = *(const uint4*)(ht.tab + 2 * (uint64_t)h);
    if (slot.x == 0xFFFFFFFFu && slot.y == 0xFFFFFFFFu) break;  // empty
    if (slot.x == gk && fp == (((uint64_t)slot.w << 32) | slot.z)) {
      const uint32_t e = slot.y;
      const uint64_t o = ht.anc[e];
      if (pos >= r + o) {
        const uint64_t p = pos - o + W - 1;
        if (p < n) emit_cand(co, p, e, 1u);
      }
    }
    h = (h + 1) & mask;
  }
}

template <int kProbeWT, int kProbeSlots>
__global__ void __launch_bounds__(kProbeTPB) __attribute__((amdgpu_waves_per_eu(8))) zc_probe_kernel(
    const uint8_t* __restrict__ data, AnchorView av, uint64_t wt0, uint64_t nwt, const uint64_t* __restrict__ tab,
    uint32_t tbits, const uint32_t* __restrict__ gfilt, const uint32_t* __restrict__ anc_off,
    const uint32_t* __restrict__ cls, const uint64_t* __restrict__ vis, const uint8_t* __restrict__ dead, uint64_t r,
    uint64_t n, uint32_t W, HistTab ht, EpochGrid eg,
    Cand* __restrict__ cand, uint64_t cand_cap, unsigned long long* __restrict__ counters) {
  ZC_URGENT();
  // the wave's index, wave-uniform (its wave-tiles' directory entries and
  // pointers then live in scalar registers, not in 20-odd VGPRs per lane)
  const uint64_t gwave = __builtin_amdgcn_readfirstlane(blockIdx.x * (kProbeTPB / 64) + (threadIdx.x >> 6));
  const uint32_t lane = threadIdx.x & 63;
  constexpr int kS = kProbeWT * kProbeSlots;
  __shared__ Cand s_cand[kProbeTPB / 64][kCandStage];
  __shared__ uint32_t s_ncand[kProbeTPB / 64];
  __shared__ uint2 s_pass[kProbeTPB / 64][kPassCap];
  __shared__ uint64_t s_fp[kProbeTPB / 64][kPassCap];
  const CandOut co{cand, cand_cap, counters, s_cand[threadIdx.x >> 6], &s_ncand[threadIdx.x >> 6]};
  if (lane == 0) *co.nstage = 0;
  uint64_t wts[kProbeWT];
  TileAnchors ta[kProbeWT];
#pragma unroll
  for (int t = 0; t < kProbeWT; ++t) {
    wts[t] = wt0 + gwave * kProbeWT + t;
    ta[t] = wts[t] < wt0 + nwt ? tile_anchors(av, wts[t]) : TileAnchors{av.rel, av.g, 0u};
  }
  // level 1: the gear value of every slot
  uint32_t g[kS];
  bool live[kS];
#pragma unroll
  for (int q = 0; q < kS; ++q) {
    const int t = q / kProbeSlots;
    const uint32_t e = lane + 64u * (q % kProbeSlots);
    live[q] = e < ta[t].cnt;
    g[q] = live[q] ? ta[t].g[e] : 0u;
  }
  // level 2: the filter word of every live slot (bit 0: the epoch's table,
  // bit 1: the historic one)
  uint32_t f[kS];
#pragma unroll
  for (int q = 0; q < kS; ++q) {
    const uint32_t fb = g[q] & ((1u << kGFiltBits) - 1);
    f[q] = live[q] && gfilt ? (gfilt[fb >> 5] >> (fb & 31)) & 1u : 0u;
    if (ht.tab) f[q] |= live[q] ? ((ht.filt[fb >> 5] >> (fb & 31)) & 1u) << 1 : 0u;
  }
  // the anchors of the wave that pass: at most kPassCap take the compacted
  // path below; a wave with more (dense or low-entropy content) walks all its
  // slots in the per-lane loop at the end instead
  uint32_t npass = 0;
#pragma unroll
  for (int q = 0; q < kS; ++q) npass += (uint32_t)__popcll(__ballot(f[q] != 0u));
  const bool dense = npass > kPassCap;
  if (!dense) {
    // level 3: the offsets of the anchors that pass; level 4: their
    // fingerprints (the table slot mixes them in), every lane's in flight at
    // once; both compacted into the wave's LDS lists {offset in the wave pair
    // | wave-tile << 24, gear} and {fingerprint}
    uint2* const lst = s_pass[threadIdx.x >> 6];
    uint64_t* const lfp = s_fp[threadIdx.x >> 6];
    uint32_t rel[kS];
#pragma unroll
    for (int q = 0; q < kS; ++q) {
      const int t = q / kProbeSlots;
      rel[q] = f[q] ? ta[t].rel[lane + 64u * (q % kProbeSlots)] : 0u;
    }
    // (anchors the walks skip -- before r + ZC_ANCHOR_MIN_OFF -- read nothing)
    uint64_t fpv[kS];
#pragma unroll
    for (int q = 0; q < kS; ++q) {
      const uint64_t pos = (wts[q / kProbeSlots] << ZC_WT_SHIFT) + rel[q];
      fpv[q] = f[q] && pos >= r + ZC_ANCHOR_MIN_OFF ? anchor_fp(data, pos) : 0ull;
    }
    static_assert(ZC_WT_SHIFT < 24 && kProbeWT <= 64, "pass-list packing");
    uint32_t np = 0;
#pragma unroll
    for (int q = 0; q < kS; ++q) {
      const uint64_t m = __ballot(f[q] != 0u);
      if (f[q]) {
        const uint32_t at = np + lane_prefix(m);
        lst[at] = make_uint2(rel[q] | (uint32_t)(q / kProbeSlots) << 24 | f[q] << 30, g[q]);
        lfp[at] = fpv[q];
      }
      np += (uint32_t)__popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // level 5: the table walks, one anchor per lane
    for (uint32_t j = lane; j < np; j += 64) {
      const uint2 a = lst[j];
      const uint64_t fp = lfp[j];
      const uint32_t t = (a.x >> 24) & 63u;
      const uint64_t pos = ((wt0 + gwave * kProbeWT + t) << ZC_WT_SHIFT) + (a.x & 0xFFFFFFu);
      if (a.x & (1u << 30)) probe_anchor(pos, a.y, fp, tab, tbits, anc_off, cls, vis, dead, r, n, W, eg, co);
      if (a.x & (1u << 31)) probe_hist(pos, a.y, fp, ht, r, n, W, co);
    }
  }
  // wave-tiles with more anchors than the slots above (a dense wave: all)
#pragma unroll
  for (int t = 0; t < kProbeWT; ++t) {
    for (uint32_t e = lane + (dense ? 0u : 64u * kProbeSlots); e < ta[t].cnt; e += 64) {
      const uint32_t gk = ta[t].g[e];
      const uint32_t fb = gk & ((1u << kGFiltBits) - 1);
      const uint64_t pos = (wts[t] << ZC_WT_SHIFT) + ta[t].rel[e];
      const bool pe = gfilt && ((gfilt[fb >> 5] >> (fb & 31)) & 1u);
      const bool ph = ht.tab && ((ht.filt[fb >> 5] >> (fb & 31)) & 1u);
      if ((!pe && !ph) || pos < r + ZC_ANCHOR_MIN_OFF) continue;
      const uint64_t fp = anchor_fp(data, pos);
      if (pe) probe_anchor(pos, gk, fp, tab, tbits, anc_off, cls, vis, dead, r, n, W, eg, co);
      if (ph) probe_hist(pos, gk, fp, ht, r, n, W, co);
    }
  }
  // the wave's staged candidates: one atomic, then a lane per entry
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const uint32_t ns = min(*co.nstage, kCandStage);
  if (ns) {
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(&counters[CNT_CAND], (unsigned long long)ns);
    base = __shfl(base, 0);
    for (uint32_t k = lane; k < ns; k += 64)
      if (base + k < cand_cap) cand[base + k] = co.stage[k];
  }
}

// ---------------------------------------------------------------------------
// zc_verify: one wave per pair, byte-exact equality of two len-byte ranges
__device__ __forceinline__ bool wave_ranges_equal(const uint8_t* __restrict__ data, uint64_t a, uint64_t b,
                                                  uint32_t len, uint32_t lane) {
  bool diff = false;
  uint32_t i = lane * 16;
  // 8 KiB of each range per step: eight 16-byte loads of each side in flight
  // per lane before any compare (the compare loop is otherwise latency-bound)
  constexpr uint32_t kStep = 8 * 64 * 16;
  for (; i + (kStep - 64 * 16) + 16 <= len; i += kStep) {
    uint4 x[8], y[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const v4u32 xv = __builtin_nontemporal_load((const v4u32*)(data + a + i + k * 1024));  // read once
      x[k] = make_uint4(xv[0], xv[1], xv[2], xv[3]);
      __builtin_memcpy(&y[k], data + b + i + k * 1024, 16);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      diff |= (x[k].x != y[k].x) | (x[k].y != y[k].y) | (x[k].z != y[k].z) | (x[k].w != y[k].w);
  }
  for (; i + 16 <= len; i += 64 * 16) {
    uint4 x, y;
    __builtin_memcpy(&x, data + a + i, 16);
    __builtin_memcpy(&y, data + b + i, 16);
    diff |= (x.x != y.x) | (x.y != y.y) | (x.z != y.z) | (x.w != y.w);
  }
  // ragged tail (len not a multiple of 16)
  const uint32_t tail0 = len & ~15u;
  for (uint32_t j = tail0 + lane; j < len; j += 64) diff |= data[a + j] != data[b + j];
  return !__any(diff);
}

// The same with the 8 KiB steps taken in a rotated order (len a multiple of
// 8 KiB): many waves comparing against ONE range (a content class's leader,
// the zero chunk of an all-zero stream) then read different lines of it at
// any moment instead of hammering the same L2 channel.
__device__ __forceinline__ bool wave_ranges_equal_rot(const uint8_t* __restrict__ data, uint64_t a, uint64_t b,
                                                      uint32_t len, uint32_t lane, uint32_t rot) {
  constexpr uint32_t kStep = 8 * 64 * 16;
  if (len % kStep) return wave_ranges_equal(data, a, b, len, lane);
  // 1 KiB blocks, eight per step, the block order rotated by `rot`
  const uint32_t nb = len / 1024;
  uint32_t blk0 = rot % nb;
  bool diff = false;
  for (uint32_t t = 0; t < nb; t += 8) {
    uint4 x[8], y[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint32_t bk = blk0 + t + k;
      bk = bk >= nb ? bk - nb : bk;
      const uint32_t i = bk * 1024 + lane * 16;
      // the member side is read once: non-temporal (whole lines, 1 KiB per
      // instruction); the leader side may be shared by many members (C5)
      const v4u32 xv = __builtin_nontemporal_load((const v4u32*)(data + a + i));
      x[k] = make_uint4(xv[0], xv[1], xv[2], xv[3]);
      __builtin_memcpy(&y[k], data + b + i, 16);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      diff |= (x[k].x != y[k].x) | (x[k].y != y[k].y) | (x[k].z != y[k].z) | (x[k].w != y[k].w);
  }
  return !__any(diff);
}

__global__ void __launch_bounds__(256) zc_verify_kernel(const uint8_t* __restrict__ data,
                                                        const uint64_t* __restrict__ win_start,
                                                        const uint64_t* __restrict__ ref_start,
                                                        uint32_t len, uint32_t npairs,
                                                        uint8_t* __restrict__ ok) {
  ZC_URGENT();
  const uint32_t wave = (uint32_t)(((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const uint32_t lane = threadIdx.x & 63;
  if (wave >= npairs) return;
  const bool eq = wave_ranges_equal(data, win_start[wave], ref_start[wave], len, lane);
  if (lane == 0) ok[wave] = eq ? 1 : 0;
}

// ---------------------------------------------------------------------------
// content classes: refs whose 64-bit keys are equal and whose bytes are equal
// form one class, led by its lowest ref index; only leaders enter the anchor
// table and the exact screen, so repeated content costs one candidate per
// window instead of one per identical chunk
__device__ __forceinline__ uint32_t key_slot(uint64_t k, uint32_t bits) {
  return (uint32_t)((k * kGolden) >> (64 - bits));
}

// ref i into the class table.  A ref with the same key as the ref before it
// is not the lowest of its key: only the first ref of each run of equal keys
// inserts (repeated content -- all-zero streams -- would otherwise serialise
// every ref on one slot's atomics).  A slot is {high word of the key | lowest
// ref}: one CAS inserts a new key; a ref of a key already present lowers the
// slot's ref with a 64-bit atomicMin (equal high words: the minimum is the
// lower ref).  key[] must be complete (the slot holder's key is read).
__device__ __forceinline__ void class_insert(const uint64_t* __restrict__ key, uint32_t i, uint64_t* ckeys,
                                             uint32_t cbits) {
  if (i > 0 && key[i - 1] == key[i]) return;
  const uint64_t k = key[i];
  const uint64_t word = (k & 0xFFFFFFFF00000000ull) | i;  // != kEmpty: i < 2^32 - 1
  const uint32_t mask = (1u << cbits) - 1;
  for (uint32_t h = key_slot(k, cbits);; h = (h + 1) & mask) {
    const unsigned long long prev =
        atomicCAS((unsigned long long*)&ckeys[h], (unsigned long long)kEmpty, (unsigned long long)word);
    if (prev == kEmpty) return;
    if ((prev >> 32) == (k >> 32) && key[(uint32_t)prev] == k) {
      atomicMin((unsigned long long*)&ckeys[h], (unsigned long long)word);
      return;
    }
  }
}

// ref i (with an anchor: gear g, fingerprint fp) into the anchor table and
// its key filter
__device__ __forceinline__ void anchor_insert(uint32_t i, uint32_t g, uint64_t fp, uint64_t* tab, uint32_t tbits,
                                              uint32_t* __restrict__ gfilt) {
  const uint32_t fb = g & ((1u << kGFiltBits) - 1);
  atomicOr(&gfilt[fb >> 5], 1u << (fb & 31));
  const uint64_t word = ((uint64_t)i << 32) | g;
  const uint32_t mask = (1u << tbits) - 1;
  for (uint32_t h = table_slot(g, fp, tbits);; h = (h + 1) & mask) {
    const unsigned long long prev =
        atomicCAS((unsigned long long*)&tab[2 * (uint64_t)h], (unsigned long long)kEmpty, (unsigned long long)word);
    if (prev == kEmpty) {
      tab[2 * (uint64_t)h + 1] = fp;
      return;
    }
  }
}

// thread per ref: the class table (lowest ref per key) and, for a ref with an
// anchor, the anchor table and its key filter
__global__ void zc_index_insert_kernel(const uint64_t* __restrict__ key, const uint32_t* __restrict__ anc_off,
                                       const uint32_t* __restrict__ cg, const uint64_t* __restrict__ cfp,
                                       uint32_t nref, uint64_t* ckeys, uint32_t cbits,
                                       uint64_t* tab, uint32_t tbits, uint32_t* __restrict__ gfilt) {
  ZC_URGENT();
  // threads [0, nref) insert into the class table, [nref, 2 nref) into the
  // anchor table: the two CAS chains run side by side
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * nref) return;
  if (t < nref) {
    class_insert(key, t, ckeys, cbits);
    return;
  }
  const uint32_t i = t - nref;
  if (!tab) return;
  // every ref with an anchor enters the anchor table (the probe keeps class
  // leaders only: classes are not known yet); the ref's three words are read
  // together (one dependent load level before the inserts, not two)
  const uint32_t ao = anc_off[i], g = cg[i];
  const uint64_t fpi = cfp[i];
  if (ao == ZC_NO_ANCHOR) return;
  anchor_insert(i, g, fpi, tab, tbits, gfilt);
}

// historic index: entries [e0, e0 + cnt) that have an anchor into its table
// and filter
__global__ void zc_hist_insert_kernel(const uint32_t* __restrict__ g, const uint64_t* __restrict__ fp,
                                      const uint32_t* __restrict__ anc, uint32_t e0, uint32_t cnt, uint64_t* tab,
                                      uint32_t bits, uint32_t* __restrict__ filt) {
  ZC_URGENT();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cnt) return;
  const uint32_t e = e0 + t, gv = g[e];
  if (anc[e] == ZC_NO_ANCHOR) return;
  const uint32_t fb = gv & ((1u << kGFiltBits) - 1);
  atomicOr(&filt[fb >> 5], 1u << (fb & 31));
  const uint64_t word = ((uint64_t)e << 32) | gv;
  const uint32_t mask = (1u << bits) - 1;
  const uint64_t fpe = fp[e];
  for (uint32_t h = table_slot(gv, fpe, bits);; h = (h + 1) & mask) {
    const unsigned long long prev = atomicCAS((unsigned long long*)&tab[2 * (uint64_t)h], (unsigned long long)kEmpty,
                                              (unsigned long long)word);
    if (prev == kEmpty) {
      tab[2 * (uint64_t)h + 1] = fpe;
      return;
    }
  }
}

// Content classes in two launches.  zc_class_lead_kernel, thread per ref: the
// lowest ref with its key (its leader candidate); cls = itself for now; a
// leader without an anchor is listed for the exact screen; a ref with a lower
// equal-key ref is listed as a pair {ref, leader} for the byte check.
// zc_class_verify_kernel, persistent waves over the pairs, one pair per wave
// at a time (eight 16-byte loads per side in flight per lane): equal bytes ->
// cls = leader (counters[CNT_CLASS]++); else a ref without an anchor is listed
// for the screen.  Every pair's bytes are read once, all pairs side by side.
__global__ void __launch_bounds__(256) zc_class_lead_kernel(
    const uint64_t* __restrict__ key, const uint32_t* __restrict__ anc_off, uint32_t nref,
    const uint64_t* __restrict__ ckeys, uint32_t cbits, uint32_t* __restrict__ cls, uint32_t* __restrict__ ancless,
    uint2* __restrict__ pairs, unsigned long long* __restrict__ counters, ShaGrid sg, const uint64_t* __restrict__ start) {
  ZC_URGENT();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nref) return;
  const uint64_t k = key[i];
  const uint32_t mask = (1u << cbits) - 1;
  uint64_t w;
  for (uint32_t h = key_slot(k, cbits);; h = (h + 1) & mask) {  // the key's slot: equal high word and an
    w = ckeys[h];                                                 // equal key at its ref
    if ((w >> 32) == (k >> 32) && key[(uint32_t)w] == k) break;
  }
  const uint32_t lead = (uint32_t)w;
  cls[i] = i;
  if (lead == i) {
    if (anc_missing(anc_off, i)) ancless[atomicAdd(&counters[CNT_ANCLESS], 1ull)] = i;
  } else if (sg.has(start[i]) && sg.has(start[lead])) {
    // both are grid chunks whose SHA-1 the side stream computes: the pair is
    // decided by key + SHA-1 prefix (zc_class_sha_kernel), listed from the top
    pairs[nref - 1 - atomicAdd(&counters[CNT_SPAIRS], 1ull)] = make_uint2(i, lead);
  } else {
    pairs[atomicAdd(&counters[CNT_PAIRS], 1ull)] = make_uint2(i, lead);
  }
}

// ZC_FLAG_SHA1: the pairs of grid chunks, thread per pair, by the 16-byte
// SHA-1 prefix (their 64-bit keys are equal already): key + prefix equality is
// ChunkIndex::findChunk's own test (chunk_index.cc:119-143), so no bytes are
// read.  Equal -> cls = leader; else a ref without an anchor goes to the screen.
// sg.sha null: every pair joined before the SHA-1 exists (the resolver's
// speculation; it checks the prefixes once they are in and redoes the stream
// if one differs)
__global__ void __launch_bounds__(256) zc_class_sha_kernel(ShaGrid sg, const uint64_t* __restrict__ start,
                                                           const uint32_t* __restrict__ anc_off, uint32_t nref,
                                                           uint32_t* __restrict__ cls, uint32_t* __restrict__ ancless,
                                                           const uint2* __restrict__ pairs,
                                                           unsigned long long* __restrict__ counters) {
  ZC_URGENT();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = t < counters[CNT_SPAIRS];
  bool same = false;
  uint2 pr = make_uint2(0, 0);
  if (live) {
    pr = pairs[nref - 1 - t];
    if (sg.sha) {
      const uint4 a = sg.prefix(start[pr.x]), b = sg.prefix(start[pr.y]);
      same = a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
    } else {
      same = true;
    }
    if (same) cls[pr.x] = pr.y;
    else if (anc_missing(anc_off, pr.x)) ancless[atomicAdd(&counters[CNT_ANCLESS], 1ull)] = pr.x;
  }
  const uint64_t joined = __popcll(__ballot(same));  // one counter atomic per wave
  if ((threadIdx.x & 63) == 0 && joined) atomicAdd(&counters[CNT_CLASS], (unsigned long long)joined);
}

__global__ void __launch_bounds__(256) zc_class_verify_kernel(
    const uint8_t* __restrict__ data, const uint64_t* __restrict__ start, const uint32_t* __restrict__ anc_off,
    uint32_t W, uint32_t* __restrict__ cls, uint32_t* __restrict__ ancless, const uint2* __restrict__ pairs,
    unsigned long long* __restrict__ counters) {
  ZC_URGENT();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t np = counters[CNT_PAIRS];
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  unsigned long long joined = 0;  // one counter atomic per wave, not per pair
  for (uint64_t q = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; q < np; q += nw) {
    const uint2 pr = pairs[q];
    const bool same = wave_ranges_equal_rot(data, start[pr.x], start[pr.y], W, lane, (uint32_t)q);
    if (lane == 0) {
      if (same) {
        cls[pr.x] = pr.y;
        ++joined;
      } else if (anc_missing(anc_off, pr.x)) {
        ancless[atomicAdd(&counters[CNT_ANCLESS], 1ull)] = pr.x;
      }
    }
  }
  if (lane == 0 && joined) atomicAdd(&counters[CNT_CLASS], joined);
}

// ---------------------------------------------------------------------------
// The probe's candidates, checked and ordered on the device (the host walk
// needs the historic ones key-checked and in position order; checking 131,072
// of them one by one on the host and radix-sorting them took 2.8 ms of an
// incremental 8 GiB backup).  Seven launches (launch_cand_order):
//   zc_cand_split: thread per candidate.  An epoch candidate (pad 0: bytes to
//     verify against its ref) is appended to out0.  A historic one (pad 1) is
//     kept iff its window's rolling key equals the entry's -- findChunk's first
//     test (chunk_index.cc:119-143; the SHA-1 prefix, its second, stays with the
//     host, which holds the prefixes) -- and takes a rank in its position
//     bucket p >> bshift (rank ~0: dropped).
//   zc_bucket_sums / zc_bucket_bscan / zc_bucket_offsets: the buckets'
//     exclusive prefix sum, in three coalesced passes.
//   zc_cand_scatter: each kept candidate to its bucket's slots, flagged 1 when
//     its window is a grid chunk whose SHA-1 the side stream computes (joined
//     by key now, its prefix checked when the digests land), else 2 (the host
//     hashes the window).
//   zc_bucket_sort: thread per bucket, its few entries by position; a bucket of
//     more than kBucketSortMax (candidates crowded into a small part of the
//     stream, tests/test_gpu_index_meta.py::test_dense_historic_candidates_vs_oracle)
//     is left unsorted and flagged, and the host sorts the list.
//   zc_cand_out: both lists and the counts into the host's pinned buffers.
constexpr uint32_t kBucketSortMax = 64;
enum { HC_EPOCH = 0, HC_KEPT = 1, HC_UNSORTED = 2, HC_EPOCH_OUT = 3, HC_LAST = 4 };

__global__ void zc_cand_split_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ blk,
                                     const Cand* __restrict__ cand, uint32_t nc, const uint64_t* __restrict__ hkey,
                                     uint64_t pw, uint32_t W, uint32_t bshift, uint32_t* __restrict__ rank,
                                     uint32_t* __restrict__ bcnt, Cand* __restrict__ out0,
                                     unsigned long long* __restrict__ hc) {
  ZC_URGENT();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nc) return;
  const Cand c = cand[i];
  uint32_t rk = ~0u;
  if (c.pad == 0) {
    out0[atomicAdd(&hc[HC_EPOCH], 1ull)] = c;
  } else if (pw + rk_acc(data, blk, c.p + 1 - W, c.p + 1) == hkey[c.ref]) {
    rk = atomicAdd(&bcnt[c.p >> bshift], 1u);
  }
  rank[i] = rk;
}

// exclusive prefix sum of cnt[0, nb) into off[0, nb], off[nb] = the total
// (also hc[HC_KEPT]), in three coalesced launches: block sums of 1024 buckets
// (256 threads x 4), their scan (one workgroup), each block's own scan plus
// its offset.  (One workgroup walking the counts with a contiguous share per
// thread took 0.70 ms beside the grid SHA-1: every load a scattered line on
// one CU.)  The scan launch also moves the epoch-candidate count hc[HC_EPOCH]
// to hc[HC_EPOCH_OUT] and clears hc[HC_EPOCH] and hc[HC_UNSORTED] for the next
// call, so hc needs no fill between calls.
constexpr uint32_t kScanItems = 4, kScanTPB = 256, kScanBlockItems = kScanItems * kScanTPB;

__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* lds, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) lds[w] = x;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t k = 0; k < w; ++k) before += lds[k];
  total = lds[0] + lds[1] + lds[2] + lds[3];
  __syncthreads();
  return before + x - v;
}

__device__ __forceinline__ void load4_cnt(const uint32_t* __restrict__ cnt, uint32_t nb, uint32_t i0, uint32_t* v) {
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) v[k] = i0 + k < nb ? cnt[i0 + k] : 0u;
}

__global__ void __launch_bounds__(kScanTPB) zc_bucket_sums_kernel(const uint32_t* __restrict__ cnt, uint32_t nb,
                                                                  uint32_t* __restrict__ bsum) {
  ZC_URGENT();
  __shared__ uint32_t lds[4];
  uint32_t v[kScanItems];
  load4_cnt(cnt, nb, blockIdx.x * kScanBlockItems + threadIdx.x * kScanItems, v);
  uint32_t total;
  (void)block_excl_scan256(v[0] + v[1] + v[2] + v[3], lds, total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// the block sums' exclusive scan in place (nblk <= kScanBlockItems: one pass)
__global__ void __launch_bounds__(kScanTPB) zc_bucket_bscan_kernel(uint32_t* __restrict__ bsum, uint32_t nblk,
                                                                   uint32_t* __restrict__ off, uint32_t nb,
                                                                   unsigned long long* __restrict__ hc) {
  ZC_URGENT();
  __shared__ uint32_t lds[4];
  uint32_t v[kScanItems];
  const uint32_t i0 = threadIdx.x * kScanItems;
  load4_cnt(bsum, nblk, i0, v);
  uint32_t total;
  uint32_t run = block_excl_scan256(v[0] + v[1] + v[2] + v[3], lds, total);
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {
    if (i0 + k < nblk) bsum[i0 + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 0) {
    off[nb] = total;
    hc[HC_KEPT] = total;
    hc[HC_EPOCH_OUT] = hc[HC_EPOCH];
    hc[HC_EPOCH] = 0;
    hc[HC_UNSORTED] = 0;
  }
}

__global__ void __launch_bounds__(kScanTPB) zc_bucket_offsets_kernel(const uint32_t* __restrict__ cnt, uint32_t nb,
                                                                     const uint32_t* __restrict__ bsum,
                                                                     uint32_t* __restrict__ off) {
  ZC_URGENT();
  __shared__ uint32_t lds[4];
  uint32_t v[kScanItems];
  const uint32_t i0 = blockIdx.x * kScanBlockItems + threadIdx.x * kScanItems;
  load4_cnt(cnt, nb, i0, v);
  uint32_t total;
  uint32_t run = bsum[blockIdx.x] + block_excl_scan256(v[0] + v[1] + v[2] + v[3], lds, total);
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {
    if (i0 + k < nb) off[i0 + k] = run;
    run += v[k];
  }
}

__global__ void zc_cand_scatter_kernel(const Cand* __restrict__ cand, uint32_t nc, const uint32_t* __restrict__ rank,
                                       const uint32_t* __restrict__ off, uint32_t bshift, uint64_t n_gsha, uint32_t W,
                                       uint64_t n, Cand* __restrict__ out) {
  ZC_URGENT();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nc) return;
  const uint32_t rk = rank[i];
  if (rk == ~0u) return;
  Cand c = cand[i];
  const uint64_t ws = c.p + 1 - W;
  const bool grid = n_gsha && ws % W == 0 && ws / W < n_gsha && ws + W <= n;
  c.pad = grid ? 1u : 2u;
  out[off[c.p >> bshift] + rk] = c;
}

__global__ void zc_bucket_sort_kernel(Cand* __restrict__ out, const uint32_t* __restrict__ off, uint32_t nb,
                                      uint32_t* __restrict__ bcnt, unsigned long long* __restrict__ hc) {
  ZC_URGENT();
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  bcnt[b] = 0;  // zero again for the next call (the buffer is zeroed once, when made)
  const uint32_t lo = off[b], hi = off[b + 1];
  if (hi - lo < 2) return;
  if (hi - lo > kBucketSortMax) {
    atomicMax(&hc[HC_UNSORTED], 1ull);
    return;
  }
  for (uint32_t i = lo + 1; i < hi; ++i) {
    const Cand x = out[i];
    uint32_t j = i;
    for (; j > lo && out[j - 1].p > x.p; --j) out[j] = out[j - 1];
    out[j] = x;
  }
}

// ---------------------------------------------------------------------------
// zc_range_digest: RollingHash::digest of [a, b) = 257^(b-a) + acc
__global__ void zc_range_digest_kernel(const uint8_t* __restrict__ data, uint64_t n,
                                       const uint64_t* __restrict__ blk, const uint64_t* __restrict__ a,
                                       const uint64_t* __restrict__ b, uint32_t nr,
                                       uint64_t* __restrict__ out) {
  ZC_URGENT();
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nr) return;
  out[i] = pow257_dev(b[i] - a[i]) + rk_acc(data, blk, a[i], b[i]);
}

// the same for at most kSmallRanges ranges passed by value (no upload)
constexpr uint32_t kSmallRanges = 4;
struct SmallRanges {
  uint64_t a[kSmallRanges], b[kSmallRanges];
  uint32_t nr;
};
__global__ void zc_range_digest_small_kernel(const uint8_t* __restrict__ data, uint64_t n,
                                             const uint64_t* __restrict__ blk, SmallRanges rg,
                                             uint64_t* __restrict__ out) {
  ZC_URGENT();
  const uint32_t i = threadIdx.x;
  if (i < rg.nr) out[i] = pow257_dev(rg.b[i] - rg.a[i]) + rk_acc(data, blk, rg.a[i], rg.b[i]);
}

// ---------------------------------------------------------------------------
// zc_fscan: exact window hash H(p) mod 2^32 at every p >= p_start, screened
// against the low words of keys without anchors; emits maximal hit runs.
__device__ __forceinline__ bool f_member(uint32_t h, const uint32_t* f32, uint32_t nf,
                                         const uint32_t* s_bits, const uint32_t* bloom = nullptr,
                                         uint32_t bbits = 0) {
  (void)bloom;
  (void)bbits;  // (the Bloom mode tests 64-bit keys: zc_fscan_kernel's fhit)
  if (s_bits) return (s_bits[h >> 18] >> ((h >> 13) & 31)) & 1u;  // bit index h >> 13
  bool m = false;
  for (uint32_t k = 0; k < nf; ++k) m |= (f32[k] == h);
  return m;
}

constexpr uint32_t kFLinearMax = 16;
constexpr uint32_t kFBitmapWords = 1u << 14;  // 2^19 bits = 64 KiB, index = h >> 13

__global__ void __launch_bounds__(ZC_TPB) zc_fscan_kernel(
    const uint8_t* __restrict__ data, uint64_t n, const uint64_t* __restrict__ blk, uint32_t W,
    uint32_t pw32, uint64_t p_start, uint64_t p_end, uint64_t tile0, const uint32_t* __restrict__ f32, uint32_t nf,
    const uint32_t* __restrict__ fbits, const uint32_t* __restrict__ bloom, uint32_t bbits, Run* __restrict__ runs,
    uint64_t runs_cap, uint64_t* __restrict__ tile_off, uint32_t* __restrict__ tile_cnt,
    unsigned long long* __restrict__ counters) {
  extern __shared__ uint32_t s_dyn[];  // bitmap (if used)
  __shared__ uint64_t s_rs[ZC_RUN_SLOTS * ZC_TPB], s_re[ZC_RUN_SLOTS * ZC_TPB];
  __shared__ uint32_t s_tmp[ZC_TPB / 64];
  __shared__ uint64_t s_base;
  __shared__ uint32_t s_keys[kFLinearMax];

  const uint32_t tid = threadIdx.x;
  const uint64_t tile = tile0 + blockIdx.x;
  const uint32_t* s_bits = nullptr;
  if (nf > kFLinearMax) {
    for (uint32_t i = tid; i < kFBitmapWords; i += ZC_TPB) s_dyn[i] = fbits[i];
    s_bits = s_dyn;
  } else if (tid < nf) {
    s_keys[tid] = f32[tid];
  }
  __syncthreads();

  const uint64_t span0 = tile * ZC_TILE + (uint64_t)tid * ZC_SPAN;
  uint64_t ps = span0 > p_start ? span0 : p_start;
  const uint64_t lim = p_end < n ? p_end : n;
  uint64_t pe = span0 + ZC_SPAN < lim ? span0 + ZC_SPAN : lim;
  uint32_t cnt = 0;
  uint64_t open = ~0ull;
  // the window value: its accumulator mod 2^32 against the key words, or
  // (Bloom mode, large key sets) mod 2^64 against the 64-bit Bloom filter
  const uint64_t pw64 = bloom ? pow257_dev(W) : 0;
  auto fstart = [&](uint64_t a, uint64_t b) -> uint64_t {
    return bloom ? rk_acc<false>(data, blk, a, b) : (uint64_t)rk_acc32(data, blk, a, b);
  };
  auto fstep = [&](uint64_t v, uint32_t bi, uint32_t bo) -> uint64_t {
    return bloom ? v * 257u + bi - (uint64_t)bo * pw64 : (uint64_t)((uint32_t)v * 257u + bi - bo * pw32);
  };
  auto fhit = [&](uint64_t v) -> bool {
    if (bloom) {
      const uint64_t key = v + pw64;
      const uint2 w = ((const uint2*)bloom)[bloom_block(key, bbits)];
      const uint32_t g = bloom_seed(key), ml = bloom_lo(g), mh = bloom_hi(g);
      return (w.x & ml) == ml && (w.y & mh) == mh;
    }
    return f_member((uint32_t)v + pw32, s_keys, nf, s_bits);
  };
  auto emit = [&](uint64_t a, uint64_t b) {
    if (cnt < ZC_RUN_SLOTS) {
      s_rs[cnt * ZC_TPB + tid] = a;
      s_re[cnt * ZC_TPB + tid] = b;
    }
    ++cnt;
  };
  if (ps < pe) {
    // window [p-W+1, p] ends at p
    uint64_t V = fstart(ps + 1 - W, ps + 1);
    if (fhit(V)) open = ps;
    uint64_t p = ps + 1;
    for (; p + 4 <= pe; p += 4) {
      uint32_t xin = load4_any(data, p), xout = load4_any(data, p - W);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        V = fstep(V, (xin >> (8 * k)) & 0xFFu, (xout >> (8 * k)) & 0xFFu);
        bool hit = fhit(V);
        if (hit && open == ~0ull) open = p + k;
        if (!hit && open != ~0ull) {
          emit(open, p + k);
          open = ~0ull;
        }
      }
    }
    for (; p < pe; ++p) {
      V = fstep(V, data[p], data[p - W]);
      bool hit = fhit(V);
      if (hit && open == ~0ull) open = p;
      if (!hit && open != ~0ull) {
        emit(open, p);
        open = ~0ull;
      }
    }
    if (open != ~0ull) emit(open, pe);
  }

  // ordered compaction, then merge runs that continue across lane spans
  uint32_t total;
  uint32_t off = block_excl_scan(cnt, s_tmp, total);
  if (total == 0) {
    if (tid == 0) {
      tile_off[tile] = 0;
      tile_cnt[tile] = 0;
    }
    return;
  }
  // lanes that overflowed their slots rescan (rare); otherwise stage in order
  // into a tile-wide LDS list, reusing s_rs/s_re after a barrier
  uint64_t my_s[ZC_RUN_SLOTS], my_e[ZC_RUN_SLOTS];
  for (uint32_t i = 0; i < ZC_RUN_SLOTS; ++i) {
    my_s[i] = s_rs[i * ZC_TPB + tid];
    my_e[i] = s_re[i * ZC_TPB + tid];
  }
  const bool fits = total <= ZC_RUN_SLOTS * ZC_TPB;
  __syncthreads();
  if (fits && cnt <= ZC_RUN_SLOTS) {
    for (uint32_t i = 0; i < cnt; ++i) {
      s_rs[off + i] = my_s[i];
      s_re[off + i] = my_e[i];
    }
  }
  // whether any lane overflowed: then skip the LDS merge and write raw runs
  __shared__ uint32_t s_over;
  if (tid == 0) s_over = 0;
  __syncthreads();
  if (cnt > ZC_RUN_SLOTS) atomicOr(&s_over, 1u);
  __syncthreads();
  if (!fits || s_over) {
    if (tid == 0) {
      uint64_t base = atomicAdd(&counters[CNT_RUNS], (unsigned long long)total);
      if (base + total > runs_cap) atomicOr(&counters[CNT_FOVF], 1ull);
      tile_off[tile] = base;
      tile_cnt[tile] = total;
      s_base = base;
    }
    __syncthreads();
    const uint64_t base = s_base;
    if (base + total > runs_cap || cnt == 0) return;
    Run* dst = runs + base + off;
    if (cnt <= ZC_RUN_SLOTS) {
      for (uint32_t i = 0; i < cnt; ++i) dst[i] = Run{my_s[i], my_e[i]};
      return;
    }
    // rescan this lane's positions, writing every run
    uint64_t V = fstart(ps + 1 - W, ps + 1);
    uint64_t o2 = fhit(V) ? ps : ~0ull;
    uint32_t w = 0;
    for (uint64_t p = ps + 1; p < pe; ++p) {
      V = fstep(V, data[p], data[p - W]);
      bool hit = fhit(V);
      if (hit && o2 == ~0ull) o2 = p;
      if (!hit && o2 != ~0ull) {
        dst[w++] = Run{o2, p};
        o2 = ~0ull;
      }
    }
    if (o2 != ~0ull) dst[w++] = Run{o2, pe};
    return;
  }
  __syncthreads();
  // merge: run i is a head unless it starts where run i-1 ends
  uint32_t nheads;
  uint32_t head_ex = 0;
  uint32_t my_heads = 0;
  // each thread handles runs i = tid, tid + 256, ... ; total <= 4 * 256
  bool is_head[ZC_RUN_SLOTS];
  for (uint32_t j = 0; j < ZC_RUN_SLOTS; ++j) {
    uint32_t i = tid * ZC_RUN_SLOTS + j;
    is_head[j] = i < total && (i == 0 || s_re[i - 1] != s_rs[i]);
    my_heads += is_head[j];
  }
  head_ex = block_excl_scan(my_heads, s_tmp, nheads);
  if (tid == 0) {
    uint64_t base = atomicAdd(&counters[CNT_RUNS], (unsigned long long)nheads);
    if (base + nheads > runs_cap) atomicOr(&counters[CNT_FOVF], 1ull);
    tile_off[tile] = base;
    tile_cnt[tile] = nheads;
    s_base = base;
  }
  __syncthreads();
  const uint64_t base = s_base;
  if (base + nheads > runs_cap) return;
  uint32_t hid = head_ex;
  for (uint32_t j = 0; j < ZC_RUN_SLOTS; ++j) {
    uint32_t i = tid * ZC_RUN_SLOTS + j;
    if (i >= total) break;
    if (is_head[j]) {
      runs[base + hid].start = s_rs[i];
      ++hid;
    }
    bool last = (i + 1 == total) || (s_re[i] != s_rs[i + 1]);
    if (last) runs[base + hid - 1].end = s_re[i];
  }
}

// ---------------------------------------------------------------------------
// zc_fscan_staged: the same exact screen at streaming speed.
//
// One wave per screen wave-tile (64 lane spans of ZC_FLSPAN bytes, a lane
// rolls H(p) mod 2^32 through its span), persistent over the wave-tiles.  Both
// byte streams a lane needs -- the in-bytes b[p] and the out-bytes b[p - W] --
// are staged through a private 2-slot LDS ring with global_load_lds_dwordx4,
// 64-byte rounds, rows 8 KiB apart (tools/ubench/stage_bench2.hip: 4 KiB row
// strides lose ~12 % of the streaming rate, 8 KiB ones do not).  The out-rows
// are staged 16-byte aligned one piece ahead of the bytes they serve; a lane
// keeps the previous piece and funnels each 16-byte out piece from two staged
// ones (the misalignment m = -W mod 16 is kernel-uniform: Q = m >> 2 is a
// template parameter, m & 3 an alignbyte).
//
// Per byte: V = 257 V + b[p] - 257^W b[p-W] (V = H(p) - 257^W); the key test
// is one compare per key (NF <= 4) or a bit of an LDS map, and its ballot is
// folded into two wave masks per 16-byte piece (lanes with any hit, lanes with
// all hits).  Only a lane whose run state changes inside a piece (a run opens
// or closes, or the piece straddles p_start) re-rolls the piece to record run
// boundaries, so all-hit and no-hit data (all-zero streams, random streams)
// pay the roll and the compare only.  Runs are closed at span ends and merged
// across the wave at the wave-tile end.
constexpr int kFRounds = ZC_FLSPAN / ZC_FROUND;          // rounds per wave-tile
constexpr int kFDmaHalf = 64 * ZC_FROUND / 1024;         // DMA instructions per stream per round
constexpr int kFDma = 2 * kFDmaHalf;
constexpr int kFPieces = ZC_FROUND / 16;
constexpr int kFRunSlots = 2;                            // runs per lane per wave-tile (else overflow)
constexpr uint32_t kFMapWords = 1u << 12;                // 2^17-bit key map, bit (h >> 15)
__host__ __device__ constexpr uint32_t frow_swizzle(uint32_t row) { return (row / (256 / ZC_FROUND)) % kFPieces; }

struct FKeys {
  uint32_t k[16];         // keys - 257^W (compared with V); unused slots repeat k[0]
  const uint32_t* dkeys;  // NF = 32: the nk keys, sorted (copied to LDS)
  uint32_t nk;            // NF >= 64: the Bloom filter's size, log2 blocks
  const uint32_t* bloom;  // NF >= 64: the Bloom filter (global memory, L2 resident)
  uint64_t pw64;          // NF >= 64: 257^W mod 2^64
  const uint2* chk;       // NF = 65: the check table (buckets of four 16-bit check words)
  uint32_t cbits;         // NF = 65: its size, log2 buckets (plus kChkPad)
};
// run slots per lane per wave-tile: the two-level Bloom mode's false hits
// (~K / 6e9 per position) need more than the exact modes' two; the one-level
// mode's filter hits are checked in the kernel (~1e-5 of them left)
template <int NF>
constexpr int kFRS = NF == 64 ? 7 : NF == 65 ? 4 : kFRunSlots;
// threads per workgroup: the Bloom mode runs 4 waves (one per SIMD; the
// filter gathers, not latency, bound it) so the LDS holds its first level
template <int NF>
constexpr int kFTPBn = NF == 64 ? 256 : ZC_FTPB;

template <int RS>
__device__ __forceinline__ void put_run(uint32_t (&rs)[RS], uint32_t (&re)[RS], uint32_t i, uint32_t a, uint32_t b) {
#pragma unroll
  for (int k = 0; k < RS; ++k)
    if (i == (uint32_t)k) {
      rs[k] = a;
      re[k] = b;
    }
}
constexpr uint32_t kFLdsKeys = 2048;  // NF = 32: keys searched in LDS (the rest of the 160 KiB)

// Rabin-Karp accumulator mod 2^32 of [a, a + W) for a, W multiples of ZC_SPAN:
// a fold of span digests, loads batched eight at a time
__device__ __forceinline__ uint32_t fold_spans32(const uint64_t* __restrict__ blk, uint64_t a, uint32_t nspan) {
  const uint32_t m = (uint32_t)span_mul();
  uint32_t acc = 0;
  const uint64_t* p = blk + a / ZC_SPAN;
  uint32_t k = 0;
  for (; k + 8 <= nspan; k += 8) {
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (uint32_t)p[k + i];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc = acc * m + v[i];
  }
  for (; k < nspan; ++k) acc = acc * m + (uint32_t)p[k];
  return acc;
}

// NF = 1, 4: compares; 0: a bit of the 2^17-bit key map (false hits at
// K / 2^17 per position); 16, 32: the map, then -- only where some lane of
// the wave hit it -- the exact key test (false hits at K / 2^32): 16
// compares, or a binary search of the sorted keys in LDS (K <= kFLdsKeys)
template <int NF>
__device__ __forceinline__ bool f_hit(uint32_t V, const FKeys& K, const uint32_t* s_map, const uint32_t* s_keys,
                                      uint32_t pw32) {
  if (NF == 1) return V == K.k[0];
  if (NF == 4) return (V == K.k[0]) | (V == K.k[1]) | (V == K.k[2]) | (V == K.k[3]);
  const uint32_t key = V + pw32, h = key >> 15;
  bool hit = (s_map[h >> 5] >> (h & 31)) & 1u;
  if (NF == 16 && __builtin_expect(__ballot(hit) != 0, 0)) {
    bool e = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) e |= V == K.k[i];
    hit = hit && e;
  }
  if (NF == 32 && __builtin_expect(__ballot(hit) != 0, 0)) {
    uint32_t lo = 0, len = K.nk;  // lower bound of key in s_keys[0, nk)
    while (len > 0) {
      const uint32_t half = len >> 1;
      if (s_keys[lo + half] < key) {
        lo += half + 1;
        len -= half + 1;
      } else {
        len = half;
      }
    }
    hit = hit && lo < K.nk && s_keys[lo] == key;
  }
  return hit;
}

// 16-byte window at byte offset 4Q + s of the 32 bytes lo||hi
template <int Q>
__device__ __forceinline__ uint4 funnel16(uint4 lo, uint4 hi, uint32_t s) {
  const uint32_t a[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  return make_uint4(__builtin_amdgcn_alignbyte(a[Q + 1], a[Q], s), __builtin_amdgcn_alignbyte(a[Q + 2], a[Q + 1], s),
                    __builtin_amdgcn_alignbyte(a[Q + 3], a[Q + 2], s),
                    __builtin_amdgcn_alignbyte(a[Q + 4], a[Q + 3], s));
}

template <int Q, int NF>
__global__ void __launch_bounds__(kFTPBn<NF>, 1) zc_fscan_staged_kernel(
    const uint8_t* __restrict__ data, uint64_t n, const uint64_t* __restrict__ blk, uint32_t W, uint32_t pw32,
    uint32_t sbyte, uint64_t p_start, uint64_t p_end, uint64_t wt0, uint64_t nwt, FKeys K,
    const uint32_t* __restrict__ fmap,
    Run* __restrict__ runs, uint64_t runs_cap, uint64_t* __restrict__ wt_off, uint32_t* __restrict__ wt_cnt,
    unsigned long long* __restrict__ counters) {
  constexpr int kTPB = kFTPBn<NF>;
  constexpr int kWaves = kTPB / 64;
  constexpr uint32_t kSlot = 64 * ZC_FROUND;  // bytes of one stream's round
  __shared__ __attribute__((aligned(16))) uint8_t ring[kWaves][2][2 * kSlot];  // [slot][in | out]
  __shared__ uint32_t s_map[NF == 0 || NF == 16 || NF == 32 ? kFMapWords : 1];
  __shared__ uint32_t s_keys[NF == 32 ? kFLdsKeys : 1];
  __shared__ uint32_t s_pf[NF == 64 ? kBloomPfWords : 1];  // the Bloom filter's first level
  constexpr int RS = kFRS<NF>;
  __shared__ uint32_t s_rs[kWaves][64 * RS], s_re[kWaves][64 * RS];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (NF == 0 || NF == 16 || NF == 32) {
    for (uint32_t i = tid; i < kFMapWords; i += kTPB) s_map[i] = fmap[i];
    if (NF == 32)
      for (uint32_t i = tid; i < K.nk; i += kTPB) s_keys[i] = K.dkeys[i];
    __syncthreads();
  }
  if (NF == 64) {
    const uint4* pf = (const uint4*)(K.bloom + (2u << K.nk));
    for (uint32_t i = tid; i < kBloomPfWords / 4; i += kTPB) ((uint4*)s_pf)[i] = pf[i];
    __syncthreads();
  }
  const uint32_t m = (uint32_t)(4 * Q) + sbyte;  // = -W mod 16
  const uint32_t wave_u = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform (scalar descriptors)
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wave_u, nw = (uint64_t)gridDim.x * kWaves;
  const uint32_t ntk = nwt > gw ? (uint32_t)((nwt - 1 - gw) / nw + 1) : 0;
  const uint32_t nR = ntk * kFRounds;
  uint8_t* myring = ring[wave_u][0];
  uint32_t* lrs = s_rs[wave];
  uint32_t* lre = s_re[wave];
  // this lane's share of DMA instruction j (rows 8 KiB apart, source piece
  // swizzled so the per-lane ds_read_b128 of a row is conflict free)
  uint32_t lane_off[kFDmaHalf];
#pragma unroll
  for (int j = 0; j < kFDmaHalf; ++j) {
    const uint32_t row = j * (1024 / ZC_FROUND) + lane / kFPieces;
    lane_off[j] = row * ZC_FLSPAN + ((lane % kFPieces) ^ frow_swizzle(row)) * 16;
  }
  const uint32_t sw = frow_swizzle(lane);
  const uint64_t out_shift = (uint64_t)W + m - 16;  // staged out-row = in-row - out_shift
  // DMA through buffer descriptors rebuilt per round (scalar work only): the
  // lane's part of each instruction is its loop-invariant 32-bit offset, and
  // the descriptor's range check makes pieces past the stream end read as
  // zero.  Out-rows before the stream start (the first wave-tiles) get a
  // wrapped offset, out of range as well; their bytes are cleared anyway.
  auto issue = [&](uint32_t Rx) {
    const uint32_t k = Rx / kFRounds, r = Rx - k * kFRounds;
    const uint64_t at = (wt0 + gw + (uint64_t)k * nw) * ZC_FWT + (uint64_t)r * ZC_FROUND;
    uint8_t* dst = myring + (Rx & 1) * (2 * kSlot);
    const uint64_t in_left = n - at;  // > 0: every issued round starts inside the stream
    const auto rin = __builtin_amdgcn_make_buffer_rsrc((void*)(data + at), (short)0,
                                                       (int)(in_left < 0x7FFFFFF0ull ? in_left : 0x7FFFFFF0ull),
                                                       0x00020000);
    const uint64_t ob = at >= out_shift ? at - out_shift : 0;
    const uint32_t oadj = at >= out_shift ? 0u : (uint32_t)(at - out_shift);  // wraps: out of range
    const uint64_t out_left = n - ob;
    const auto rout = __builtin_amdgcn_make_buffer_rsrc((void*)(data + ob), (short)0,
                                                        (int)(out_left < 0x7FFFFFF0ull ? out_left : 0x7FFFFFF0ull),
                                                        0x00020000);
#pragma unroll
    for (int j = 0; j < kFDmaHalf; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_void_t*)(dst + j * 1024), 16, (int)lane_off[j], 0, 0, 0);
    // the out-bytes are the in-bytes another lane read a moment ago (W
    // earlier); their last use: in the Bloom mode marked non-temporal (nt),
    // so the streamed lines leave L2 to the filter
    constexpr int kOutAux = NF >= 64 ? 2 : 0;
#pragma unroll
    for (int j = 0; j < kFDmaHalf; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rout, (lds_void_t*)(dst + kSlot + j * 1024), 16,
                                               (int)(lane_off[j] + oadj), 0, 0, kOutAux);
  };
  if (nR > 0) issue(0);
  if (nR > 1) issue(1);

  uint32_t V = 0;
  uint64_t V64 = 0;  // NF = 64: the 64-bit window accumulator
  uint4 carry = make_uint4(0, 0, 0, 0);
  uint64_t wtbase = 0, ps = 0;
  bool open = false, ovf = false;
  uint64_t open_mask = 0;  // wave-uniform mirror of `open`
  bool need_valid = false, head = false;
  uint32_t rstart = 0, nrun = 0;
  uint32_t rs[RS], re[RS];

#pragma unroll 1
  for (uint32_t R = 0; R < nR; ++R) {
    const uint32_t k = R / kFRounds, r = R - k * kFRounds;
    if (r == 0) {
      // a new wave-tile: drain everything in flight (its first two rounds and
      // the previous wave-tile's stores), then the lane's start state: V of
      // the window ending just before the span, and the out-piece before it
      wait_vmcnt<0>();
      wtbase = (wt0 + gw + (uint64_t)k * nw) * ZC_FWT;
      ps = wtbase + (uint64_t)lane * ZC_FLSPAN;
      // (bytes before the stream count as zero: V(p) = acc of [max(0, p - W + 1), p])
      V = 0;
      carry = make_uint4(0, 0, 0, 0);
      if (ps < n) {
        if (ps >= W)
          V = (W % ZC_SPAN == 0) ? fold_spans32(blk, ps - W, W / ZC_SPAN) : rk_acc32(data, blk, ps - W, ps);
        else
          V = fold_spans32(blk, 0, (uint32_t)(ps / ZC_SPAN));
        if (ps >= (uint64_t)W + m) {
          carry = *(const uint4*)(data + ps - W - m);
        } else if (ps + 16 > (uint64_t)W + m) {  // the piece straddles the stream start
          uint32_t w[4] = {0, 0, 0, 0};
          for (uint32_t i = 0; i < 16; ++i) {
            const int64_t at = (int64_t)ps - (int64_t)W - (int64_t)m + i;
            if (at >= 0) w[i >> 2] |= (uint32_t)data[at] << (8 * (i & 3));
          }
          carry = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
      if constexpr (NF >= 64) V64 = ps < n ? rk_acc<false>(data, blk, ps >= W ? ps - W : 0, ps) : 0;
      head = wtbase < (uint64_t)W + 16;
      need_valid = wtbase < p_start || wtbase + ZC_FWT > p_end;
      open = false;
      open_mask = 0;
      ovf = false;
      nrun = 0;
    } else if (R + 1 < nR) {
      wait_vmcnt<kFDma>();
    } else {
      wait_vmcnt<0>();
    }
    const uint8_t* slot = myring + (R & 1) * (2 * kSlot);
    uint4 vin[kFPieces], vst[kFPieces];
#pragma unroll
    for (int p = 0; p < kFPieces; ++p) {
      vin[p] = *(const uint4*)(slot + lane * ZC_FROUND + ((p ^ sw) << 4));
      vst[p] = *(const uint4*)(slot + kSlot + lane * ZC_FROUND + ((p ^ sw) << 4));
    }
    wait_lgkmcnt<0>();  // the slot is free
    if constexpr (NF >= 64) {
      // Bloom mode: the window values of the whole round first, then one
      // gather of a filter word per position, all in flight together and
      // issued before the next round's DMA (a later load could not be waited
      // for without draining that DMA); the per-piece pass below then reads
      // hit masks
      uint32_t xo[kFPieces][4], hm[kFPieces];
      // the out-bytes of piece p (b[p - W], zero before the stream)
      auto out_piece = [&](int p, uint32_t (&o)[4]) {
        const uint64_t pp = ps + (uint64_t)r * ZC_FROUND + 16 * p;
        const uint4 vout = funnel16<Q>(p == 0 ? carry : vst[p - 1], vst[p], sbyte);
        o[0] = vout.x;
        o[1] = vout.y;
        o[2] = vout.z;
        o[3] = vout.w;
        if (head && pp < W) {
          const uint64_t z = (uint64_t)W - pp;
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const uint64_t lo = 4 * d;
            o[d] = z >= lo + 4 ? 0u : (z > lo ? o[d] & (~0u << (8 * (z - lo))) : o[d]);
          }
        }
      };
      if constexpr (NF == 64) {
#pragma unroll
        for (int p = 0; p < kFPieces; ++p) out_piece(p, xo[p]);
      }
      if constexpr (NF == 64) {
        // two halves of two pieces: 32 gathers in flight per lane each.  A
        // position first tests the filter's first level in LDS; one whose bit
        // is clear gathers block 0 instead of its own (all such lanes of the
        // wave share one line), so the L2 gathers scale with the first level's
        // fill, not with the positions
        const uint2* const bl = (const uint2*)K.bloom;
        const uint32_t bsh = 32u - K.nk;
  #pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          uint2 bw[2][16];
          uint32_t gs[2][16], pre[2];
  #pragma unroll
          for (int pi = 0; pi < 2; ++pi) {
            const int p = 2 * hf + pi;
            const uint32_t xin[4] = {vin[p].x, vin[p].y, vin[p].z, vin[p].w};
            uint32_t bi[16], pw[16];
  #pragma unroll
            for (int d = 0; d < 4; ++d)
  #pragma unroll
              for (int q = 0; q < 4; ++q) {
                V64 = V64 * 257u + ((xin[d] >> (8 * q)) & 0xFFu) - (uint64_t)((xo[p][d] >> (8 * q)) & 0xFFu) * K.pw64;
                const uint64_t key = V64 + K.pw64;
                // bloom_block: the high word of key * golden; bloom_pf: the low word's top bits
                const uint64_t kg = key * 0x9E3779B97F4A7C15ull;
                const uint32_t hi = (uint32_t)(kg >> 32);
                const uint32_t f = (uint32_t)kg >> (32 - kBloomPfBits);
                bi[4 * d + q] = hi >> bsh;
                pw[4 * d + q] = s_pf[f >> 5] >> (f & 31u);
                gs[pi][4 * d + q] = bloom_seed(key);
              }
            uint32_t pm = 0;
  #pragma unroll
            for (int i = 0; i < 16; ++i) {
              pm |= (pw[i] & 1u) << i;
              bw[pi][i] = bl[(pw[i] & 1u) ? bi[i] : 0u];
            }
            pre[pi] = pm;
          }
  #pragma unroll
          for (int pi = 0; pi < 2; ++pi) {
            uint32_t m16 = 0;
  #pragma unroll
            for (int i = 0; i < 16; ++i) m16 |= bloom_test(bw[pi][i].x, bw[pi][i].y, gs[pi][i]) << i;
            hm[2 * hf + pi] = m16 & pre[pi];
          }
        }
      } else {
        // one level (large key sets, where an LDS first level passes nearly
        // every position): every position gathers its block of an L2-sized
        // filter (~8 keys per block: ~2 % false hits), and each filter hit
        // reads the key's bucket of the check table (8 bytes): its check word
        // there -- a hit; an empty slot -- a miss; a full bucket -- the next
        // bucket.  A hit the check lets through falsely (~1e-5 of the filter's
        // false hits) is a run the walk's exact key test drops.
        const uint2* const bl = (const uint2*)K.bloom;
        const uint32_t bsh = 32u - K.nk, csh = 32u - K.cbits;
        // piece by piece (16 gathers in flight per lane, two waves per SIMD),
        // pipelined: piece p + 1's filter gathers are issued behind piece p's
        // check-table reads, so the check's round trip overlaps them
        uint2 bw[2][16], ev[2][16];
        uint32_t gs[2][16], cb[2][16], cw[2][8], hx[2];  // cw: the check words, two per register
        auto gather = [&](int p) {  // the keys of piece p and their filter blocks
          const int b = p & 1;
          const uint32_t xin[4] = {vin[p].x, vin[p].y, vin[p].z, vin[p].w};
          uint32_t xp[4];
          out_piece(p, xp);
#pragma unroll
          for (int d = 0; d < 4; ++d)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              V64 = V64 * 257u + ((xin[d] >> (8 * q)) & 0xFFu) - (uint64_t)((xp[d] >> (8 * q)) & 0xFFu) * K.pw64;
              const uint64_t key = V64 + K.pw64;
              const uint32_t hi = (uint32_t)((key * kGolden) >> 32);  // bloom_block, chk_bucket
              gs[b][4 * d + q] = bloom_seed(key);
              cb[b][4 * d + q] = hi >> csh;
              bw[b][4 * d + q] = bl[hi >> bsh];
            }
        };
        auto test = [&](int p) {  // the filter test, and the hits' check-table reads
          const int b = p & 1;
          uint32_t h = 0;
#pragma unroll
          for (int i = 0; i < 16; ++i) h |= bloom_test(bw[b][i].x, bw[b][i].y, gs[b][i]) << i;
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if ((h >> i) & 1u) ev[b][i] = K.chk[cb[b][i]];
#pragma unroll
          for (int i = 0; i < 8; ++i) cw[b][i] = chk_word_of_seed(gs[b][2 * i]) | chk_word_of_seed(gs[b][2 * i + 1]) << 16;
          hx[b] = h;
        };
        auto check = [&](int p) {  // the check words: exact hits of piece p
          const int b = p & 1;
          uint32_t h = hx[b], slow = 0;
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if ((h >> i) & 1u) {
              const uint32_t v = chk_match(ev[b][i], (cw[b][i >> 1] >> (16 * (i & 1))) & 0xFFFFu);
              if (v == 0) h &= ~(1u << i);  // an empty slot: not in the set
              else if (v == 2) slow |= 1u << i;  // a full bucket without it
            }
          if (__builtin_expect(__ballot(slow != 0) != 0, 0)) {
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if ((slow >> i) & 1u) {
                const uint32_t c = (cw[b][i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
                uint32_t k = cb[b][i] + 1, v;
                while ((v = chk_match(K.chk[k], c)) == 2) ++k;  // the last pad bucket ends every chain
                if (v == 0) h &= ~(1u << i);
              }
          }
          hm[p] = h;
        };
        gather(0);
        test(0);
#pragma unroll
        for (int p = 1; p < kFPieces; ++p) {
          gather(p);
          check(p - 1);
          test(p);
        }
        check(kFPieces - 1);
      }
      if (R + 2 < nR) issue(R + 2);
#pragma unroll
      for (int p = 0; p < kFPieces; ++p) {
        const uint64_t pp = ps + (uint64_t)r * ZC_FROUND + 16 * p;
        const uint32_t xin[4] = {vin[p].x, vin[p].y, vin[p].z, vin[p].w};
        uint64_t any = 0, all = ~0ull;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint64_t b = __ballot((hm[p] >> i) & 1u);
          any |= b;
          all &= b;
        }
        uint64_t need = (open_mask & ~all) | (~open_mask & any);
        if (need_valid) {
          const uint64_t some = __ballot(pp < p_start || pp + 16 > p_end);
          need = (need & ~some) | (some & (any | open_mask));
        }
        if (__builtin_expect(need != 0, 0)) {
          if ((need >> lane) & 1) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const uint64_t pos = pp + i;
              const bool h = ((hm[p] >> i) & 1u) && pos >= p_start && pos < p_end;
              const uint32_t rel = (uint32_t)(pos - wtbase);
              if (h && !open) {
                open = true;
                rstart = rel;
              } else if (!h && open) {
                open = false;
                if (nrun < RS) put_run(rs, re, nrun, rstart, rel);
                else ovf = true;
                ++nrun;
              }
            }
          }
          open_mask = __ballot(open);
        }
        (void)xin;
      }
    } else {
    if (R + 2 < nR) issue(R + 2);

#pragma unroll
    for (int p = 0; p < kFPieces; ++p) {
      const uint64_t pp = ps + (uint64_t)r * ZC_FROUND + 16 * p;  // first position of the piece
      const uint4 vout = funnel16<Q>(p == 0 ? carry : vst[p - 1], vst[p], sbyte);
      const uint32_t xin[4] = {vin[p].x, vin[p].y, vin[p].z, vin[p].w};
      uint32_t xout[4] = {vout.x, vout.y, vout.z, vout.w};
      if (head && pp < W) {
        // out-bytes b[pp - W + i] with pp - W + i < 0 are zero
        const uint64_t z = (uint64_t)W - pp;  // bytes of the piece to clear
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint64_t lo = 4 * d;
          xout[d] = z >= lo + 4 ? 0u : (z > lo ? xout[d] & (~0u << (8 * (z - lo))) : xout[d]);
        }
      }
      const uint32_t V0 = V;
      uint64_t any = 0, all = ~0ull;
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          V = V * 257u + ((xin[d] >> (8 * q)) & 0xFFu) - ((xout[d] >> (8 * q)) & 0xFFu) * pw32;
          const uint64_t b = __ballot(f_hit<NF>(V, K, s_map, s_keys, pw32));
          any |= b;
          all &= b;
        }
      uint64_t need = (open_mask & ~all) | (~open_mask & any);
      if (need_valid) {
        // pieces with positions outside [p_start, p_end): lanes with hits or
        // an open run take the exact path (it closes runs at p_end)
        const uint64_t some = __ballot(pp < p_start || pp + 16 > p_end);
        need = (need & ~some) | (some & (any | open_mask));
      }
      if (__builtin_expect(need != 0, 0)) {
        if ((need >> lane) & 1) {
          uint32_t Vx = V0;
#pragma unroll
          for (int d = 0; d < 4; ++d)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              Vx = Vx * 257u + ((xin[d] >> (8 * q)) & 0xFFu) - ((xout[d] >> (8 * q)) & 0xFFu) * pw32;
              const uint64_t pos = pp + 4 * d + q;
              const bool h = f_hit<NF>(Vx, K, s_map, s_keys, pw32) && pos >= p_start && pos < p_end;
              const uint32_t rel = (uint32_t)(pos - wtbase);
              if (h && !open) {
                open = true;
                rstart = rel;
              } else if (!h && open) {
                open = false;
                if (nrun < RS) put_run(rs, re, nrun, rstart, rel);
                else ovf = true;
                ++nrun;
              }
            }
        }
        open_mask = __ballot(open);
      }
    }
    }
    carry = vst[kFPieces - 1];

    if (r == kFRounds - 1) {
      // wave-tile end: close runs at span ends, merge across lanes, write
      if (open) {
        if (nrun < RS) put_run(rs, re, nrun, rstart, (lane + 1) * ZC_FLSPAN);
        else ovf = true;
        ++nrun;
        open = false;
      }
      const uint64_t wt = wtbase / ZC_FWT;
      if (__ballot(ovf) != 0) {
        if (lane == 0) {
          wt_off[wt] = 0;
          wt_cnt[wt] = ZC_FWT_OVERFLOW;
        }
        continue;
      }
      uint32_t tot;
      const uint32_t excl = wave_excl_scan(nrun, lane, &tot);
      if (tot == 0) {
        if (lane == 0) {
          wt_off[wt] = 0;
          wt_cnt[wt] = 0;
        }
        continue;
      }
#pragma unroll
      for (int k = 0; k < RS; ++k)
        if ((uint32_t)k < nrun) {
          lrs[excl + k] = rs[k];
          lre[excl + k] = re[k];
        }
      wait_lgkmcnt<0>();
      __builtin_amdgcn_wave_barrier();
      // entry i is a head unless it starts where entry i - 1 ends; lane owns
      // entries lane + 64 j (tot <= 64 RS)
      uint64_t hmk[RS];
      uint32_t nheads = 0;
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const uint32_t i = lane + 64u * j;
        const bool h = i < tot && (i == 0 || lre[i - 1] != lrs[i]);
        hmk[j] = __ballot(h);
        nheads += (uint32_t)__popcll(hmk[j]);
      }
      uint64_t base = 0;
      if (lane == 0) base = atomicAdd(&counters[CNT_RUNS], (unsigned long long)nheads);
      base = __shfl(base, 0, 64);
      if (lane == 0) {
        wt_off[wt] = base;
        wt_cnt[wt] = nheads;
        if (base + nheads > runs_cap) atomicOr(&counters[CNT_FOVF], 1ull);
      }
      if (base + nheads > runs_cap) continue;
      // group index of entry i = heads at or before i, minus one
      uint32_t before = 0;
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const uint32_t i = lane + 64u * j;
        const bool h = (hmk[j] >> lane) & 1;
        const uint32_t g = before + lane_prefix(hmk[j]) + (h ? 1u : 0u) - 1u;
        if (i < tot) {
          if (h) runs[base + g].start = wtbase + lrs[i];
          if (i + 1 == tot || lre[i] != lrs[i + 1]) runs[base + g].end = wtbase + lre[i];
        }
        before += (uint32_t)__popcll(hmk[j]);
      }
    }
  }
}

// Bloom filter of a key set (thread per key)
__global__ void zc_bloom_add_kernel(uint32_t* __restrict__ bloom, uint32_t bits, const uint64_t* __restrict__ keys,
                                    uint32_t n) {
  ZC_URGENT();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t b = bloom_block(keys[i], bits), g = bloom_seed(keys[i]);
  atomicOr(&bloom[2 * b], bloom_lo(g));
  atomicOr(&bloom[2 * b + 1], bloom_hi(g));
  const uint32_t f = bloom_pf(keys[i]);
  atomicOr(&bloom[(2u << bits) + (f >> 5)], 1u << (f & 31));
}

// 64-bit key sets of the screen's run filter: open addressing (empty = 0),
// and a short sorted list
__device__ __forceinline__ bool key64_in(uint64_t k, const uint64_t* __restrict__ set, uint32_t sbits, int zero_key,
                                         const uint64_t* __restrict__ list, uint32_t nl) {
  if (k == 0) return zero_key != 0;
  if (set) {
    const uint32_t mask = (1u << sbits) - 1;
    for (uint32_t h = (uint32_t)((k * kGolden) >> (64 - sbits));; h = (h + 1) & mask) {
      const uint64_t v = set[h];
      if (v == k) return true;
      if (v == 0) break;
    }
  }
  uint32_t lo = 0, len = nl;
  while (len > 0) {
    const uint32_t half = len >> 1;
    if (list[lo + half] < k) {
      lo += half + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  return lo < nl && list[lo] == k;
}

constexpr uint64_t kKey64FilterMax = 64;  // longer runs are left to the walk

// thread per screen run: a short run keeps only [first, last] of the
// positions whose 64-bit window key (257^W + the window's accumulator) is
// in the sets; none: the run becomes empty
// Bloom-mode runs of at most kKey64FilterMax positions, trimmed to the
// positions whose exact 64-bit key is in the set (the runs' first and last
// hits; none: the run is emptied).  Runs of up to kKey64LaneMax positions
// take a lane each (zc_key64_filter_kernel: most runs are a false Bloom hit
// or two); longer ones a wave each, one position per lane
// (zc_key64_filter_wave_kernel), so no lane walks 64 positions in turn.
constexpr uint64_t kKey64LaneMax = 8;
__device__ __forceinline__ void key64_trim(Run* __restrict__ runs, uint64_t i, const Run& r, uint64_t first,
                                           uint64_t last) {
  if (first == ~0ull) {
    runs[i].end = r.start;
  } else {
    runs[i].start = first;
    runs[i].end = last + 1;
  }
}
__global__ void __launch_bounds__(64) zc_key64_filter_kernel(const uint8_t* __restrict__ data,
                                                             const uint64_t* __restrict__ blk, uint32_t W, uint64_t pw,
                                                             Run* __restrict__ runs, uint64_t nruns,
                                                             const uint64_t* __restrict__ set, uint32_t sbits,
                                                             int zero_key, const uint64_t* __restrict__ list,
                                                             uint32_t nl) {
  ZC_URGENT();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nruns) return;
  const Run r = runs[i];
  if (r.end - r.start > kKey64LaneMax) return;
  uint64_t first = ~0ull, last = 0;
  for (uint64_t p = r.start; p < r.end; ++p)
    if (key64_in(pw + rk_acc(data, blk, p + 1 - W, p + 1), set, sbits, zero_key, list, nl)) {
      if (first == ~0ull) first = p;
      last = p;
    }
  key64_trim(runs, i, r, first, last);
}
__global__ void __launch_bounds__(256) zc_key64_filter_wave_kernel(const uint8_t* __restrict__ data,
                                                                  const uint64_t* __restrict__ blk, uint32_t W,
                                                                  uint64_t pw, Run* __restrict__ runs, uint64_t nruns,
                                                                  const uint64_t* __restrict__ set, uint32_t sbits,
                                                                  int zero_key, const uint64_t* __restrict__ list,
                                                                  uint32_t nl) {
  ZC_URGENT();
  static_assert(kKey64FilterMax <= 64, "a lane per position");
  // a bounded grid of waves strides over the runs (most are short and left to
  // zc_key64_filter_kernel: a wave skips them after one load)
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < nruns; i += nw) {
    const Run r = runs[i];
    if (r.end - r.start <= kKey64LaneMax || r.end - r.start > kKey64FilterMax) continue;
    const uint64_t p = r.start + lane;
    bool hit = false;
    if (p < r.end) hit = key64_in(pw + rk_acc(data, blk, p + 1 - W, p + 1), set, sbits, zero_key, list, nl);
    const uint64_t m = __ballot(hit);
    if (lane == 0)
      key64_trim(runs, i, r, m ? r.start + (uint64_t)__builtin_ctzll(m) : ~0ull,
                 m ? r.start + 63 - (uint64_t)__builtin_clzll(m) : 0);
  }
}

// ---------------------------------------------------------------------------
// zc_sha1: thread per range (FIPS 180-4)
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

__device__ __forceinline__ void sha1_block(uint32_t* st, const uint32_t* wbe) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = wbe[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
#pragma unroll
  for (int t = 0; t < 80; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      // gfx950's three-input boolean op: bit i of the table is the result for
      // (src0, src1, src2) = bits (2, 1, 0) of i, i.e. src0/1/2 weigh 0xF0/0xCC/0xAA
      // (0x96 = x ^ y ^ z, 0xE8 = majority, 0xCA = choose): one VALU op where the
      // compiler emits two or three
      wt = rotl32(__builtin_amdgcn_bitop3_b32(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15], 0x96) ^
                      w[t & 15],
                  1);
      w[t & 15] = wt;
    }
    uint32_t f, k;
    if (t < 20) { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA); k = 0x5A827999u; }  // b ? c : d (src0 = 0xF0)
    else if (t < 40) { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0x96); k = 0x6ED9EBA1u; }
    else if (t < 60) { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8); k = 0x8F1BBCDCu; }
    else { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0x96); k = 0xCA62C1D6u; }
    uint32_t tmp = rotl32(a, 5) + f + e + k + wt;
    e = d; d = c; c = rotl32(b, 30); b = a; a = tmp;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// SHA-1 of [base, base + L) into out[20 i ..]
// digest i (big-endian, 20 bytes) to out + 20 i as five dword stores (out is
// 4-byte aligned: every digest buffer starts an allocation); the grid kernel's
// out may be pinned host memory, where byte stores would each be a bus write
__device__ __forceinline__ void put_digest(uint8_t* __restrict__ out, uint32_t i, const uint32_t* st) {
  uint32_t* o = reinterpret_cast<uint32_t*>(out + (uint64_t)i * 20);
#pragma unroll
  for (int k = 0; k < 5; ++k) o[k] = __builtin_bswap32(st[k]);
}

__device__ __forceinline__ void sha1_range(const uint8_t* __restrict__ data, uint64_t base, uint32_t L, uint32_t i,
                           uint8_t* __restrict__ out) {
  uint32_t st[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  uint32_t w[16];
  uint32_t full = L / 64;
  if ((base & 15) == 0) {
    // aligned ranges (every grid chunk): 16-byte loads, kAhead blocks in
    // flight while the current one is hashed (one block of SHA-1 is shorter
    // than HBM's latency under load).  Two, not four: 81 VGPRs instead of 146,
    // so two SHA-1 waves fit on a SIMD beside the scan's two
    // (tools/ubench/overlap_bench.hip: alone 2.59 vs 2.72 ms per 8 GiB)
    constexpr uint32_t kAhead = 2;
    const uint4* p = (const uint4*)(data + base);
    uint4 nx[kAhead][4] = {};
#pragma unroll
    for (uint32_t j = 0; j < kAhead; ++j)
      if (j < full) {
#pragma unroll
        for (int k = 0; k < 4; ++k) nx[j][k] = p[4 * j + k];
      }
    for (uint32_t b0 = 0; b0 < full; b0 += kAhead) {
#pragma unroll
      for (uint32_t j = 0; j < kAhead; ++j) {
        if (b0 + j < full) {
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
    }
  } else {
    for (uint32_t blkI = 0; blkI < full; ++blkI) {
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = bswap32(load4_any(data, base + (uint64_t)blkI * 64 + 4 * k));
      sha1_block(st, w);
    }
  }
  // final block(s): remaining bytes, 0x80, zeros, 64-bit big-endian bit length
  uint32_t rem = L - full * 64;
  const uint64_t tb = base + (uint64_t)full * 64;
  uint32_t nfinal = (rem + 9 <= 64) ? 1 : 2;
  for (uint32_t f = 0; f < nfinal; ++f) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      uint32_t v = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t idx = f * 64 + 4 * k + q;  // index within the padded tail
        uint32_t byte;
        if (idx < rem) byte = data[tb + idx];
        else if (idx == rem) byte = 0x80;
        else byte = 0;
        v = (v << 8) | byte;
      }
      w[k] = v;
    }
    if (f == nfinal - 1) {
      uint64_t bits = (uint64_t)L * 8;
      w[14] = (uint32_t)(bits >> 32);
      w[15] = (uint32_t)bits;
    }
    sha1_block(st, w);
  }
  put_digest(out, i, st);
}

__global__ __launch_bounds__(64) void zc_sha1_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ a,
                               const uint32_t* __restrict__ len, uint32_t nr, uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nr) sha1_range(data, a[i], len[i], i, out);
}

// the same for the grid chunks [i W, min((i + 1) W, n)) of an n-byte stream
__global__ __launch_bounds__(64) void zc_sha1_grid_kernel(const uint8_t* __restrict__ data, uint64_t n, uint32_t W, uint32_t nr,
                                    uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nr) return;
  const uint64_t base = (uint64_t)i * W;
  sha1_range(data, base, (uint32_t)std::min<uint64_t>(W, n - base), i, out);
}

// SHA-1 of a 16-byte aligned range whose length is a multiple of 16 (every
// whole grid chunk when W = 0 mod 16): no unaligned or byte-wise path, so the
// kernel holds 2 blocks in flight in few registers -- two of its waves fit on a
// SIMD next to the scan's two (zc_scan_kernel_v128)
__device__ __forceinline__ void sha1_range16(const uint8_t* __restrict__ data, uint64_t base, uint32_t L, uint32_t i,
                                             uint8_t* __restrict__ out) {
  uint32_t st[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  uint32_t w[16];
  const uint32_t full = L / 64;
  const uint4* p = (const uint4*)(data + base);
  constexpr uint32_t kAhead = 2;
  uint4 nx[kAhead][4];
#pragma unroll
  for (uint32_t j = 0; j < kAhead; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) nx[j][k] = j < full ? p[4 * j + k] : make_uint4(0, 0, 0, 0);
  for (uint32_t b0 = 0; b0 < full; b0 += kAhead) {
#pragma unroll
    for (uint32_t j = 0; j < kAhead; ++j) {
      if (b0 + j < full) {
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
  }
  // the final block: the last rem = L mod 64 bytes (0, 16, 32 or 48), 0x80,
  // zeros, the 64-bit big-endian bit length (rem + 9 <= 64: one block)
  const uint32_t rem = L & 63u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint4 v = (uint32_t)(16 * q) < rem ? p[4 * full + q] : make_uint4(0, 0, 0, 0);
    w[4 * q] = bswap32(v.x);
    w[4 * q + 1] = bswap32(v.y);
    w[4 * q + 2] = bswap32(v.z);
    w[4 * q + 3] = bswap32(v.w);
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = (uint32_t)k == rem / 4 ? 0x80000000u : w[k];
  const uint64_t bits = (uint64_t)L * 8;
  w[14] = (uint32_t)(bits >> 32);
  w[15] = (uint32_t)bits;
  sha1_block(st, w);
  put_digest(out, i, st);
}

// the whole grid chunks i < nr, each [i W, (i + 1) W), W = 0 mod 16
__global__ __launch_bounds__(64) void zc_sha1_grid16_kernel(const uint8_t* __restrict__ data, uint32_t W, uint32_t nr,
                                                            uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nr) sha1_range16(data, (uint64_t)i * W, W, i, out);
}

// one range by value (the stream's last, partial grid chunk)
__global__ __launch_bounds__(64) void zc_sha1_one_kernel(const uint8_t* __restrict__ data, uint64_t base, uint32_t L,
                                                         uint32_t i, uint8_t* __restrict__ out) {
  if (threadIdx.x == 0) sha1_range(data, base, L, i, out);
}

// ---------------------------------------------------------------------------
// synthetic streams: byte k = byte (k mod 8) of splitmix64 word floor(k/8)
// (the same recipe as oracle/zc_oracle.cpp zco_fill_splitmix64)
__global__ void zc_fill_kernel(uint8_t* __restrict__ d, uint64_t n, uint64_t seed) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t nw = n / 8;
  for (; i < nw + 1; i += stride) {
    uint64_t z = seed + (i + 1) * kGolden;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    if (i < nw) {
      ((uint64_t*)d)[i] = z;
    } else {
      for (uint64_t k = nw * 8; k < n; ++k) d[k] = (uint8_t)(z >> (8 * (k - nw * 8)));
    }
  }
}

inline unsigned blocks_for(uint64_t items, unsigned per) { return (unsigned)((items + per - 1) / per); }

}  // namespace

uint64_t pow257(uint64_t e) { return pow257_dev(e); }

static int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

hipError_t launch_scan_tiles(const uint8_t* data, uint64_t n, uint64_t tile0, uint64_t ntiles, int32_t anchor_lo,
                             uint64_t* blk, PoolOut po, unsigned long long* counters, hipStream_t s,
                             GridKeysOut gko, hipEvent_t start, hipEvent_t stop) {
  if (!ntiles) return hipSuccess;
  if (gko.key && (!gko.hkey || ((uint64_t)ZC_LSPAN << gko.lshift) > (1ull << ZC_WT_SHIFT))) return hipErrorInvalidValue;
  // the tiles' wave-tiles, a wave each at a time, kScanWgPerCu workgroups per CU
  const uint64_t wt0 = tile0 * (ZC_SCAN_TPB / 64), nwt = ntiles * (ZC_SCAN_TPB / 64);
  const unsigned grid = (unsigned)std::min<uint64_t>((nwt + kScanWaves - 1) / kScanWaves,
                                                     (uint64_t)cu_count() * kScanWgPerCu);
  if (start || stop)
    hipExtLaunchKernelGGL(zc_scan_kernel, dim3(grid), dim3(64 * kScanWaves), 0, s, start, stop, 0, data, n, wt0, nwt,
                          anchor_lo, blk, po, counters, gko);
  else
    hipLaunchKernelGGL(zc_scan_kernel, dim3(grid), dim3(64 * kScanWaves), 0, s, data, n, wt0, nwt, anchor_lo, blk,
                       po, counters, gko);
  return hipGetLastError();
}

hipError_t launch_scan_tail(const uint8_t* data, uint64_t n, int32_t anchor_lo, uint64_t* blk, PoolOut po,
                            unsigned long long* counters, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
  if (n % ZC_STILE) {
    if (start || stop)
      hipExtLaunchKernelGGL(zc_scan_tail_kernel, dim3(ZC_SCAN_TPB / 64), dim3(ZC_WT_BLOCK), 0, s, start, stop, 0, data,
                            n, (uint64_t)(n / ZC_STILE), anchor_lo, blk, po, counters);
    else
      hipLaunchKernelGGL(zc_scan_tail_kernel, dim3(ZC_SCAN_TPB / 64), dim3(ZC_WT_BLOCK), 0, s, data, n, n / ZC_STILE,
                         anchor_lo, blk, po, counters);
  }
  return hipGetLastError();
}

hipError_t launch_scan(const uint8_t* data, uint64_t n, int32_t anchor_lo, uint64_t* blk, PoolOut po,
                       unsigned long long* counters, hipStream_t s) {
  hipError_t e = launch_scan_tiles(data, n, 0, n / ZC_STILE, anchor_lo, blk, po, counters, s);
  if (e != hipSuccess) return e;
  return launch_scan_tail(data, n, anchor_lo, blk, po, counters, s);
}

hipError_t launch_anchor_rescan(const uint8_t* data, uint64_t n, int32_t anchor_lo, const uint32_t* tiles,
                                const uint32_t* sbase, uint32_t ntiles, int pass, uint32_t* base, uint32_t* cnt,
                                uint32_t* srel, uint32_t* sg, hipStream_t s) {
  if (!ntiles) return hipSuccess;
  hipLaunchKernelGGL(zc_anchor_rescan_kernel, dim3(ntiles), dim3(ZC_WT_BLOCK), 0, s, data, n, anchor_lo, tiles, sbase,
                     pass, base, cnt, srel, sg);
  return hipGetLastError();
}





hipError_t launch_epoch_index(const uint8_t* data, uint64_t n, const uint64_t* blk, AnchorView av, uint64_t r_e,
                              uint32_t nconf, uint32_t nsref, uint32_t W, uint64_t pw, const EpochIndex& ix,
                              hipStream_t s, hipEvent_t after_meta) {
  const uint32_t nref = nconf + nsref;
  // fused: the tables are empty and every key is in (the scan wrote them)
  const bool fused = ix.tables_clean && nconf == 0 && nsref && ix.key_from == nsref;
  const EpochClear ec{ix.ckeys, nref && !fused ? 1u << ix.cbits : 0u, ix.tab,
                      ix.tab && !fused ? 2ull << ix.tbits : 0ull, ix.gfilt, ix.tab && !fused ? kGFiltWords : 0u,
                      ix.counters, ix.scnt, ix.h_scnt};
  const FusedInsert fi{fused ? ix.ckeys : nullptr, ix.cbits, ix.tab, ix.tbits, ix.gfilt};
  // enough threads for the grid chunks, and for the clears at a few words each
  const uint64_t words = (uint64_t)ec.cwords + ec.twords + ec.gwords;
  const uint32_t split = (uint32_t)(blocks_for(nsref, 128) * 128);  // the anchor threads' first
  const uint64_t threads =
      std::max<uint64_t>({(uint64_t)split + nsref, std::min<uint64_t>(words / 4, 1u << 20), CNT_LAST});
  hipLaunchKernelGGL(zc_chunk_meta_kernel, dim3(blocks_for(threads, 128)), dim3(128), 0, s, data, n, blk, av, r_e,
                     nsref, split, W, pw, ix.start + nconf, ix.vis + nconf, ix.dead + nconf, ix.key + nconf,
                     ix.cg + nconf, ix.cfp + nconf, ix.anc + nconf, ix.hkey, ix.key_from, ec, fi);
  if (after_meta) {
    const hipError_t e = hipEventRecord(after_meta, s);
    if (e != hipSuccess) return e;
  }
  if (!nref) return hipGetLastError();
  if (!fused)
    hipLaunchKernelGGL(zc_index_insert_kernel, dim3(blocks_for(2ull * nref, 256)), dim3(256), 0, s, ix.key, ix.anc,
                       ix.cg, ix.cfp, nref, ix.ckeys, ix.cbits, ix.tab, ix.tbits, ix.gfilt);
  hipLaunchKernelGGL(zc_class_lead_kernel, dim3(blocks_for(nref, 256)), dim3(256), 0, s, ix.key, ix.anc, nref,
                     ix.ckeys, ix.cbits, ix.cls, ix.ancless, ix.pairs, ix.counters,
                     ShaGrid{ix.gsha, ix.gsha ? ix.n_gsha : 0, n, W}, ix.start);
  // persistent: up to 16 waves per CU (the pair count is on the device)
  const unsigned vblocks = (unsigned)std::min<uint64_t>(blocks_for(nref, 4), (uint64_t)cu_count() * 4);
  hipLaunchKernelGGL(zc_class_verify_kernel, dim3(vblocks), dim3(256), 0, s, data, ix.start, ix.anc, W, ix.cls,
                     ix.ancless, ix.pairs, ix.counters);
  return hipGetLastError();
}

hipError_t launch_class_sha(const uint8_t* gsha, uint64_t n_gsha, uint64_t n, uint32_t W, const EpochIndex& ix,
                            uint32_t nref, hipStream_t s) {
  if (!nref) return hipSuccess;
  hipLaunchKernelGGL(zc_class_sha_kernel, dim3(blocks_for(nref, 256)), dim3(256), 0, s, ShaGrid{gsha, n_gsha, n, W},
                     ix.start, ix.anc, nref, ix.cls, ix.ancless, ix.pairs, ix.counters);
  return hipGetLastError();
}

uint32_t probe_filter_words() { return kGFiltWords; }

// 16-byte stores over the three tables (each a whole number of 16-byte units)
__global__ void zc_tables_clear_kernel(uint4* __restrict__ ckeys, uint64_t cq, uint4* __restrict__ tab, uint64_t tq,
                                       uint4* __restrict__ gfilt, uint64_t gq) {
  // (urgent: it runs beside the grid SHA-1, and the historic registration
  // queued behind it waits for it; at normal priority it took 0.1-1.8 ms there)
  ZC_URGENT();
  const uint64_t gt = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, gs = (uint64_t)gridDim.x * blockDim.x;
  const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u), zero = make_uint4(0u, 0u, 0u, 0u);
  for (uint64_t j = gt; j < cq; j += gs) ckeys[j] = ones;
  for (uint64_t j = gt; j < tq; j += gs) tab[j] = ones;
  for (uint64_t j = gt; j < gq; j += gs) gfilt[j] = zero;
}

hipError_t launch_tables_clear(uint64_t* ckeys, uint64_t cwords, uint64_t* tab, uint64_t twords, uint32_t* gfilt,
                               uint64_t gwords, hipStream_t s) {
  if ((cwords | twords) % 2 || gwords % 4) return hipErrorInvalidValue;
  const uint64_t cq = cwords / 2, tq = twords / 2, gq = gwords / 4;
  if (!(cq + tq + gq)) return hipSuccess;
  const unsigned blocks = (unsigned)std::min<uint64_t>(blocks_for(std::max({cq, tq, gq}), 256), 2048);
  hipLaunchKernelGGL(zc_tables_clear_kernel, dim3(blocks), dim3(256), 0, s, (uint4*)ckeys, cq, (uint4*)tab, tq,
                     (uint4*)gfilt, gq);
  return hipGetLastError();
}

hipError_t launch_ref_meta(const uint8_t* data, const uint64_t* blk, AnchorView av, const uint64_t* starts,
                           uint32_t cnt, uint32_t W, uint64_t pw, uint64_t* key, uint32_t* anc_off, uint32_t* cg,
                           uint64_t* cfp, hipStream_t s) {
  if (!cnt) return hipSuccess;
  const uint32_t split = (uint32_t)(blocks_for(cnt, 128) * 128);
  hipLaunchKernelGGL(zc_ref_meta_kernel, dim3(blocks_for((uint64_t)split + cnt, 128)), dim3(128), 0, s, data, blk, av,
                     starts, cnt, split, W, pw, key, anc_off, cg, cfp);
  return hipGetLastError();
}

__global__ void zc_counters_out_kernel(const unsigned long long* __restrict__ counters,
                                       unsigned long long* __restrict__ h_cnt) {
  ZC_URGENT();
  if (threadIdx.x < CNT_LAST) h_cnt[threadIdx.x] = counters[threadIdx.x];
}

hipError_t launch_counters_out(const unsigned long long* counters, unsigned long long* h_cnt, hipStream_t s) {
  static_assert(CNT_LAST <= 64, "one wave");
  hipLaunchKernelGGL(zc_counters_out_kernel, dim3(1), dim3(64), 0, s, counters, h_cnt);
  return hipGetLastError();
}

hipError_t launch_ref_gather(const uint32_t* src, const uint32_t* dst, uint32_t cnt, const uint64_t* ckey,
                             const uint32_t* canc, const uint32_t* cg, const uint64_t* cfp, uint64_t* key,
                             uint32_t* anc, uint32_t* g, uint64_t* fp, hipStream_t s) {
  if (!cnt) return hipSuccess;
  hipLaunchKernelGGL(zc_ref_gather_kernel, dim3(blocks_for(cnt, 256)), dim3(256), 0, s, src, dst, cnt, ckey, canc,
                     cg, cfp, key, anc, g, fp);
  return hipGetLastError();
}

hipError_t launch_hist_insert(const uint32_t* g, const uint64_t* fp, const uint32_t* anc, uint32_t e0, uint32_t cnt,
                              uint64_t* tab, uint32_t bits, uint32_t* filt, hipStream_t s) {
  if (!cnt) return hipSuccess;
  hipLaunchKernelGGL(zc_hist_insert_kernel, dim3(blocks_for(cnt, 256)), dim3(256), 0, s, g, fp, anc, e0, cnt, tab,
                     bits, filt);
  return hipGetLastError();
}

hipError_t launch_slide_dir(uint32_t* base, const uint32_t* cnt_arr, uint32_t cnt, uint32_t shift, hipStream_t s) {
  if (!cnt || !shift) return hipSuccess;
  hipLaunchKernelGGL(zc_slide_dir_kernel, dim3(blocks_for(cnt, 256)), dim3(256), 0, s, base, cnt_arr, cnt, shift);
  return hipGetLastError();
}


hipError_t launch_probe(const uint8_t* data, AnchorView av, uint64_t wt0, uint64_t nwt, const uint64_t* tab,
                        uint32_t tbits, const uint32_t* gfilt, const uint32_t* anc_off, const uint32_t* cls,
                        const uint64_t* vis, const uint8_t* dead, uint64_t r, uint64_t p_end, uint32_t W,
                        const HistTab& ht, uint64_t r_e, uint32_t nconf, uint32_t nspec, Cand* cand,
                        uint64_t cand_cap, unsigned long long* counters, hipStream_t s) {
  if (!nwt || (!tab && !ht.tab)) return hipSuccess;
  const EpochGrid eg{r_e, nconf, nspec};
  if (!tab) gfilt = nullptr;
  // 4 wave-tiles per wave, 2 slots per lane each (128 anchors per wave-tile
  // before the extra loop; 64 expected at W = 64 KiB): 60 us per 8 GiB vs 68
  // for 2 x 4 and 8 x 2 (the probe is bound by its random reads: ~100 MB of
  // table slots and fingerprint bytes per 8 GiB)
  constexpr int kWT = 4, kSlots = 2;
  const uint64_t waves = (nwt + kWT - 1) / kWT;
  hipLaunchKernelGGL((zc_probe_kernel<kWT, kSlots>), dim3(blocks_for(waves * 64, kProbeTPB)), dim3(kProbeTPB), 0, s,
                     data, av, wt0, nwt, tab, tbits, gfilt, anc_off, cls, vis, dead, r, p_end, W, ht, eg, cand,
                     cand_cap, counters);
  return hipGetLastError();
}

hipError_t launch_verify_pairs(const uint8_t* data, const uint64_t* win_start, const uint64_t* ref_start,
                               uint32_t len, uint32_t npairs, uint8_t* ok, hipStream_t s) {
  if (!npairs) return hipSuccess;
  hipLaunchKernelGGL(zc_verify_kernel, dim3(blocks_for((uint64_t)npairs * 64, 256)), dim3(256), 0, s,
                     data, win_start, ref_start, len, npairs, ok);
  return hipGetLastError();
}

hipError_t launch_range_digest_small(const uint8_t* data, uint64_t n, const uint64_t* blk, const uint64_t* a,
                                     const uint64_t* b, uint32_t nr, uint64_t* out, hipStream_t s) {
  if (!nr) return hipSuccess;
  if (nr > kSmallRanges) return hipErrorInvalidValue;
  SmallRanges rg{};
  for (uint32_t k = 0; k < nr; ++k) {
    rg.a[k] = a[k];
    rg.b[k] = b[k];
  }
  rg.nr = nr;
  hipLaunchKernelGGL(zc_range_digest_small_kernel, dim3(1), dim3(64), 0, s, data, n, blk, rg, out);
  return hipGetLastError();
}

// the results to the host's pinned buffers in one pass (the runtime's
// device-to-host blits ran beside the grid SHA-1 at its priority: 27 us for
// the 32-byte counters, 129 us for 2 MB): the lists, 16-byte stores, then the
// counters (system-scope stores; the host reads them after the stream syncs)
__global__ void zc_cand_out_kernel(const Cand* __restrict__ out0, const Cand* __restrict__ out,
                                   const unsigned long long* __restrict__ hc, Cand* __restrict__ h_out0,
                                   Cand* __restrict__ h_out, unsigned long long* __restrict__ h_hc) {
  ZC_URGENT();
  const uint64_t n0 = hc[HC_EPOCH_OUT], nk = hc[HC_KEPT];
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n0 + nk; i += gs) {
    if (i < nk) h_out[i] = out[i];
    else h_out0[i - nk] = out0[i - nk];
  }
  if (blockIdx.x == 0 && threadIdx.x < HC_LAST) h_hc[threadIdx.x] = hc[threadIdx.x];
}

hipError_t launch_cand_order(const uint8_t* data, const uint64_t* blk, const Cand* cand, uint32_t nc,
                             const uint64_t* hkey, uint64_t pw, uint32_t W, uint64_t n, uint64_t n_gsha,
                             CandOrderBufs b, hipStream_t s) {
  if (!nc) return hipSuccess;
  const uint32_t nblk = (uint32_t)blocks_for(b.nb, kScanBlockItems);
  if (nblk > kScanBlockItems) return hipErrorInvalidValue;  // (nb <= 2^20 by the caller's bucket size)
  hipLaunchKernelGGL(zc_cand_split_kernel, dim3(blocks_for(nc, 256)), dim3(256), 0, s, data, blk, cand, nc, hkey, pw, W,
                     b.bshift, b.rank, b.bcnt, b.out0, b.hc);
  hipLaunchKernelGGL(zc_bucket_sums_kernel, dim3(nblk), dim3(kScanTPB), 0, s, b.bcnt, b.nb, b.bsum);
  hipLaunchKernelGGL(zc_bucket_bscan_kernel, dim3(1), dim3(kScanTPB), 0, s, b.bsum, nblk, b.boff, b.nb, b.hc);
  hipLaunchKernelGGL(zc_bucket_offsets_kernel, dim3(nblk), dim3(kScanTPB), 0, s, b.bcnt, b.nb, b.bsum, b.boff);
  hipLaunchKernelGGL(zc_cand_scatter_kernel, dim3(blocks_for(nc, 256)), dim3(256), 0, s, cand, nc, b.rank, b.boff,
                     b.bshift, n_gsha, W, n, b.out);
  hipLaunchKernelGGL(zc_bucket_sort_kernel, dim3(blocks_for(b.nb, 256)), dim3(256), 0, s, b.out, b.boff, b.nb, b.bcnt,
                     b.hc);
  hipLaunchKernelGGL(zc_cand_out_kernel, dim3(std::min<unsigned>(blocks_for(nc, 256), 1024)), dim3(256), 0, s, b.out0,
                     b.out, b.hc, b.h_out0, b.h_out, b.h_hc);
  return hipGetLastError();
}

hipError_t launch_range_digest(const uint8_t* data, uint64_t n, const uint64_t* blk, const uint64_t* a,
                               const uint64_t* b, uint32_t nr, uint64_t* out, hipStream_t s) {
  if (!nr) return hipSuccess;
  hipLaunchKernelGGL(zc_range_digest_kernel, dim3(blocks_for(nr, 128)), dim3(128), 0, s, data, n, blk, a,
                     b, nr, out);
  return hipGetLastError();
}

hipError_t launch_fscan(const uint8_t* data, uint64_t n, const uint64_t* blk, uint32_t W, uint32_t pw32,
                        uint64_t p_start, uint64_t p_end, uint64_t tile0, uint64_t ntiles, const uint32_t* f32,
                        uint32_t nf, const uint32_t* fbits, const uint32_t* bloom, uint32_t bloom_bits, Run* runs,
                        uint64_t runs_cap, uint64_t* tile_off, uint32_t* tile_cnt, unsigned long long* counters,
                        hipStream_t s) {
  if (!ntiles) return hipSuccess;
  size_t dyn = !bloom && nf > kFLinearMax ? kFBitmapWords * sizeof(uint32_t) : 0;
  hipLaunchKernelGGL(zc_fscan_kernel, dim3((unsigned)ntiles), dim3(ZC_TPB), dyn, s, data, n, blk, W, pw32,
                     p_start, p_end, tile0, f32, nf, fbits, bloom, bloom_bits, runs, runs_cap, tile_off, tile_cnt,
                     counters);
  return hipGetLastError();
}

template <int Q>
static hipError_t launch_fscan_staged_q(int nfk, unsigned grid, hipStream_t s, const uint8_t* data, uint64_t n,
                                        const uint64_t* blk, uint32_t W, uint32_t pw32, uint32_t sbyte,
                                        uint64_t p_start, uint64_t p_end, uint64_t wt0, uint64_t nwt, FKeys K, const uint32_t* fmap,
                                        Run* runs, uint64_t runs_cap, uint64_t* wt_off, uint32_t* wt_cnt,
                                        unsigned long long* counters) {
#define ZC_FS(NF)                                                                                                  \
  hipLaunchKernelGGL((zc_fscan_staged_kernel<Q, NF>), dim3(grid), dim3(kFTPBn<NF>), 0, s, data, n, blk, W, pw32, \
                     sbyte, p_start, p_end, wt0, nwt, K, fmap, runs, runs_cap, wt_off, wt_cnt, counters)
  if (nfk == 1) ZC_FS(1);
  else if (nfk == 64) ZC_FS(64);
  else if (nfk == 65) ZC_FS(65);
  else if (nfk == 4) ZC_FS(4);
  else if (nfk == 16) ZC_FS(16);
  else if (nfk == 32) ZC_FS(32);
  else ZC_FS(0);
#undef ZC_FS
  return hipGetLastError();
}

hipError_t launch_fscan_staged(const uint8_t* data, uint64_t n, const uint64_t* blk, uint32_t W, uint32_t pw32,
                               uint64_t p_start, uint64_t p_end, uint64_t wt0, uint64_t nwt, const uint32_t* keys32,
                               const uint32_t* d_keys32, uint32_t nf, const uint32_t* fbits17, Run* runs,
                               uint64_t runs_cap,
                               uint64_t* wt_off, uint32_t* wt_cnt, unsigned long long* counters, hipStream_t s) {
  if (!nwt) return hipSuccess;
  if (W < 32 || n < 64 || p_end > n || (wt0 + nwt - 1) * ZC_FWT >= p_end || nf == 0) return hipErrorInvalidValue;
  FKeys K;
  const int nfk = nf == 1 ? 1 : nf <= 4 ? 4 : nf <= 16 ? 16 : nf <= kFLdsKeys ? 32 : 0;
  for (int i = 0; i < 16; ++i) K.k[i] = (nfk == 1 || nfk == 4 || nfk == 16 ? keys32[i < (int)nf ? i : 0] : 0u) - pw32;
  K.dkeys = d_keys32;
  K.nk = nfk == 32 ? nf : 0u;
  const uint32_t m = (16u - W % 16u) % 16u;
  const unsigned waves = (unsigned)std::min<uint64_t>(nwt, (uint64_t)cu_count() * (ZC_FTPB / 64));
  const unsigned grid = (waves + ZC_FTPB / 64 - 1) / (ZC_FTPB / 64);
  switch (m >> 2) {
    case 0: return launch_fscan_staged_q<0>(nfk, grid, s, data, n, blk, W, pw32, m & 3, p_start, p_end, wt0, nwt, K, fbits17,
                                            runs, runs_cap, wt_off, wt_cnt, counters);
    case 1: return launch_fscan_staged_q<1>(nfk, grid, s, data, n, blk, W, pw32, m & 3, p_start, p_end, wt0, nwt, K, fbits17,
                                            runs, runs_cap, wt_off, wt_cnt, counters);
    case 2: return launch_fscan_staged_q<2>(nfk, grid, s, data, n, blk, W, pw32, m & 3, p_start, p_end, wt0, nwt, K, fbits17,
                                            runs, runs_cap, wt_off, wt_cnt, counters);
    default: return launch_fscan_staged_q<3>(nfk, grid, s, data, n, blk, W, pw32, m & 3, p_start, p_end, wt0, nwt, K,
                                             fbits17, runs, runs_cap, wt_off, wt_cnt, counters);
  }
}

hipError_t launch_fscan_staged_bloom(const uint8_t* data, uint64_t n, const uint64_t* blk, uint32_t W, uint32_t pw32,
                                     uint64_t p_start, uint64_t p_end, uint64_t wt0, uint64_t nwt,
                                     const uint32_t* bloom, uint32_t bloom_bits, const uint16_t* chk,
                                     uint32_t chk_bits, Run* runs, uint64_t runs_cap, uint64_t* wt_off,
                                     uint32_t* wt_cnt, unsigned long long* counters, hipStream_t s) {
  if (!nwt) return hipSuccess;
  if (W < 32 || n < 64 || p_end > n || (wt0 + nwt - 1) * ZC_FWT >= p_end || !bloom) return hipErrorInvalidValue;
  if (bloom_bits < 1 || bloom_bits > 31 || (chk && (chk_bits < 1 || chk_bits > 31))) return hipErrorInvalidValue;
  FKeys K{};
  K.bloom = bloom;
  K.nk = bloom_bits;
  K.pw64 = pow257_dev(W);
  K.chk = (const uint2*)chk;
  K.cbits = chk_bits;
  const int nfk = chk ? 65 : 64;
  const uint32_t m = (16u - W % 16u) % 16u;
  const unsigned kW64 = (chk ? kFTPBn<65> : kFTPBn<64>) / 64;
  const unsigned waves = (unsigned)std::min<uint64_t>(nwt, (uint64_t)cu_count() * kW64);
  const unsigned grid = (waves + kW64 - 1) / kW64;
  switch (m >> 2) {
    case 0: return launch_fscan_staged_q<0>(nfk, grid, s, data, n, blk, W, pw32, m & 3, p_start, p_end, wt0, nwt, K,
                                            nullptr, runs, runs_cap, wt_off, wt_cnt, counters);
    case 1: return launch_fscan_staged_q<1>(nfk, grid, s, data, n, blk, W, pw32, m & 3, p_start, p_end, wt0, nwt, K,
                                            nullptr, runs, runs_cap, wt_off, wt_cnt, counters);
    case 2: return launch_fscan_staged_q<2>(nfk, grid, s, data, n, blk, W, pw32, m & 3, p_start, p_end, wt0, nwt, K,
                                            nullptr, runs, runs_cap, wt_off, wt_cnt, counters);
    default: return launch_fscan_staged_q<3>(nfk, grid, s, data, n, blk, W, pw32, m & 3, p_start, p_end, wt0, nwt, K,
                                             nullptr, runs, runs_cap, wt_off, wt_cnt, counters);
  }
}

hipError_t launch_bloom_add(uint32_t* bloom, uint32_t bits, const uint64_t* keys, uint32_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(zc_bloom_add_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, bloom, bits, keys, n);
  return hipGetLastError();
}

// the check table of a key set (thread per key): the key's check word into
// the first empty slot from its bucket on (CAS on the slot's 32-bit word);
// present already, or the table's end reached: done (the latter flagged)
__global__ void zc_chk_add_kernel(uint16_t* __restrict__ chk, uint32_t bits, const uint64_t* __restrict__ keys,
                                  uint32_t n, unsigned int* __restrict__ ovf) {
  ZC_URGENT();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t c = chk_word(keys[i]);
  const uint64_t nslots = ((1ull << bits) + kChkPad - 1) * 4;  // the last bucket stays empty
  for (uint64_t sl = (uint64_t)chk_bucket(keys[i], bits) * 4; sl < nslots; ++sl) {
    unsigned int* w = (unsigned int*)(chk + (sl & ~1ull));
    const uint32_t sh = (uint32_t)(sl & 1) * 16;
    unsigned int old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      const uint32_t cur = (old >> sh) & 0xFFFFu;
      if (cur == c) return;
      if (cur != 0) break;
      const unsigned int want = old | (c << sh);
      if (__hip_atomic_compare_exchange_strong(w, &old, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT))
        return;
    }
  }
  atomicOr(ovf, 1u);
}

hipError_t launch_chk_add(uint16_t* chk, uint32_t bits, const uint64_t* keys, uint32_t n, unsigned int* ovf,
                          hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(zc_chk_add_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, chk, bits, keys, n, ovf);
  return hipGetLastError();
}

hipError_t launch_key64_filter(const uint8_t* data, const uint64_t* blk, uint32_t W, uint64_t pw, Run* runs,
                               uint64_t nruns, const uint64_t* set, uint32_t sbits, int zero_key,
                               const uint64_t* list, uint32_t nl, hipStream_t s) {
  if (!nruns) return hipSuccess;
  // a launch's work-items must stay below 2^32: 64-thread blocks, one lane per run
  if (nruns >= (1ull << 32) - 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(zc_key64_filter_kernel, dim3(blocks_for(nruns, 64)), dim3(64), 0, s, data, blk, W, pw, runs,
                     nruns, set, sbits, zero_key, list, nl);
  // one wave per run, at most 4096 workgroups of 4 waves striding over them
  const uint64_t wblocks = std::min<uint64_t>((nruns + 3) / 4, 4096);
  hipLaunchKernelGGL(zc_key64_filter_wave_kernel, dim3((unsigned)wblocks), dim3(256), 0, s, data, blk, W, pw, runs,
                     nruns, set, sbits, zero_key, list, nl);
  return hipGetLastError();
}

hipError_t launch_sha1_grid(const uint8_t* data, uint64_t n, uint32_t W, uint32_t nr, uint8_t* out20,
                            hipStream_t s) {
  if (!nr || !W || (uint64_t)(nr - 1) * W >= n) return nr ? hipErrorInvalidValue : hipSuccess;
  if (W % 16 || ((uintptr_t)data & 15)) {
    hipLaunchKernelGGL(zc_sha1_grid_kernel, dim3(blocks_for(nr, 64)), dim3(64), 0, s, data, n, W, nr, out20);
    return hipGetLastError();
  }
  // whole chunks on the lean aligned kernel, a partial last one by itself
  const uint32_t whole = (uint32_t)std::min<uint64_t>(nr, n / W);
  if (whole)
    hipLaunchKernelGGL(zc_sha1_grid16_kernel, dim3(blocks_for(whole, 64)), dim3(64), 0, s, data, W, whole, out20);
  if (whole < nr)
    hipLaunchKernelGGL(zc_sha1_one_kernel, dim3(1), dim3(64), 0, s, data, (uint64_t)whole * W,
                       (uint32_t)(n - (uint64_t)whole * W), whole, out20);
  return hipGetLastError();
}

hipError_t launch_sha1(const uint8_t* data, const uint64_t* a, const uint32_t* len, uint32_t nr,
                       uint8_t* out20, hipStream_t s) {
  if (!nr) return hipSuccess;
  hipLaunchKernelGGL(zc_sha1_kernel, dim3(blocks_for(nr, 64)), dim3(64), 0, s, data, a, len, nr, out20);
  return hipGetLastError();
}

hipError_t launch_fill_splitmix64(uint8_t* data, uint64_t n, uint64_t seed, hipStream_t s) {
  if (!n) return hipSuccess;
  uint64_t nw = n / 8 + 1;
  unsigned blocks = (unsigned)(nw / 256 + 1 < 16384 ? nw / 256 + 1 : 16384);
  hipLaunchKernelGGL(zc_fill_kernel, dim3(blocks), dim3(256), 0, s, data, n, seed);
  return hipGetLastError();
}

}  // namespace zc
