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
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zc_device.h"

namespace zc {

namespace {

constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;

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

// Exclusive prefix sum over the 256 threads of a block.
__device__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_tmp, uint32_t& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_tmp[wid] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < ZC_TPB / 64; ++w) {
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
__device__ uint64_t rk_acc(const uint8_t* __restrict__ data, const uint64_t* __restrict__ blk,
                           uint64_t a, uint64_t b) {
  uint64_t acc = 0;
  uint64_t a_up = (a + ZC_SPAN - 1) / ZC_SPAN * ZC_SPAN;
  if (a_up >= b) {
    for (uint64_t i = a; i < b; ++i) acc = acc * 257u + data[i];
    return acc;
  }
  for (uint64_t i = a; i < a_up; ++i) acc = acc * 257u + data[i];
  uint64_t b_dn = b / ZC_SPAN * ZC_SPAN;
  const uint64_t m = span_mul();
  for (uint64_t k = a_up / ZC_SPAN; k < b_dn / ZC_SPAN; ++k) acc = acc * m + blk[k];
  for (uint64_t i = b_dn; i < b; ++i) acc = acc * 257u + data[i];
  return acc;
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
// zc_scan
struct ScanLane {
  uint32_t glo, ghi;  // gear hash and its 32-position bit-31 history
  uint32_t hlo, hhi;  // 64-bit Rabin-Karp accumulator of the span so far
};

__device__ __forceinline__ void gear_step(uint32_t b, ScanLane& s) {
  s.ghi = __builtin_amdgcn_alignbit(s.ghi, s.glo, 31);  // (ghi << 1) | (glo >> 31)
  s.glo = (s.glo << 1) + b;
}

__device__ __forceinline__ void digest_step(uint32_t b, ScanLane& s) {
  // acc*257 + b == ((acc << 8) | b) + acc   (mod 2^64)
  uint32_t slo = (s.hlo << 8) | b;
  uint32_t shi = __builtin_amdgcn_alignbit(s.hhi, s.hlo, 24);
  uint64_t h = (((uint64_t)s.hhi << 32) | s.hlo) + (((uint64_t)shi << 32) | slo);
  s.hlo = (uint32_t)h;
  s.hhi = (uint32_t)(h >> 32);
}

struct LaneSlots {
  uint32_t* rel;
  uint32_t* glo;
  uint32_t* ghi;
};

__device__ __forceinline__ void record_anchor(const LaneSlots& sl, uint32_t& cnt, uint64_t span0,
                                              uint32_t rel, uint32_t g, uint32_t gh) {
  if (span0 + rel < ZC_ANCHOR_MIN_OFF) return;  // window would reach before the stream
  if (cnt < ZC_LANE_SLOTS) {
    sl.rel[cnt * ZC_TPB] = rel;
    sl.glo[cnt * ZC_TPB] = g;
    sl.ghi[cnt * ZC_TPB] = gh;
  }
  ++cnt;
}

template <bool DIGEST>
__device__ __forceinline__ void scan_dword(uint32_t x, uint32_t rel, ScanLane& s,
                                           const LaneSlots& sl, uint32_t& cnt, uint64_t span0) {
  uint32_t g[4], gh[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t b = (x >> (8 * k)) & 0xFFu;
    gear_step(b, s);
    if (DIGEST) digest_step(b, s);
    g[k] = s.glo;
    gh[k] = s.ghi;
  }
  bool any = ((int32_t)g[0] >= ZC_ANCHOR_LO) | ((int32_t)g[1] >= ZC_ANCHOR_LO) |
             ((int32_t)g[2] >= ZC_ANCHOR_LO) | ((int32_t)g[3] >= ZC_ANCHOR_LO);
  if (__builtin_expect(any, 0)) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if ((int32_t)g[k] >= ZC_ANCHOR_LO) record_anchor(sl, cnt, span0, rel + k, g[k], gh[k]);
  }
}

// warm the gear with the 64 bytes before the span (virtual zeros before 0)
__device__ __forceinline__ void gear_warm(const uint8_t* __restrict__ data, uint64_t span0, ScanLane& s) {
  if (span0 >= 64) {
    const uint4* w = (const uint4*)(data + span0 - 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint4 v = w[k];
      uint32_t xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) gear_step((xs[j] >> (8 * q)) & 0xFFu, s);
    }
  } else {
    for (uint64_t i = 0; i < span0; ++i) gear_step(data[i], s);
  }
}

__global__ void __launch_bounds__(ZC_TPB) zc_scan_kernel(
    const uint8_t* __restrict__ data, uint64_t n, uint64_t* __restrict__ blk,
    Anchor* __restrict__ pool, uint64_t pool_cap, uint64_t* __restrict__ tile_off,
    uint32_t* __restrict__ tile_cnt, unsigned long long* __restrict__ counters) {
  __shared__ uint32_t s_rel[ZC_LANE_SLOTS * ZC_TPB];
  __shared__ uint32_t s_glo[ZC_LANE_SLOTS * ZC_TPB];
  __shared__ uint32_t s_ghi[ZC_LANE_SLOTS * ZC_TPB];
  __shared__ uint32_t s_tmp[ZC_TPB / 64];
  __shared__ uint64_t s_base;

  const uint32_t tid = threadIdx.x;
  const uint64_t tile = blockIdx.x;
  const uint64_t span0 = tile * ZC_TILE + (uint64_t)tid * ZC_SPAN;
  LaneSlots sl{s_rel + tid, s_glo + tid, s_ghi + tid};
  uint32_t cnt = 0;

  if (span0 < n) {
    ScanLane s{0, 0, 0, 0};
    gear_warm(data, span0, s);
    const uint64_t len = (n - span0 < ZC_SPAN) ? (n - span0) : ZC_SPAN;
    if (len == ZC_SPAN) {
      const uint4* p = (const uint4*)(data + span0);
      uint4 cur[8], nxt[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) cur[k] = p[k];
#pragma unroll 1
      for (int bt = 0; bt < ZC_SPAN / 128; ++bt) {
        if (bt + 1 < ZC_SPAN / 128) {
#pragma unroll
          for (int k = 0; k < 8; ++k) nxt[k] = p[(bt + 1) * 8 + k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t rel = bt * 128 + k * 16;
          scan_dword<true>(cur[k].x, rel + 0, s, sl, cnt, span0);
          scan_dword<true>(cur[k].y, rel + 4, s, sl, cnt, span0);
          scan_dword<true>(cur[k].z, rel + 8, s, sl, cnt, span0);
          scan_dword<true>(cur[k].w, rel + 12, s, sl, cnt, span0);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
      }
    } else {
      // the stream's last, partial span
      for (uint32_t i = 0; i < (uint32_t)len; ++i) {
        uint32_t b = data[span0 + i];
        gear_step(b, s);
        digest_step(b, s);
        if ((int32_t)s.glo >= ZC_ANCHOR_LO) record_anchor(sl, cnt, span0, i, s.glo, s.ghi);
      }
    }
    blk[span0 / ZC_SPAN] = ((uint64_t)s.hhi << 32) | s.hlo;
  }

  // ordered compaction of the tile's anchors (lane order, then position)
  uint32_t total;
  uint32_t off = block_excl_scan(cnt, s_tmp, total);
  if (tid == 0) {
    uint64_t base = total ? atomicAdd(&counters[CNT_POOL], (unsigned long long)total) : 0;
    if (base + total > pool_cap) atomicOr(&counters[CNT_OVERFLOW], 1ull);
    tile_off[tile] = base;
    tile_cnt[tile] = total;
    s_base = base;
  }
  __syncthreads();
  const uint64_t base = s_base;
  if (cnt == 0 || base + total > pool_cap) return;
  Anchor* dst = pool + base + off;
  if (cnt <= ZC_LANE_SLOTS) {
    for (uint32_t i = 0; i < cnt; ++i) {
      uint32_t r = sl.rel[i * ZC_TPB];
      dst[i].pos = span0 + r;
      dst[i].fp = ((uint64_t)sl.ghi[i * ZC_TPB] << 32) | sl.glo[i * ZC_TPB];
    }
  } else {
    // more anchors than LDS slots (never for random data): rescan the span
    ScanLane s{0, 0, 0, 0};
    gear_warm(data, span0, s);
    const uint64_t len = (n - span0 < ZC_SPAN) ? (n - span0) : ZC_SPAN;
    uint32_t w = 0;
    for (uint32_t i = 0; i < (uint32_t)len; ++i) {
      gear_step(data[span0 + i], s);
      if ((int32_t)s.glo >= ZC_ANCHOR_LO && span0 + i >= ZC_ANCHOR_MIN_OFF) {
        dst[w].pos = span0 + i;
        dst[w].fp = ((uint64_t)s.ghi << 32) | s.glo;
        ++w;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// zc_chunk_meta: thread per chunk [start, start+W)
__global__ void zc_chunk_meta_kernel(const uint8_t* __restrict__ data, uint64_t n,
                                     const uint64_t* __restrict__ blk, const Anchor* __restrict__ pool,
                                     const uint64_t* __restrict__ tile_off,
                                     const uint32_t* __restrict__ tile_cnt,
                                     const uint64_t* __restrict__ starts, uint32_t nchunks, uint32_t W,
                                     uint64_t pw, uint64_t* __restrict__ key, uint64_t* __restrict__ fp,
                                     uint32_t* __restrict__ anc_off) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nchunks) return;
  const uint64_t c = starts[i];
  key[i] = pw + rk_acc(data, blk, c, c + W);
  uint32_t off = ZC_NO_ANCHOR;
  uint64_t f = 0;
  if (W > ZC_ANCHOR_MIN_OFF) {
    const uint64_t lo = c + ZC_ANCHOR_MIN_OFF, hi = c + W - 1;  // inclusive
    for (uint64_t t = lo / ZC_TILE; t <= hi / ZC_TILE; ++t) {
      const Anchor* a = pool + tile_off[t];
      uint32_t m = tile_cnt[t];
      uint32_t L = 0, R = m;  // first entry with pos >= lo
      while (L < R) {
        uint32_t mid = (L + R) >> 1;
        if (a[mid].pos < lo) L = mid + 1; else R = mid;
      }
      if (L < m) {
        if (a[L].pos <= hi) {
          off = (uint32_t)(a[L].pos - c);
          f = a[L].fp;
        }
        break;  // anchors of later tiles are beyond this one
      }
    }
  }
  anc_off[i] = off;
  fp[i] = f;
}

// ---------------------------------------------------------------------------
// anchor table: open addressing on the 64-bit fingerprint, duplicates kept
constexpr uint64_t kEmpty = ~0ull;

__device__ __forceinline__ uint64_t table_key(uint64_t fp) { return fp == kEmpty ? kEmpty - 1 : fp; }

__global__ void zc_table_clear_kernel(uint64_t* tkeys, uint32_t tsize) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < tsize) tkeys[i] = kEmpty;
}

__global__ void zc_table_insert_kernel(uint64_t* tkeys, uint32_t* tvals, uint32_t tbits,
                                       const uint64_t* __restrict__ fp,
                                       const uint32_t* __restrict__ anc_off, uint32_t nrefs) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrefs || anc_off[i] == ZC_NO_ANCHOR) return;
  const uint64_t k = table_key(fp[i]);
  const uint32_t mask = (1u << tbits) - 1;
  uint32_t h = (uint32_t)((k * kGolden) >> (64 - tbits));
  for (;;) {
    unsigned long long prev = atomicCAS((unsigned long long*)&tkeys[h], (unsigned long long)kEmpty,
                                        (unsigned long long)k);
    if (prev == kEmpty) {
      tvals[h] = i;
      return;
    }
    h = (h + 1) & mask;
  }
}

// ---------------------------------------------------------------------------
// zc_probe: thread per anchor of the stream
__global__ void zc_probe_kernel(const Anchor* __restrict__ pool, uint64_t npool,
                                const uint64_t* __restrict__ tkeys, const uint32_t* __restrict__ tvals,
                                uint32_t tbits, const uint64_t* __restrict__ chunk_start,
                                const uint32_t* __restrict__ anc_off, const uint64_t* __restrict__ vis,
                                const uint8_t* __restrict__ dead, uint64_t r, uint64_t n, uint32_t W,
                                Cand* __restrict__ cand, uint64_t cand_cap,
                                unsigned long long* __restrict__ counters) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npool) return;
  const Anchor a = pool[i];
  if (a.pos < r + ZC_ANCHOR_MIN_OFF) return;
  const uint64_t k = table_key(a.fp);
  const uint32_t mask = (1u << tbits) - 1;
  uint32_t h = (uint32_t)((k * kGolden) >> (64 - tbits));
  for (;;) {
    uint64_t tk = tkeys[h];
    if (tk == kEmpty) break;
    if (tk == k) {
      uint32_t ref = tvals[h];
      uint64_t o = anc_off[ref];
      if (a.pos >= r + o) {
        uint64_t ws = a.pos - o, p = ws + W - 1;
        if (p < n && p >= vis[ref] && !dead[ref]) {
          unsigned long long slot = atomicAdd(&counters[CNT_CAND], 1ull);
          if (slot < cand_cap) {
            cand[slot].p = p;
            cand[slot].ref = ref;
            cand[slot].pad = 0;
          }
        }
      }
    }
    h = (h + 1) & mask;
  }
}

// ---------------------------------------------------------------------------
// zc_verify: one wave per pair, byte-exact equality of two len-byte ranges
__global__ void __launch_bounds__(256) zc_verify_kernel(const uint8_t* __restrict__ data,
                                                        const uint64_t* __restrict__ win_start,
                                                        const uint64_t* __restrict__ ref_start,
                                                        uint32_t len, uint32_t npairs,
                                                        uint8_t* __restrict__ ok) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (wave >= npairs) return;
  const uint64_t a = win_start[wave], b = ref_start[wave];
  bool diff = false;
  uint32_t i = lane * 16;
  for (; i + 16 <= len; i += 64 * 16) {
    uint4 x, y;
    __builtin_memcpy(&x, data + a + i, 16);
    __builtin_memcpy(&y, data + b + i, 16);
    diff |= (x.x != y.x) | (x.y != y.y) | (x.z != y.z) | (x.w != y.w);
  }
  // ragged tail (len not a multiple of 16)
  uint32_t tail0 = len & ~15u;
  for (uint32_t j = tail0 + lane; j < len; j += 64) diff |= data[a + j] != data[b + j];
  bool any = __any(diff);
  if (lane == 0) ok[wave] = any ? 0 : 1;
}

// ---------------------------------------------------------------------------
// zc_range_digest: RollingHash::digest of [a, b) = 257^(b-a) + acc
__global__ void zc_range_digest_kernel(const uint8_t* __restrict__ data, uint64_t n,
                                       const uint64_t* __restrict__ blk, const uint64_t* __restrict__ a,
                                       const uint64_t* __restrict__ b, uint32_t nr,
                                       uint64_t* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nr) return;
  out[i] = pow257_dev(b[i] - a[i]) + rk_acc(data, blk, a[i], b[i]);
}

// ---------------------------------------------------------------------------
// zc_fscan: exact window hash H(p) mod 2^32 at every p >= p_start, screened
// against the low words of keys without anchors; emits maximal hit runs.
__device__ __forceinline__ bool f_member(uint32_t h, const uint32_t* f32, uint32_t nf,
                                         const uint32_t* s_bits) {
  if (s_bits) return (s_bits[h >> 18] >> ((h >> 13) & 31)) & 1u;  // bit index h >> 13
  bool m = false;
  for (uint32_t k = 0; k < nf; ++k) m |= (f32[k] == h);
  return m;
}

constexpr uint32_t kFLinearMax = 16;
constexpr uint32_t kFBitmapWords = 1u << 14;  // 2^19 bits = 64 KiB, index = h >> 13

__global__ void __launch_bounds__(ZC_TPB) zc_fscan_kernel(
    const uint8_t* __restrict__ data, uint64_t n, const uint64_t* __restrict__ blk, uint32_t W,
    uint32_t pw32, uint64_t p_start, const uint32_t* __restrict__ f32, uint32_t nf,
    const uint32_t* __restrict__ fbits, Run* __restrict__ runs, uint64_t runs_cap,
    uint64_t* __restrict__ tile_off, uint32_t* __restrict__ tile_cnt,
    unsigned long long* __restrict__ counters) {
  extern __shared__ uint32_t s_dyn[];  // bitmap (if used)
  __shared__ uint64_t s_rs[ZC_RUN_SLOTS * ZC_TPB], s_re[ZC_RUN_SLOTS * ZC_TPB];
  __shared__ uint32_t s_tmp[ZC_TPB / 64];
  __shared__ uint64_t s_base;
  __shared__ uint32_t s_keys[kFLinearMax];

  const uint32_t tid = threadIdx.x;
  const uint64_t tile = blockIdx.x;
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
  uint64_t pe = span0 + ZC_SPAN < n ? span0 + ZC_SPAN : n;
  uint32_t cnt = 0;
  uint64_t open = ~0ull;
  auto emit = [&](uint64_t a, uint64_t b) {
    if (cnt < ZC_RUN_SLOTS) {
      s_rs[cnt * ZC_TPB + tid] = a;
      s_re[cnt * ZC_TPB + tid] = b;
    }
    ++cnt;
  };
  if (ps < pe) {
    // window [p-W+1, p] ends at p; V = its accumulator mod 2^32
    uint32_t V = rk_acc32(data, blk, ps + 1 - W, ps + 1);
    uint32_t h = V + pw32;
    if (f_member(h, s_keys, nf, s_bits)) open = ps;
    uint64_t p = ps + 1;
    for (; p + 4 <= pe; p += 4) {
      uint32_t xin = load4_any(data, p), xout = load4_any(data, p - W);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        V = V * 257u + ((xin >> (8 * k)) & 0xFFu) - ((xout >> (8 * k)) & 0xFFu) * pw32;
        bool hit = f_member(V + pw32, s_keys, nf, s_bits);
        if (hit && open == ~0ull) open = p + k;
        if (!hit && open != ~0ull) {
          emit(open, p + k);
          open = ~0ull;
        }
      }
    }
    for (; p < pe; ++p) {
      V = V * 257u + data[p] - (uint32_t)data[p - W] * pw32;
      bool hit = f_member(V + pw32, s_keys, nf, s_bits);
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
      if (base + total > runs_cap) atomicOr(&counters[CNT_OVERFLOW], 2ull);
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
    uint32_t V = rk_acc32(data, blk, ps + 1 - W, ps + 1);
    uint64_t o2 = f_member(V + pw32, s_keys, nf, s_bits) ? ps : ~0ull;
    uint32_t w = 0;
    for (uint64_t p = ps + 1; p < pe; ++p) {
      V = V * 257u + data[p] - (uint32_t)data[p - W] * pw32;
      bool hit = f_member(V + pw32, s_keys, nf, s_bits);
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
    if (base + nheads > runs_cap) atomicOr(&counters[CNT_OVERFLOW], 2ull);
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
// zc_sha1: thread per range (FIPS 180-4)
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

__device__ void sha1_block(uint32_t* st, const uint32_t* wbe) {
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
      wt = rotl32(w[(t - 3) & 15] ^ w[(t - 8) & 15] ^ w[(t - 14) & 15] ^ w[t & 15], 1);
      w[t & 15] = wt;
    }
    uint32_t f, k;
    if (t < 20) { f = (b & c) | (~b & d); k = 0x5A827999u; }
    else if (t < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1u; }
    else if (t < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDCu; }
    else { f = b ^ c ^ d; k = 0xCA62C1D6u; }
    uint32_t tmp = rotl32(a, 5) + f + e + k + wt;
    e = d; d = c; c = rotl32(b, 30); b = a; a = tmp;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__global__ void zc_sha1_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ a,
                               const uint32_t* __restrict__ len, uint32_t nr, uint8_t* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nr) return;
  uint32_t st[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  const uint64_t base = a[i];
  const uint32_t L = len[i];
  uint32_t w[16];
  uint32_t full = L / 64;
  for (uint32_t blkI = 0; blkI < full; ++blkI) {
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = bswap32(load4_any(data, base + (uint64_t)blkI * 64 + 4 * k));
    sha1_block(st, w);
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
  for (int k = 0; k < 5; ++k) {
    uint32_t v = st[k];
    out[(uint64_t)i * 20 + 4 * k + 0] = v >> 24;
    out[(uint64_t)i * 20 + 4 * k + 1] = v >> 16;
    out[(uint64_t)i * 20 + 4 * k + 2] = v >> 8;
    out[(uint64_t)i * 20 + 4 * k + 3] = v;
  }
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

hipError_t launch_scan(const uint8_t* data, uint64_t n, uint64_t* blk, Anchor* pool,
                       uint64_t pool_cap, uint64_t* tile_off, uint32_t* tile_cnt,
                       unsigned long long* counters, hipStream_t s) {
  uint64_t ntiles = (n + ZC_TILE - 1) / ZC_TILE;
  if (!ntiles) return hipSuccess;
  hipLaunchKernelGGL(zc_scan_kernel, dim3((unsigned)ntiles), dim3(ZC_TPB), 0, s, data, n, blk, pool,
                     pool_cap, tile_off, tile_cnt, counters);
  return hipGetLastError();
}

hipError_t launch_chunk_meta(const uint8_t* data, uint64_t n, const uint64_t* blk,
                             const Anchor* pool, const uint64_t* tile_off, const uint32_t* tile_cnt,
                             const uint64_t* starts, uint32_t nchunks, uint32_t W, uint64_t pw,
                             uint64_t* key, uint64_t* fp, uint32_t* anc_off, hipStream_t s) {
  if (!nchunks) return hipSuccess;
  hipLaunchKernelGGL(zc_chunk_meta_kernel, dim3(blocks_for(nchunks, 128)), dim3(128), 0, s, data, n,
                     blk, pool, tile_off, tile_cnt, starts, nchunks, W, pw, key, fp, anc_off);
  return hipGetLastError();
}

hipError_t launch_table_clear(uint64_t* tkeys, uint32_t tsize, hipStream_t s) {
  hipLaunchKernelGGL(zc_table_clear_kernel, dim3(blocks_for(tsize, 256)), dim3(256), 0, s, tkeys, tsize);
  return hipGetLastError();
}

hipError_t launch_table_insert(uint64_t* tkeys, uint32_t* tvals, uint32_t tbits, const uint64_t* fp,
                               const uint32_t* anc_off, uint32_t nrefs, hipStream_t s) {
  if (!nrefs) return hipSuccess;
  hipLaunchKernelGGL(zc_table_insert_kernel, dim3(blocks_for(nrefs, 256)), dim3(256), 0, s, tkeys,
                     tvals, tbits, fp, anc_off, nrefs);
  return hipGetLastError();
}

hipError_t launch_probe(const Anchor* pool, uint64_t npool, const uint64_t* tkeys,
                        const uint32_t* tvals, uint32_t tbits, const uint64_t* chunk_start,
                        const uint32_t* anc_off, const uint64_t* vis, const uint8_t* dead,
                        uint64_t r, uint64_t n, uint32_t W, Cand* cand, uint64_t cand_cap,
                        unsigned long long* counters, hipStream_t s) {
  if (!npool) return hipSuccess;
  hipLaunchKernelGGL(zc_probe_kernel, dim3(blocks_for(npool, 256)), dim3(256), 0, s, pool, npool, tkeys,
                     tvals, tbits, chunk_start, anc_off, vis, dead, r, n, W, cand, cand_cap, counters);
  return hipGetLastError();
}

hipError_t launch_verify_pairs(const uint8_t* data, const uint64_t* win_start, const uint64_t* ref_start,
                               uint32_t len, uint32_t npairs, uint8_t* ok, hipStream_t s) {
  if (!npairs) return hipSuccess;
  hipLaunchKernelGGL(zc_verify_kernel, dim3(blocks_for((uint64_t)npairs * 64, 256)), dim3(256), 0, s,
                     data, win_start, ref_start, len, npairs, ok);
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
                        uint64_t p_start, const uint32_t* f32, uint32_t nf, const uint32_t* fbits,
                        Run* runs, uint64_t runs_cap, uint64_t* tile_off, uint32_t* tile_cnt,
                        unsigned long long* counters, hipStream_t s) {
  uint64_t ntiles = (n + ZC_TILE - 1) / ZC_TILE;
  if (!ntiles) return hipSuccess;
  size_t dyn = nf > kFLinearMax ? kFBitmapWords * sizeof(uint32_t) : 0;
  hipLaunchKernelGGL(zc_fscan_kernel, dim3((unsigned)ntiles), dim3(ZC_TPB), dyn, s, data, n, blk, W, pw32,
                     p_start, f32, nf, fbits, runs, runs_cap, tile_off, tile_cnt, counters);
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
