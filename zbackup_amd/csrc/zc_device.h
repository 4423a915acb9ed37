// zc_device.h -- shared constants and host-side launch entry points of the
// HIP kernels in zc_kernels.hip.  Internal to libzchunk (not the public ABI,
// which is include/zchunk.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zc {

// Stream geometry.  One lane owns a contiguous span of ZC_SPAN bytes; the
// 64-bit Rabin-Karp digest of every span is kept (the "block digests"), so
// the rolling hash of any byte range is a short Horner fold over spans.
constexpr int ZC_SPAN = 1024;                                // digest granularity
constexpr int ZC_TPB = 256;                                  // 4 waves
// zc_scan: lane span 4 KiB, a wave's 64 spans a 256 KiB wave-tile, 2 MiB
// tiles of ZC_SCAN_TPB / 64 wave-tiles (the unit of launch_scan_tiles); each
// wave stages 128-byte rounds through its own one-slot LDS ring, ZC_SCAN_WAVES
// waves per persistent workgroup.  (The *_CFG macros exist for the geometry
// sweeps of tools/ubench/scan_ablate.hip.)
#ifndef ZC_SCAN_TPB_CFG
#define ZC_SCAN_TPB_CFG 512
#endif
#ifndef ZC_LSPAN_CFG
#define ZC_LSPAN_CFG 4096
#endif
#ifndef ZC_ROUND_CFG
#define ZC_ROUND_CFG 128
#endif
#ifndef ZC_WLIST_CFG
#define ZC_WLIST_CFG 144
#endif
constexpr int ZC_SCAN_TPB = ZC_SCAN_TPB_CFG;
constexpr int ZC_LSPAN = ZC_LSPAN_CFG;
constexpr uint64_t ZC_STILE = (uint64_t)ZC_LSPAN * ZC_SCAN_TPB;
constexpr int ZC_ROUND = ZC_ROUND_CFG;
constexpr int ZC_SCAN_WAVES = 4;
constexpr int ZC_WLIST = ZC_WLIST_CFG;                       // per-wave LDS list of pieces with anchors
static_assert(ZC_LSPAN % ZC_SPAN == 0 && ZC_LSPAN / ZC_SPAN % 2 == 0 && ZC_LSPAN <= 4096, "lane span");
static_assert(ZC_ROUND >= 64 && ZC_ROUND <= 256 && ZC_SPAN % ZC_ROUND == 0, "round");
// wave-tile: the 64 lane spans (256 KiB) one scan wave covers per tile;
// wave-tile t holds stream positions [t << ZC_WT_SHIFT, (t + 1) << ZC_WT_SHIFT)
constexpr int ilog2_c(uint64_t v) { return v <= 1 ? 0 : 1 + ilog2_c(v >> 1); }
constexpr int ZC_WT_SHIFT = ilog2_c(64ull * ZC_LSPAN);
static_assert((64ull * ZC_LSPAN) == (1ull << ZC_WT_SHIFT), "wave-tile = 64 lane spans");
// threads of the blocks that process one wave-tile bytewise, a 1 KiB sub-span each
constexpr int ZC_WT_BLOCK = (1 << ZC_WT_SHIFT) / ZC_SPAN;
// zc_fscan: lane span 1 KiB, 256 KiB per workgroup
constexpr uint64_t ZC_TILE = (uint64_t)ZC_SPAN * ZC_TPB;
constexpr int ZC_RUN_SLOTS = 4;                              // LDS screen-run slots per lane
// zc_fscan_staged: one wave per screen wave-tile of 64 lane spans of
// ZC_FLSPAN bytes (512 KiB), in-bytes and out-bytes (p - W) staged through
// LDS in ZC_FROUND-byte rounds; 8 waves per workgroup, persistent
constexpr int ZC_FLSPAN = 8192;
constexpr int ZC_FROUND = 64;
constexpr int ZC_FTPB = 512;
constexpr uint64_t ZC_FWT = 64ull * ZC_FLSPAN;
static_assert(ZC_FWT % ZC_TILE == 0, "screen wave-tiles cover whole zc_fscan tiles");
constexpr uint32_t ZC_FWT_OVERFLOW = 0xFFFFFFFFu;            // wave-tile left for zc_fscan

// Content anchors.  st(q) = sum_{j<16} b[q-2j] * 2^j (mod 2^16), a 16-bit
// gear over the bytes of q's parity (window [q-30, q]); q is an anchor iff
// (int16)st(q) >= anchor_lo, i.e. st in [anchor_lo, 0x7FFF]: 1 position in
// rate_inv for random bytes (rate_inv = 2^16 / (2^15 - anchor_lo), chosen per
// stream from W so a W-byte chunk holds ~16 anchors), never inside a run of
// one repeated byte (st 0 or -c).  Every position is tested, so a window holds
// the anchors of its content at any alignment.  A chunk's anchor is its first
// one at offset >= ZC_ANCHOR_MIN_OFF; the table key is {st(q-1), st(q)} (the
// 32 bytes ending at q; its top 12 bits are fixed by the anchor test, its low
// 20 free), confirmed by a 64-bit fingerprint of the 8 bytes ending at q.
// (Two 16-bit streams instead of one 32-bit gear: the scan advances both with
// one v_pk_mad_u16)
constexpr uint32_t ZC_ANCHOR_MIN_OFF = 63;
constexpr uint32_t ZC_NO_ANCHOR = 0xFFFFFFFFu;

inline uint32_t anchor_rate_inv(uint32_t W) {
  uint32_t rate_inv = 16;
  while (rate_inv < 4096 && rate_inv * 2 <= W / 16) rate_inv *= 2;
  return rate_inv;
}
inline int32_t anchor_lo_for(uint32_t W) { return (int32_t)(0x8000u - 0x10000u / anchor_rate_inv(W)); }

// Anchors of the stream, per wave-tile t: cnt[t] anchors, sorted by position,
// at index base[t] of the pool (rel = position - (t << ZC_WT_SHIFT), g = gear
// value there); base bit 31 set = the entries sit in the side pool (wave-tiles
// whose anchors overflowed their pool share, rescanned exactly).
// The scan gives wave-tile t the pool share [t * wcap, (t + 1) * wcap).
struct AnchorView {
  const uint32_t* base;
  const uint32_t* cnt;
  const uint32_t* rel;
  const uint32_t* g;
  const uint32_t* srel;
  const uint32_t* sg;
};
constexpr uint32_t ZC_SIDE_POOL = 0x80000000u;

// wave-tiles covered by the scan's 2 MiB tiles (incl. ones past the end)
inline uint64_t wave_tiles(uint64_t n) { return (n + ZC_STILE - 1) / ZC_STILE * (ZC_SCAN_TPB / 64); }
// pool share per wave-tile: twice the expected anchor count plus slack
inline uint32_t wave_tile_cap(uint32_t W) { return 2u * ((1u << ZC_WT_SHIFT) / anchor_rate_inv(W)) + 64u; }

// where the scan writes anchors: wave-tile wt's share of the pool starts at
// entry (wt - wt0) * wcap (wt0 = the first wave-tile of the HBM window; the
// directory pointers base/cnt are indexed by absolute wave-tile)
struct PoolOut {
  uint32_t* base;
  uint32_t* cnt;
  uint32_t* rel;
  uint32_t* g;
  uint32_t wcap;
  uint64_t wt0;
};

// The first epoch's grid-chunk keys, written by the scan at each wave-tile's
// end: with W a multiple of the 4 KiB lane span dividing the
// 256 KiB wave-tile, grid chunk i = [i W, (i + 1) W) is 2^lshift whole lane
// spans of one wave, and its key 257^W + the Horner fold of its span digests
// is a reduction over those lanes.  key (device) and hkey (the host's pinned
// copy) take chunk i at index i; null key: not written.
struct GridKeysOut {
  uint64_t* key;
  uint64_t* hkey;
  uint64_t pw;      // 257^W
  uint32_t lshift;  // log2(W / ZC_LSPAN)
};

// Blocked Bloom filter of the exact screen's large key sets (more than the
// LDS holds), over the full 64-bit window keys: 2^bits blocks of two 32-bit
// words (8 bytes, one gather), a key sets three bits in each word
// Past kBloomOneLevelMin keys the LDS first level below passes most positions
// (61 % at 500 K keys, 85 % at 1 M): the screen then gathers every position's
// block from a filter sized for an XCD's L2 (~8 keys per block, 2 MiB at 2 M
// keys) and checks the filter's hits in the check table (chk_* below).
// Measured (1 GiB random, GiB/s, two levels / one level): 300 K 287 / 197,
// 400 K 234 / 194, 500 K 26 / 191 (the two-level false hits overflow the run
// slots), 800 K 117 / 190
constexpr size_t kBloomOneLevelMin = 384u << 10;
inline uint32_t bloom_bits_for(size_t keys) {
  if (keys >= kBloomOneLevelMin) {
    uint32_t b = 18;
    while (b < 24 && ((size_t)8 << b) < keys) ++b;
    return b;
  }
  // a block per two keys up to 512 K keys (300 K keys -> 2 MiB, half an XCD's
  // L2: ~8e-5 false hits per position, screened out on the device by the
  // 64-bit run filter), a block per key beyond (1 M keys -> 8 MiB: ~5e-5).
  // (Two keys per block past 512 K -- 1 M keys in 4 MiB -- let 15x the false
  // hits through, 6e-4 per position: the runs they open cost more than the
  // L2 misses of the larger filter, 22 vs 107 GiB/s)
  uint32_t b = 17;
  while (b < 24 && ((size_t)(keys > (512u << 10) ? 1 : 2) << b) < keys) ++b;
  return b;
}
// The Bloom buffer: 2^bits blocks of two words, then a 2^19-bit first level
// (one bit per key, from the low word of key * golden) that the staged
// screen holds in LDS: positions whose bit is clear skip the block gather
constexpr uint32_t kBloomPfBits = 19;
constexpr uint32_t kBloomPfWords = 1u << (kBloomPfBits - 5);
inline size_t bloom_words(uint32_t bits) { return ((size_t)2 << bits) + kBloomPfWords; }
// (from the LOW word of key * golden, the block from its high word: a first
// level on the block index's own bits let through positions whose block
// then shared bits with a key's -- 15x the false hits at 1 M keys)
__host__ __device__ inline uint32_t bloom_pf(uint64_t key) {
  return (uint32_t)(key * 0x9E3779B97F4A7C15ull) >> (32 - kBloomPfBits);
}
__host__ __device__ inline uint32_t bloom_block(uint64_t key, uint32_t bits) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}
// the six bit positions of a key in its block: 5-bit fields of one 32-bit
// mix of both key words (two VALU ops; the block index and the first level
// come from key * golden)
__host__ __device__ inline uint32_t bloom_seed(uint64_t key) {
  return ((uint32_t)key ^ (uint32_t)(key >> 32)) * 0x85EBCA6Bu;
}
// all six bits of seed g set in block word pair (x, y)?  Shifts by the
// 5-bit fields: the hardware shift takes its amount mod 32, so each field
// costs one shift (and one more to move it down)
__host__ __device__ inline uint32_t bloom_test(uint32_t x, uint32_t y, uint32_t g) {
  const uint32_t tx = (x >> (g & 31u)) & (x >> ((g >> 5) & 31u)) & (x >> ((g >> 10) & 31u));
  const uint32_t ty = (y >> ((g >> 15) & 31u)) & (y >> ((g >> 20) & 31u)) & (y >> ((g >> 25) & 31u));
  return tx & ty & 1u;
}
// The one-level screen's check table: 2^bits buckets of four 16-bit check
// words (8 bytes, one read), then kChkPad buckets.  A key's bucket is the
// high bits of key * golden (its Bloom block's bits, and more); its check
// word the top half of bloom_seed (0 -> 1: 0 marks an empty slot).  A full
// bucket overflows into the next; the pad buckets end every chain (the last
// stays empty).  >= 16 slots per key: a bucket is full ~1e-4 of the time.
constexpr uint32_t kChkPad = 64;
__host__ __device__ inline uint32_t chk_word_of_seed(uint32_t g) {
  const uint32_t c = g >> 16;
  return c ? c : 1u;
}
__host__ __device__ inline uint32_t chk_word(uint64_t key) { return chk_word_of_seed(bloom_seed(key)); }
__host__ __device__ inline uint32_t chk_bucket(uint64_t key, uint32_t bits) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}
// 1: c is in bucket v; 0: it is not and the bucket has an empty slot (so c
// is not in the table); 2: the bucket is full without c (look on)
__host__ __device__ inline uint32_t chk_match(uint2 v, uint32_t c) {
  const uint32_t s0 = v.x & 0xFFFFu, s1 = v.x >> 16, s2 = v.y & 0xFFFFu, s3 = v.y >> 16;
  if (s0 == c || s1 == c || s2 == c || s3 == c) return 1;
  return (s0 == 0 || s1 == 0 || s2 == 0 || s3 == 0) ? 0 : 2;
}
inline uint32_t chk_bits_for(size_t keys) {
  uint32_t b = 10;
  while (((size_t)4 << b) < 16 * keys) ++b;
  return b;
}
__host__ __device__ inline uint32_t bloom_lo(uint32_t g) {
  return (1u << (g & 31u)) | (1u << ((g >> 5) & 31u)) | (1u << ((g >> 10) & 31u));
}
__host__ __device__ inline uint32_t bloom_hi(uint32_t g) {
  return (1u << ((g >> 15) & 31u)) | (1u << ((g >> 20) & 31u)) | (1u << ((g >> 25) & 31u));
}

struct Run {  // maximal run [start, end) of screen hits of the F scan
  uint64_t start, end;
};

struct Cand {  // anchor-probe candidate: window ending at p may equal chunk ref
  uint64_t p;
  uint32_t ref;
  uint32_t pad;  // 0: ref of the epoch, 1: historic entry `ref`
};

// Counters word layout (uint64 each)
// CNT_POOL: anchors found; CNT_OVERFLOW: wave-tiles over their pool share;
// CNT_FOVF: screen-run buffer overflow flag; CNT_ANCLESS: class leaders
// without an anchor; CNT_CLASS: refs that are not the leader of their class
// CNT_PAIRS: equal-key pairs to byte-check; CNT_SPAIRS: pairs of grid chunks
// whose SHA-1 the side stream computes (ZC_FLAG_SHA1), decided by SHA-1 prefix
enum { CNT_POOL = 0, CNT_OVERFLOW = 1, CNT_CAND = 2, CNT_RUNS = 3, CNT_FOVF = 4, CNT_ANCLESS = 5, CNT_CLASS = 6,
       CNT_PAIRS = 7, CNT_SPAIRS = 8, CNT_LAST = 9 };

// --- launchers (return hipError_t of the launch) ---------------------------
hipError_t launch_scan(const uint8_t* data, uint64_t n, int32_t anchor_lo, uint64_t* blk, PoolOut po,
                       unsigned long long* counters, hipStream_t s);
// the same in pieces: full 2 MiB tiles [tile0, tile0 + ntiles), then the
// partial last tile (if any); the pieces may run as the stream arrives
hipError_t launch_scan_tiles(const uint8_t* data, uint64_t n, uint64_t tile0, uint64_t ntiles, int32_t anchor_lo,
                             uint64_t* blk, PoolOut po, unsigned long long* counters, hipStream_t s,
                             GridKeysOut gko = GridKeysOut{nullptr, nullptr, 0, 0}, hipEvent_t start = nullptr,
                             hipEvent_t stop = nullptr);
// the W for which the scan can write the grid keys (GridKeysOut), else 0
inline uint32_t scan_key_lshift_or_none(uint32_t W, bool& ok) {
  ok = W >= (uint32_t)ZC_LSPAN && W % ZC_LSPAN == 0 && ((64u * ZC_LSPAN) % W) == 0;
  uint32_t l = 0;
  while (ok && ((uint32_t)ZC_LSPAN << l) < W) ++l;
  return l;
}
// (start / stop: events the launch itself records at the kernel's start and
// end -- hipExtLaunchKernel -- in place of markers around it: a marker between
// the scan and the next kernel cost ~7 us.  The tail returns whether it launched.)
hipError_t launch_scan_tail(const uint8_t* data, uint64_t n, int32_t anchor_lo, uint64_t* blk, PoolOut po,
                            unsigned long long* counters, hipStream_t s, hipEvent_t start = nullptr,
                            hipEvent_t stop = nullptr);

// exact rescan of the wave-tiles the scan marked overflowed (directory count
// 0xFFFFFFFF): pass 0 sets cnt[tiles[i]] to the exact count; pass 1 writes the
// anchors to the side pool at sbase[i] and points base[] there
hipError_t launch_anchor_rescan(const uint8_t* data, uint64_t n, int32_t anchor_lo, const uint32_t* tiles,
                                const uint32_t* sbase, uint32_t ntiles, int pass, uint32_t* base, uint32_t* cnt,
                                uint32_t* srel, uint32_t* sg, hipStream_t s);

// The device side of an epoch's index, three launches:
//   1. grid chunks i < nsref starting at r_e + i * W (refs nconf + i): start,
//      visibility, key, first anchor {offset, gear, fingerprint}; and every
//      table and counter below cleared;
//   2. per ref: the content-class table (lowest ref per key) and, for refs
//      with an anchor, the anchor table {gear | ref << 32, fingerprint} and
//      its key filter;
//   3. per ref: cls = the lowest ref with an equal key whose bytes are equal
//      (else itself; counters[CNT_CLASS] += refs that are not leaders), and
//      the class leaders without an anchor listed at ancless
//      (counters[CNT_ANCLESS]).  With gsha (ZC_FLAG_SHA1: the grid chunks'
//      SHA-1, 20 bytes per chunk [q W, (q + 1) W), q < n_gsha), pairs of
//      two such grid chunks are not byte-checked: they are counted in
//      counters[CNT_SPAIRS] and decided by launch_class_sha once the SHA-1
//      has been computed.
// Refs [0, nconf) must have start/key/cg/cfp/anc uploaded (vis = 0, dead = 0).
// The class table has 2^cbits >= 2 nref slots, the anchor table 2^tbits
// (2 << tbits words of tab; tab may be null when the stream has no anchors).
struct EpochIndex {
  uint64_t* start;
  uint64_t* vis;
  uint8_t* dead;
  uint64_t* key;
  uint32_t* cg;
  uint64_t* cfp;
  uint32_t* anc;
  uint32_t* cls;
  uint64_t* ckeys;  // class table: 2^cbits slots {key high word | lowest ref}
  uint32_t cbits;
  uint64_t* tab;
  uint32_t tbits;
  uint32_t* gfilt;
  uint32_t* ancless;
  unsigned long long* counters;
  uint2* pairs;  // scratch: nref {ref, leader} pairs for the byte check
  const uint8_t* gsha;  // null: every pair by bytes
  uint64_t n_gsha;
  uint64_t* hkey = nullptr;  // pinned host copy of the grid chunks' keys (key + nconf), or null
  // the scan's counters (2) to hand to the host (pinned h_scnt) and clear, or null
  unsigned long long* scnt = nullptr;
  unsigned long long* h_scnt = nullptr;
  // grid chunks [0, key_from) already have key[] and hkey[] (the scan wrote
  // them: GridKeysOut); the metadata kernel computes the rest
  uint32_t key_from = 0;
  // the class table, anchor table and filter are empty already (cleared at
  // the end of the last stream): with every key in, the metadata kernel also
  // does the index inserts (no separate clear, no zc_index_insert launch)
  bool tables_clean = false;
};
hipError_t launch_epoch_index(const uint8_t* data, uint64_t n, const uint64_t* blk, AnchorView av, uint64_t r_e,
                              uint32_t nconf, uint32_t nsref, uint32_t W, uint64_t pw, const EpochIndex& ix,
                              hipStream_t s,
                              hipEvent_t after_meta = nullptr);
// the SHA-1 pairs of the last launch_epoch_index (counters[CNT_SPAIRS]): key +
// SHA-1-prefix equality (ChunkIndex::findChunk's test, chunk_index.cc:119-143)
// decides the class; gsha must be complete (ordered after the SHA-1 kernel),
// or null: every such pair joins its class (a speculation checked later)
hipError_t launch_class_sha(const uint8_t* gsha, uint64_t n_gsha, uint64_t n, uint32_t W, const EpochIndex& ix,
                            uint32_t nref, hipStream_t s);
uint32_t probe_filter_words();
// the epoch tables emptied (class table and anchor table to all ones, filter
// to zero), at the end of a stream, while the host finishes it
hipError_t launch_tables_clear(uint64_t* ckeys, uint64_t cwords, uint64_t* tab, uint64_t twords, uint32_t* gfilt,
                               uint64_t gwords, hipStream_t s);

// key and first anchor of chunks [starts[i], starts[i] + W) (resident)
hipError_t launch_ref_meta(const uint8_t* data, const uint64_t* blk, AnchorView av, const uint64_t* starts,
                           uint32_t cnt, uint32_t W, uint64_t pw, uint64_t* key, uint32_t* anc_off, uint32_t* cg,
                           uint64_t* cfp, hipStream_t s);
// key, first anchor, gear and fingerprint of entry dst[t] = those of ref src[t]
// (t < cnt): chunks joining the historic index whose metadata an epoch computed
// the batch's counters into the host's pinned copy, by a kernel queued behind
// the batch (a runtime copy there started ~6 us after the last kernel ended)
hipError_t launch_counters_out(const unsigned long long* counters, unsigned long long* h_cnt, hipStream_t s);
hipError_t launch_ref_gather(const uint32_t* src, const uint32_t* dst, uint32_t cnt, const uint64_t* ckey,
                             const uint32_t* canc, const uint32_t* cg, const uint64_t* cfp, uint64_t* key,
                             uint32_t* anc, uint32_t* g, uint64_t* fp, hipStream_t s);
// The historic index: entries whose bytes have left HBM, {key, SHA-1 prefix}
// on the host, {first anchor offset, gear, fingerprint} on the device; those
// with an anchor sit in an anchor table of the epoch table's layout
// (2^bits 16-byte slots) with its own key filter (probe_filter_words words).
struct HistTab {
  const uint64_t* tab;  // null: no historic entry has an anchor
  uint32_t bits;
  const uint32_t* filt;
  const uint32_t* anc;  // first anchor offset per entry
};
// entries [e0, e0 + cnt) of g / fp with an anchor (anc) into the table and its filter
hipError_t launch_hist_insert(const uint32_t* g, const uint64_t* fp, const uint32_t* anc, uint32_t e0, uint32_t cnt,
                              uint64_t* tab, uint32_t bits, uint32_t* filt, hipStream_t s);
// after the window slid by `shift` pool entries: directory entries [0, cnt)
// that point into the main pool are moved down with it
hipError_t launch_slide_dir(uint32_t* base, const uint32_t* cnt_arr, uint32_t cnt, uint32_t shift, hipStream_t s);

// every anchor of wave-tiles [wt0, wt0 + nwt) probes the filter, then the
// table; candidate windows start at >= r (the reset point) and end before p_end
// (the table holds every ref with an anchor; candidates name class leaders, and
// leave out windows that are a grid chunk r_e + j W (j < nspec, ref nconf + j)
// of the candidate's class: the walk takes those at the grid)
// (tab may be null: the historic table alone; ht.tab null: none)
hipError_t launch_probe(const uint8_t* data, AnchorView av, uint64_t wt0, uint64_t nwt, const uint64_t* tab,
                        uint32_t tbits, const uint32_t* gfilt, const uint32_t* anc_off, const uint32_t* cls,
                        const uint64_t* vis, const uint8_t* dead, uint64_t r, uint64_t p_end, uint32_t W,
                        const HistTab& ht, uint64_t r_e, uint32_t nconf, uint32_t nspec, Cand* cand,
                        uint64_t cand_cap, unsigned long long* counters, hipStream_t s);

// The probe's candidates split and ordered on the device (zc_cand_split, a
// three-launch bucket scan, zc_cand_scatter, zc_bucket_sort): epoch
// candidates (pad 0) appended to out0 (count hc[3]); historic ones whose
// window key equals hkey[ref] to out in position order (count hc[1]; pad 1:
// the window is a grid chunk q W, q < n_gsha, whose SHA-1 the side stream
// computes; 2: not), unless hc[2] != 0: a bucket too large to sort on the
// device (the host sorts out by p then).  Buckets are p >> bshift,
// nb = (n >> bshift) + 1 <= 2^20 of them.  Scratch: bcnt (nb, all zero
// between calls: zero it when made), boff (nb + 1), bsum (nb / 1024 + 1),
// rank (nc), hc (4, zero when made; the calls keep it so).  Results land in
// the pinned host buffers h_out0 / h_out / h_hc (no runtime copies).
struct CandOrderBufs {
  uint32_t bshift, nb;
  uint32_t* bcnt;
  uint32_t* boff;
  uint32_t* bsum;
  uint32_t* rank;
  Cand* out0;
  Cand* out;
  unsigned long long* hc;
  // pinned host memory the results are written to (nc entries each, 4 counters)
  Cand* h_out0;
  Cand* h_out;
  unsigned long long* h_hc;
};
hipError_t launch_cand_order(const uint8_t* data, const uint64_t* blk, const Cand* cand, uint32_t nc,
                             const uint64_t* hkey, uint64_t pw, uint32_t W, uint64_t n, uint64_t n_gsha,
                             CandOrderBufs b, hipStream_t s);

hipError_t launch_verify_pairs(const uint8_t* data, const uint64_t* win_start,
                               const uint64_t* ref_start, uint32_t len, uint32_t npairs,
                               uint8_t* ok, hipStream_t s);

// RollingHash digest of each [a[i], b[i]) (device arrays)
hipError_t launch_range_digest(const uint8_t* data, uint64_t n, const uint64_t* blk,
                               const uint64_t* a, const uint64_t* b, uint32_t nr, uint64_t* out,
                               hipStream_t s);
// the same for nr <= 4 ranges given by host arrays (passed by value)
hipError_t launch_range_digest_small(const uint8_t* data, uint64_t n, const uint64_t* blk, const uint64_t* a,
                                     const uint64_t* b, uint32_t nr, uint64_t* out, hipStream_t s);

// exact screen, lane per 1 KiB: zc_fscan tiles [tile0, tile0 + ntiles) of
// ZC_TILE bytes, positions p in [p_start, p_end); runs of tile t at
// runs[tile_off[t] ...], tile_cnt[t] of them (merged inside the tile)
hipError_t launch_fscan(const uint8_t* data, uint64_t n, const uint64_t* blk, uint32_t W,
                        uint32_t pw32, uint64_t p_start, uint64_t p_end, uint64_t tile0, uint64_t ntiles,
                        const uint32_t* f32, uint32_t nf, const uint32_t* fbits, const uint32_t* bloom,
                        uint32_t bloom_bits, Run* runs, uint64_t runs_cap, uint64_t* tile_off, uint32_t* tile_cnt,
                        unsigned long long* counters, hipStream_t s);

// exact screen, staged: screen wave-tiles [wt0, wt0 + nwt) of ZC_FWT bytes,
// each starting before p_end <= n (W >= 32, n >= 64), positions p in
// [p_start, p_end); the nf keys, sorted and distinct, in keys32 (host memory)
// and d_keys32 (device): nf <= 4 compared directly; else the 2^17-bit map
// fbits17 (device, bit (h >> 15)), whose hits are confirmed exactly for
// nf <= 2048 (16 compares, or a binary search of the keys in LDS); wt_cnt[wt]
// = ZC_FWT_OVERFLOW marks a wave-tile whose runs did not fit (to be redone by
// launch_fscan)
hipError_t launch_fscan_staged(const uint8_t* data, uint64_t n, const uint64_t* blk, uint32_t W, uint32_t pw32,
                               uint64_t p_start, uint64_t p_end, uint64_t wt0, uint64_t nwt, const uint32_t* keys32,
                               const uint32_t* d_keys32, uint32_t nf, const uint32_t* fbits17, Run* runs,
                               uint64_t runs_cap, uint64_t* wt_off, uint32_t* wt_cnt, unsigned long long* counters,
                               hipStream_t s);

// the large-key-set screen: nf > 2048 keys go through the Bloom filter
// `bloom` (2^bloom_bits uint2 blocks) of the 64-bit window key, rolled at
// every position.  Two levels (chk null: the LDS first level, then the
// block), its runs then trimmed by key64_filter; or one level: every position
// gathers its block and the filter's hits are checked in the check table
// `chk` (2^chk_bits + kChkPad buckets)
hipError_t launch_fscan_staged_bloom(const uint8_t* data, uint64_t n, const uint64_t* blk, uint32_t W, uint32_t pw32,
                                     uint64_t p_start, uint64_t p_end, uint64_t wt0, uint64_t nwt,
                                     const uint32_t* bloom, uint32_t bloom_bits, const uint16_t* chk,
                                     uint32_t chk_bits, Run* runs, uint64_t runs_cap, uint64_t* wt_off,
                                     uint32_t* wt_cnt, unsigned long long* counters, hipStream_t s);
// add the 64-bit keys[0, n) to a check table (2^bits + kChkPad buckets); a
// key that found no slot before the table's end sets *ovf
hipError_t launch_chk_add(uint16_t* chk, uint32_t bits, const uint64_t* keys, uint32_t n, unsigned int* ovf,
                          hipStream_t s);
// set the bits of the 64-bit keys[0, n) in a Bloom filter
hipError_t launch_bloom_add(uint32_t* bloom, uint32_t bits, const uint64_t* keys, uint32_t n, hipStream_t s);
// Short screen runs (<= 64 positions) are trimmed to the positions whose
// exact 64-bit window key is in the sets (a hash set of 2^sbits slots, empty
// slot = 0, key 0 present iff zero_key; plus nl sorted keys `list`); a run
// with none becomes empty (start = end).  Longer runs are left as they are.
hipError_t launch_key64_filter(const uint8_t* data, const uint64_t* blk, uint32_t W, uint64_t pw, Run* runs,
                               uint64_t nruns, const uint64_t* set, uint32_t sbits, int zero_key,
                               const uint64_t* list, uint32_t nl, hipStream_t s);

hipError_t launch_sha1(const uint8_t* data, const uint64_t* a, const uint32_t* len, uint32_t nr,
                       uint8_t* out20, hipStream_t s);
// SHA-1 (20 bytes each) of the grid chunks [i W, min((i + 1) W, n)) of an n-byte stream,
// i < nr = ceil(n / W)
hipError_t launch_sha1_grid(const uint8_t* data, uint64_t n, uint32_t W, uint32_t nr, uint8_t* out20,
                            hipStream_t s);

hipError_t launch_fill_splitmix64(uint8_t* data, uint64_t n, uint64_t seed, hipStream_t s);

// Host-side helpers shared with the engine
uint64_t pow257(uint64_t e);

// zc_lzo.hip: bundle payload assembly + lzo1x_1 compression (zc_lzo_core.h)
struct LzoScratch;
struct LzoTimes {
  double parse_ms;  // zc_lzo_parse_kernel, summed over the call's batches
  uint64_t blocks;
};
LzoScratch* lzo_scratch_new();
void lzo_scratch_free(LzoScratch* s);
const LzoTimes* lzo_times(const LzoScratch* s);
// d_dst <- d_src[off[i] ..+ size[i]) for i = 0 .. n-1, back to back
hipError_t lzo_gather(LzoScratch* s, const uint8_t* d_src, const uint64_t* off, const uint64_t* size, size_t n,
                      uint8_t* d_dst, hipStream_t st);
// zlib adler32 (from 1) of each range d_base[off[i] ..+ len[i]) -> out (host)
hipError_t lzo_adler32(LzoScratch* s, const uint8_t* d_base, const uint64_t* off, const uint64_t* len, size_t n,
                       uint32_t* out, hipStream_t st);
// payload i = d_payload[pay_off[i] ..+ pay_size[i]) -> framed lzo1x_1 output at
// d_out + out_off[i]; out_size (host) receives the framed sizes
hipError_t lzo_compress(LzoScratch* s, const uint8_t* d_payload, const uint64_t* pay_off, const uint64_t* pay_size,
                        size_t n, uint8_t* d_out, const uint64_t* out_off, uint64_t* out_size, hipStream_t st);

}  // namespace zc
