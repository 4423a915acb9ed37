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
// zc_scan: 512-lane persistent workgroups, lane span 4 KiB (2 MiB tiles),
// per-wave LDS rings of ZC_RING slots of 128-byte rounds
constexpr int ZC_SCAN_TPB = 512;
constexpr int ZC_LSPAN = 4096;
constexpr uint64_t ZC_STILE = (uint64_t)ZC_LSPAN * ZC_SCAN_TPB;
constexpr int ZC_ROUND = 128;
constexpr int ZC_RING = 2;
constexpr int ZC_WLIST = 144;                                // per-wave LDS list of pieces with anchors
constexpr int ZC_ANC_SLOTS = 16;                             // anchor slots per lane span
// zc_fscan: lane span 1 KiB, 256 KiB per workgroup
constexpr uint64_t ZC_TILE = (uint64_t)ZC_SPAN * ZC_TPB;
constexpr int ZC_RUN_SLOTS = 4;                              // LDS screen-run slots per lane

// Content anchors.  gear(q) = sum_{j<32} b[q-j] * 2^j (mod 2^32); q is an
// anchor iff (int32)gear(q) >= anchor_lo, i.e. gear in [anchor_lo, 0x7FFFFFFF]:
// 1 position in rate_inv for random bytes (rate_inv = 2^32 / (2^31 - anchor_lo),
// chosen per stream from W so a W-byte chunk holds ~16 anchors), never inside a
// run of one repeated byte (gear 0 or -c).  A chunk's anchor is its first one
// at offset >= ZC_ANCHOR_MIN_OFF; the table key is the gear value, confirmed
// by a 64-bit fingerprint of the 64 bytes ending at the anchor.
constexpr uint32_t ZC_ANCHOR_MIN_OFF = 63;
constexpr uint32_t ZC_NO_ANCHOR = 0xFFFFFFFFu;

inline int32_t anchor_lo_for(uint32_t W) {
  uint32_t rate_inv = 16;
  while (rate_inv < 4096 && rate_inv * 2 <= W / 16) rate_inv *= 2;
  return (int32_t)(0x80000000u - (uint32_t)(0x100000000ull / rate_inv));
}

// Anchors of the stream, per 4 KiB lane span s: cnt[s] anchors, in position
// order; if cnt[s] <= ZC_ANC_SLOTS they sit in the fixed slots, slot-major
// (slot k of span s at rel/g[k * stride + s], so the first anchors of
// consecutive spans are contiguous), otherwise in the overflow pool at
// ovf_off[s].  Position = s * ZC_LSPAN + rel; g = gear value at that position.
struct AnchorView {
  const uint32_t* cnt;
  const uint16_t* rel;
  const uint32_t* g;
  const uint64_t* ovf_off;
  const uint16_t* orel;
  const uint32_t* og;
  uint64_t stride;  // = anchor_slot_stride(n)
};

// lane spans covered by the scan's tiles (incl. ones past the end of the stream)
__host__ __device__ inline uint64_t anchor_slot_stride(uint64_t n) {
  return (n + ZC_STILE - 1) / ZC_STILE * ZC_SCAN_TPB;
}

struct Run {  // maximal run [start, end) of screen hits of the F scan
  uint64_t start, end;
};

struct Cand {  // anchor-probe candidate: window ending at p may equal chunk ref
  uint64_t p;
  uint32_t ref;
  uint32_t pad;
};

// Counters word layout (uint64 each)
// CNT_POOL: anchors found; CNT_OVERFLOW: lane spans over ZC_ANC_SLOTS anchors;
// CNT_FOVF: screen-run buffer overflow flag
// CNT_ANCLESS: refs without an anchor
enum { CNT_POOL = 0, CNT_OVERFLOW = 1, CNT_CAND = 2, CNT_RUNS = 3, CNT_FOVF = 4, CNT_ANCLESS = 5, CNT_LAST = 8 };

// --- launchers (return hipError_t of the launch) ---------------------------
hipError_t launch_scan(const uint8_t* data, uint64_t n, int32_t anchor_lo, uint64_t* blk, uint16_t* arel,
                       uint32_t* ag, uint32_t* acnt, uint32_t* ovf_list, uint32_t ovf_cap,
                       unsigned long long* counters, hipStream_t s);

// ovf_list holds (span, count) pairs of lane spans with more than
// ZC_ANC_SLOTS anchors; the dense kernel writes ovf_off[span] = offs[i] and
// the span's anchors at that offset of the overflow pool
hipError_t launch_anchor_dense(const uint8_t* data, uint64_t n, int32_t anchor_lo, const uint32_t* spans,
                               uint32_t nspans, const uint64_t* offs, uint64_t* ovf_off, uint16_t* orel,
                               uint32_t* og, hipStream_t s);

// grid chunks i < nchunks of an epoch starting at r_e (start = r_e + i * W)
hipError_t launch_chunk_meta(const uint8_t* data, uint64_t n, const uint64_t* blk, AnchorView av, uint64_t r_e,
                             uint32_t nchunks, uint32_t W, uint64_t pw, uint64_t* start, uint64_t* vis,
                             uint8_t* dead, uint64_t* key, uint32_t* cg, uint64_t* cfp, uint32_t* anc_off,
                             hipStream_t s);

hipError_t launch_anchorless(const uint32_t* anc_off, uint32_t nref, uint32_t* list, uint32_t cap,
                             unsigned long long* counters, hipStream_t s);

hipError_t launch_table_clear(uint64_t* tkeys, uint32_t tsize, hipStream_t s);
hipError_t launch_table_insert(uint64_t* tkeys, uint32_t* tvals, uint32_t tbits,
                               const uint32_t* cg, const uint32_t* anc_off, uint32_t nrefs,
                               hipStream_t s);

hipError_t launch_probe(const uint8_t* data, AnchorView av, uint64_t nspans, const uint64_t* tkeys,
                        const uint32_t* tvals, uint32_t tbits, const uint32_t* anc_off, const uint64_t* cfp, const uint64_t* vis, const uint8_t* dead,
                        uint64_t r, uint64_t n, uint32_t W, Cand* cand, uint64_t cand_cap,
                        unsigned long long* counters, hipStream_t s);

hipError_t launch_verify_pairs(const uint8_t* data, const uint64_t* win_start,
                               const uint64_t* ref_start, uint32_t len, uint32_t npairs,
                               uint8_t* ok, hipStream_t s);

hipError_t launch_range_digest(const uint8_t* data, uint64_t n, const uint64_t* blk,
                               const uint64_t* a, const uint64_t* b, uint32_t nr, uint64_t* out,
                               hipStream_t s);

hipError_t launch_fscan(const uint8_t* data, uint64_t n, const uint64_t* blk, uint32_t W,
                        uint32_t pw32, uint64_t p_start, const uint32_t* f32, uint32_t nf,
                        const uint32_t* fbits, Run* runs, uint64_t runs_cap, uint64_t* tile_off, uint32_t* tile_cnt,
                        unsigned long long* counters, hipStream_t s);

hipError_t launch_sha1(const uint8_t* data, const uint64_t* a, const uint32_t* len, uint32_t nr,
                       uint8_t* out20, hipStream_t s);

hipError_t launch_fill_splitmix64(uint8_t* data, uint64_t n, uint64_t seed, hipStream_t s);

// Host-side helpers shared with the engine
uint64_t pow257(uint64_t e);

}  // namespace zc
