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
constexpr int ZC_SPAN = 1024;
constexpr int ZC_TPB = 256;                                  // 4 waves
constexpr uint64_t ZC_TILE = (uint64_t)ZC_SPAN * ZC_TPB;     // 256 KiB per workgroup
constexpr int ZC_LANE_SLOTS = 8;                             // LDS anchor slots per lane
constexpr int ZC_RUN_SLOTS = 4;                              // LDS screen-run slots per lane

// Content anchors.  gear(q) = sum_{j<32} b[q-j] * 2^j (mod 2^32); q is an
// anchor iff (int32)gear(q) >= ZC_ANCHOR_LO, i.e. gear in [0x7FC00000,
// 0x7FFFFFFF] (1 position in 1024 for random bytes; never inside a run of
// one repeated byte, whose gear is 0 or -c).  The anchor fingerprint is
// (hist(q) << 32) | gear(q) where hist collects bit 31 of the 32 previous
// gear values; it depends on the 63 bytes ending at q, so a chunk's anchor
// offset must be >= ZC_ANCHOR_MIN_OFF.
constexpr int32_t ZC_ANCHOR_LO = 0x7FC00000;
constexpr uint32_t ZC_ANCHOR_MIN_OFF = 63;
constexpr uint32_t ZC_NO_ANCHOR = 0xFFFFFFFFu;

struct Anchor {
  uint64_t pos;
  uint64_t fp;
};

struct Run {  // maximal run [start, end) of screen hits of the F scan
  uint64_t start, end;
};

struct Cand {  // anchor-probe candidate: window ending at p may equal chunk ref
  uint64_t p;
  uint32_t ref;
  uint32_t pad;
};

// Counters word layout (uint64 each)
enum { CNT_POOL = 0, CNT_OVERFLOW = 1, CNT_CAND = 2, CNT_RUNS = 3, CNT_LAST = 8 };

// --- launchers (return hipError_t of the launch) ---------------------------
hipError_t launch_scan(const uint8_t* data, uint64_t n, uint64_t* blk, Anchor* pool,
                       uint64_t pool_cap, uint64_t* tile_off, uint32_t* tile_cnt,
                       unsigned long long* counters, hipStream_t s);

hipError_t launch_chunk_meta(const uint8_t* data, uint64_t n, const uint64_t* blk,
                             const Anchor* pool, const uint64_t* tile_off, const uint32_t* tile_cnt,
                             const uint64_t* starts, uint32_t nchunks, uint32_t W, uint64_t pw,
                             uint64_t* key, uint64_t* fp, uint32_t* anc_off, hipStream_t s);

hipError_t launch_table_clear(uint64_t* tkeys, uint32_t tsize, hipStream_t s);
hipError_t launch_table_insert(uint64_t* tkeys, uint32_t* tvals, uint32_t tbits,
                               const uint64_t* fp, const uint32_t* anc_off, uint32_t nrefs,
                               hipStream_t s);

hipError_t launch_probe(const Anchor* pool, uint64_t npool, const uint64_t* tkeys,
                        const uint32_t* tvals, uint32_t tbits, const uint64_t* chunk_start,
                        const uint32_t* anc_off, const uint64_t* vis, const uint8_t* dead,
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
