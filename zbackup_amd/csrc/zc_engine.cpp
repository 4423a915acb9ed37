// zc_engine.cpp -- host side of libzchunk: the C ABI (include/zchunk.h), device
// buffer management and the boundary resolver.
//
// The resolver replays the state machine of /root/reference/backup_creator.cc
// (fill phase, rotate phase, max-size cut, match, finish) over the candidate
// lists the kernels produce, instead of over every byte:
//
//   * Grid chunks.  After a reset at r the reference cuts chunk k =
//     [r+kW, r+(k+1)W) in the iteration whose probe is at p = r+(k+2)W-1
//     (backup_creator.cc:89-93), so chunk k is visible to probes p >= its
//     "vis" time r+(k+2)W-1 (chunk_storage.cc:31-46 adds it synchronously).
//   * Matches.  A probe at p >= r+W-1 matches iff the window [p-W+1, p] has
//     the rolling key and SHA-1 prefix of a visible index entry
//     (chunk_index.cc:119-143).  Candidates come from the anchor probe
//     (windows sharing a content anchor with a chunk, verified byte-exact on
//     the GPU) and from the exact-hash screen (keys without an anchor, and the
//     static index, verified by 64-bit key + bytes or SHA-1).
//   * On a match at m: grid chunks with vis <= m are saved (NEW), the pending
//     bytes [s, m-W+1) are flushed (NEW, or BYTES under 128 bytes:
//     backup_creator.cc:110-145), the window is emitted (DUP) and r = m+1.
//     If r stays on the same grid (r - r_epoch = 0 mod W) the epoch goes on;
//     otherwise a new epoch recomputes the grid chunks from r.
//   * Finish (backup_creator.cc:147-172): the pending bytes plus the ring,
//     as one piece or as a W-byte chunk and the remainder.
//   * Horizons.  The first epoch covers the whole stream.  An epoch started by
//     a grid-shifting match covers probes up to a horizon kHorizon0 bytes
//     ahead; if it reaches the horizon without one, the grid chunks saved by
//     then become confirmed refs and the next epoch resumes at the horizon
//     (same grid, the horizon doubled).  Device work per epoch is bounded by
//     the bytes it covers, so a stream with many grid shifts stays linear.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <exception>
#include <condition_variable>
#include <functional>
#include <iterator>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/zchunk.h"
#include "zc_device.h"

using namespace zc;

namespace {

using Clock = std::chrono::steady_clock;
inline double ms_since(Clock::time_point t) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t).count();
}

struct ZcError {
  int code;
  std::string msg;
};
// a speculative SHA-1 class join proved wrong (Resolver::spec_): redo the
// stream without speculation
struct Respeculate {};

#define HCK(x)                                                                         \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      throw ZcError{ZC_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)};       \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  void ensure(size_t n) {
    if (n <= cap && p) return;
    release();
    size_t want = n ? n : 1;
    hipError_t e = hipMalloc(&p, want * sizeof(T));
    if (e != hipSuccess) {
      p = nullptr;
      throw ZcError{ZC_ERR_NOMEM, std::string("hipMalloc(") + std::to_string(want * sizeof(T)) +
                                      "): " + hipGetErrorString(e)};
    }
    cap = want;
  }
  // grow to at least n elements (doubling), keeping the first `keep`
  void grow_keep(size_t n, size_t keep, hipStream_t s) {
    if (n <= cap && p) return;
    const size_t want = std::max<size_t>(n, cap * 2);
    T* np = nullptr;
    hipError_t e = hipMalloc(&np, want * sizeof(T));
    if (e != hipSuccess)
      throw ZcError{ZC_ERR_NOMEM, std::string("hipMalloc(") + std::to_string(want * sizeof(T)) +
                                      "): " + hipGetErrorString(e)};
    if (keep && p) {
      e = hipMemcpyAsync(np, p, std::min(keep, cap) * sizeof(T), hipMemcpyDeviceToDevice, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e != hipSuccess) {
        (void)hipFree(np);
        throw ZcError{ZC_ERR_HIP, std::string("grow_keep: ") + hipGetErrorString(e)};
      }
    }
    release();
    p = np;
    cap = want;
  }
  size_t bytes() const { return p ? cap * sizeof(T) : 0; }
};

// pinned host memory: device->host copies land here without a bounce
template <class T>
struct HostBuf {
  T* p = nullptr;
  size_t cap = 0;
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  ~HostBuf() { release(); }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  void ensure(size_t n) {
    if (n <= cap && p) return;
    release();
    size_t want = std::max<size_t>(n, 1);
    hipError_t e = hipHostMalloc((void**)&p, want * sizeof(T), hipHostMallocDefault);
    if (e != hipSuccess) {
      p = nullptr;
      throw ZcError{ZC_ERR_NOMEM, std::string("hipHostMalloc(") + std::to_string(want * sizeof(T)) +
                                      "): " + hipGetErrorString(e)};
    }
    cap = want;
  }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
};

// A growable array of trivially copyable records whose capacity beyond its
// size is plain memory the owner may write ahead into (an epoch's grid records
// are written while the device batch runs, and adopted by the walk's resize).
template <class T>
class RecordVec {
 public:
  RecordVec() = default;
  RecordVec(const RecordVec&) = delete;
  RecordVec& operator=(const RecordVec&) = delete;
  ~RecordVec() { free(p_); }
  size_t size() const { return n_; }
  size_t capacity() const { return cap_; }
  bool empty() const { return n_ == 0; }
  T* data() { return p_; }
  const T* data() const { return p_; }
  T& operator[](size_t i) { return p_[i]; }
  const T& operator[](size_t i) const { return p_[i]; }
  void clear() { n_ = 0; }
  void reserve(size_t c) {
    if (c > cap_) grow(c);
  }
  void resize(size_t n) {  // new elements keep whatever the memory holds
    if (n > cap_) grow(std::max(n, 2 * cap_));
    n_ = n;
  }
  void push_back(const T& v) {
    if (n_ == cap_) grow(std::max<size_t>(64, 2 * cap_));
    p_[n_++] = v;
  }
  void erase_front(size_t k) {  // drop the first k elements
    k = std::min(k, n_);
    if (k < n_) memmove(p_, p_ + k, (n_ - k) * sizeof(T));
    n_ -= k;
  }

 private:
  void grow(size_t c) {
    T* q = (T*)realloc(p_, c * sizeof(T));
    if (!q) throw std::bad_alloc();
    p_ = q;
    cap_ = c;
  }
  T* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
};

struct StaticEntry {
  uint64_t key;
  uint8_t sha[16];
  uint8_t seeded;  // 1: zc_seed_index; 0: added by one of this context's streams
};

constexpr uint64_t kInf = ~0ull;
constexpr size_t kFeedChunk = 8u << 20;
constexpr size_t kFBatchMax = 1u << 20;
constexpr uint64_t kHostSegment = 64ull << 20;  // zc_chunk_host copy/scan pipeline granularity
constexpr uint64_t kHorizon0 = 256ull << 10;    // first horizon of an epoch after a grid shift (>= 64 W)

// an allocator whose value construction is default-initialisation: growing a
// vector of plain records does not zero memory that is written right after
// (the record writes are the host's share of a stream: ~5 MB per 8 GiB)
template <class T>
struct DefaultInit : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = DefaultInit<U>;
  };
  DefaultInit() = default;
  template <class U>
  DefaultInit(const DefaultInit<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept {
    ::new ((void*)p) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new ((void*)p) U(std::forward<A>(a)...);
  }
};

// The record writes of long grid runs (a stream's records are ~40 bytes each,
// 131,072 per 8 GiB: one core writes them at its store bandwidth) are split
// over the spinning team below.
static_assert(sizeof(zc_record) == 40 && offsetof(zc_record, size) == 8 && offsetof(zc_record, kind) == 12 &&
                  offsetof(zc_record, rolling) == 16 && offsetof(zc_record, sha1) == 24,
              "the streamed record writes assume this layout");

// Seven helper threads for a short job that follows a wait: arm() wakes them
// before the wait (a sleeping thread's wake-up costs more than the job
// itself: the records' SHA-1 fill took 0.4-1.0 ms on the host pool against
// 0.2 ms on one thread), they spin until run() hands them their parts (or
// until the deadline passes, then sleep again).
class SpinTeam {
 public:
  static SpinTeam& get() {
    static std::mutex mk;
    static SpinTeam* team = nullptr;
    static pid_t owner = 0;
    std::lock_guard<std::mutex> lk(mk);
    if (!team || owner != getpid()) {
      team = new SpinTeam;
      owner = getpid();
      live_.store(team, std::memory_order_release);
    }
    return *team;
  }
  // disarm() on the team if this process has one (none is made for it)
  static void disarm_any() {
    SpinTeam* t = live_.load(std::memory_order_acquire);
    if (t) t->disarm();
  }
  // the helpers spin for at most `ms` from now
  void arm(double ms = 8.0) {
    deadline_.store(now_ns() + (int64_t)(ms * 1e6), std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(m_);
      ++wake_;
    }
    cv_.notify_all();
  }
  // the helpers stop spinning now (the jobs they were armed for are done):
  // they do not compete with the caller's host work until the next arm()
  void disarm() { deadline_.store(0, std::memory_order_relaxed); }
  // f(begin, end) over [0, n) in kParts parts; the helpers that are not
  // spinning (not armed, or past the deadline) are not waited for: their
  // parts run on this thread
  int run(size_t n, const std::function<void(size_t, size_t)>& f) {
    std::lock_guard<std::mutex> one(run_);
    job_ = &f;
    n_ = n;
    // done_ is cleared before any part can be claimed: a helper that claims a
    // part of this job (the moment its claim word is reset) counts it after
    // the clear, never into the previous job's count
    done_.store(0, std::memory_order_relaxed);
    for (auto& c : claim_) c.store(0, std::memory_order_release);  // (job_, n_, done_ published with it)
    seq_.fetch_add(1, std::memory_order_release);
    int mine = 0;
    for (int k = 0; k < kParts; ++k)  // claim every part nobody took yet, from the last
      if (claim_[kParts - 1 - k].exchange(1, std::memory_order_acq_rel) == 0) {
        part(kParts - 1 - k);
        ++mine;
      }
    while (done_.load(std::memory_order_acquire) + mine < kParts) _mm_pause();
    job_ = nullptr;
    return mine;  // parts done here (kParts: no helper was spinning)
  }

 private:
  static constexpr int kHelpers = 7, kParts = kHelpers + 1;
  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  SpinTeam() {
    for (int w = 0; w < kHelpers; ++w) th_.emplace_back([this, w] { loop(w); });
    for (auto& t : th_) t.detach();  // process lifetime
  }
  void part(int k) {
    const size_t a = n_ * k / kParts, b = n_ * (k + 1) / kParts;
    if (b > a) (*job_)(a, b);
  }
  void loop(int w) {
    uint64_t woken = 0, seen = seq_.load();
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return wake_ != woken; });
        woken = wake_;
      }
      // spin until the deadline passes, taking this helper's part of every
      // job started meanwhile (a sequence number seen before the wake-up is
      // never taken for a new job: only a changed one is)
      seen = seq_.load(std::memory_order_acquire);
      while (now_ns() < deadline_.load(std::memory_order_relaxed)) {
        const uint64_t s = seq_.load(std::memory_order_acquire);
        if (s != seen) {
          seen = s;
          if (claim_[w].exchange(1, std::memory_order_acq_rel) == 0) {
            part(w);
            done_.fetch_add(1, std::memory_order_release);
          }
        }
        _mm_pause();
      }
    }
  }
  static inline std::atomic<SpinTeam*> live_{nullptr};
  std::vector<std::thread> th_;
  std::mutex run_, m_;
  std::condition_variable cv_;
  uint64_t wake_ = 0;
  std::atomic<int64_t> deadline_{0};
  std::atomic<uint64_t> seq_{0};
  std::atomic<int> claim_[kParts];
  std::atomic<int> done_{0};
  const std::function<void(size_t, size_t)>* job_ = nullptr;
  size_t n_ = 0;
};

// records of grid chunks k0 .. k0 + n - 1 of an epoch at r0 (offset r0 + k W,
// size W, one kind, rolling hash key[k] or 0), in parallel when many: two
// 40-byte records are five 16-byte words, streamed past the caches (no
// read-for-ownership of the lines they overwrite).  (With ZC_FLAG_SHA1 the
// records' prefixes are written into them after the grid SHA-1 lands; writing
// the records through the caches for that measured the same, round 5.)
constexpr uint64_t kParallelRecordsMin = 32768;

void fill_grid_records(zc_record* out, uint64_t n, uint64_t r0, uint64_t k0, uint32_t W, uint32_t kind,
                       const uint64_t* key) {
  auto fill = [&](size_t a, size_t b) {
    auto put = [&](size_t j) {
      zc_record& r = out[j];
      r.offset = r0 + (k0 + j) * W;
      r.size = W;
      r.kind = kind;
      r.rolling = key ? key[k0 + j] : 0;
      memset(r.sha1, 0, sizeof r.sha1);
    };
    size_t j = a;
    for (; j < b && ((uintptr_t)(out + j) & 15); ++j) put(j);
    const uint64_t sk = (uint64_t)W | ((uint64_t)kind << 32);
    for (; j + 2 <= b; j += 2) {
      const uint64_t o0 = r0 + (k0 + j) * W, o1 = o0 + W;
      const uint64_t h0 = key ? key[k0 + j] : 0, h1 = key ? key[k0 + j + 1] : 0;
      __m128i* d = (__m128i*)(out + j);
      _mm_stream_si128(d + 0, _mm_set_epi64x((long long)sk, (long long)o0));
      _mm_stream_si128(d + 1, _mm_set_epi64x(0, (long long)h0));
      _mm_stream_si128(d + 2, _mm_set_epi64x((long long)o1, 0));
      _mm_stream_si128(d + 3, _mm_set_epi64x((long long)h1, (long long)sk));
      _mm_stream_si128(d + 4, _mm_setzero_si128());
    }
    for (; j < b; ++j) put(j);
    _mm_sfence();
  };
  if (n >= kParallelRecordsMin) SpinTeam::get().run(n, fill);  // (armed by the epoch before its wait)
  else fill(0, n);
}

class Resolver;

// the one-level screen's check table holds the by-value set plus this many of
// an epoch's own anchorless keys (grown when an epoch brings more)
constexpr uint64_t kChkRoomDefault = 65536;

// a candidate window of the walk: the window ending at p equals ref (an epoch
// ref or a historic entry)
struct CandPos {
  uint64_t p;
  uint32_t ref;
};

}  // namespace

struct zc_ctx {
  int device = 0;
  uint32_t W = 0;
  uint32_t flags = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // host -> HBM copies overlapped with the scan
  hipStream_t sha_stream = nullptr;   // SHA-1 of the grid chunks, beside the scan (ZC_FLAG_SHA1)
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_meta = nullptr, ev_in = nullptr, ev_idx = nullptr;
  hipEvent_t ev_sha = nullptr;  // the grid chunks' SHA-1 (sha_stream) are complete
  hipEvent_t ev_grec = nullptr;  // an epoch's chunk metadata is in: its grid records can be written
  hipEvent_t ev_copy = nullptr;  // the copy stream's work queued with an epoch's batch is done
  hipEvent_t ev_batch = nullptr;  // an epoch's batch is done (untimed)
  std::string err;

  // host feed
  uint8_t* stage = nullptr;  // pinned staging for the zero-copy feed contract
  DevBuf<uint8_t> d_stream;
  uint64_t n_stream = 0;
  bool finished = false;
  const uint8_t* d_last = nullptr;  // the stream the records describe
  uint64_t n_last = 0;

  // bounded feed window (zc_set_window; 0: the whole stream is kept in HBM):
  // stream bytes [wbase, wend) sit at dwin[0 ..) and, mirrored, in the pinned
  // host buffer hwin that the feed writes into (getInputBuffer)
  uint64_t win_cap = 0;
  DevBuf<uint8_t> dwin;
  HostBuf<uint8_t> hwin;
  // the window's buffers made on a helper thread (zc_set_window), joined by
  // window_open: pinning 1 GiB of host memory takes ~0.3 s, which a caller can
  // overlap with its index load (ChunkIndex::loadIndex) this way
  std::thread win_alloc;
  std::string win_alloc_err;
  uint64_t wbase = 0, wend = 0;
  bool slide_pending = false;  // a segment was resolved: slide before the next input
  bool windowed_last = false;  // the last stream came through the window
  Resolver* res = nullptr;     // the stream being fed (bounded window)

  // index entries known by value: seeded ones (zc_seed_index) and this
  // context's chunks without an anchor; probed by the exact screen
  std::vector<StaticEntry> statics;  // entries of size W
  std::unordered_map<uint64_t, std::vector<uint32_t>> smap;  // key -> statics
  uint64_t statics_ver = 1;  // bumped when the by-value set changes
  // the by-value set's screen structures for large sets (built for statics_ver)
  uint64_t sc_ver = 0;
  std::vector<uint32_t> sc_fbits;  // zc_fscan's 2^19-bit map
  DevBuf<uint32_t> bloom_s, bloom_w;  // Bloom filter of the set (and per epoch with the epoch's keys)
  uint32_t bloom_bits = 0;
  // the one-level screen (kBloomOneLevelMin keys and more): its check table
  // (and per epoch with the epoch's keys), or none (the two-level screen)
  DevBuf<uint16_t> chk_s, chk_w;
  DevBuf<unsigned int> chk_ovf;
  uint32_t chk_bits = 0;
  uint64_t chk_room = kChkRoomDefault;  // epoch keys the check table leaves room for
  bool bloom_one = false;
  DevBuf<uint64_t> kset;              // 64-bit keys, open addressing (empty = 0)
  uint32_t kset_bits = 0;
  int kset_zero = 0;
  DevBuf<uint64_t> flist;  // the epoch's anchorless keys, sorted (64-bit)
  // historic index: this context's W-byte chunks whose bytes are gone from HBM
  // (earlier streams, or evicted from the window), each with its first anchor
  std::vector<uint64_t, DefaultInit<uint64_t>> hkey;  // (resize leaves new entries to be written)
  std::vector<uint8_t, DefaultInit<uint8_t>> hsha;  // 16 bytes per entry (resize leaves them to be written)
  uint32_t nhist = 0;
  uint32_t nhist_seeded = 0;  // entries [0, nhist_seeded) came from zc_seed_index_meta
  DevBuf<uint32_t> hanc, hg;
  DevBuf<uint64_t> hfp, htab;
  DevBuf<uint64_t> hkey_d;  // the entries' keys on the device too (the candidates' key check)
  DevBuf<uint32_t> hfilt;
  uint32_t hbits = 0;
  bool hist_dirty = false;  // the table holds entries no longer in the index: rebuild before use

  // records: recs[rec_head, nrec_done) are complete (digests and chunk ids
  // filled in) and not yet taken (zc_take_records); records past nrec_done are
  // being cut.  The taken prefix is dropped once it is most of the vector, so
  // draining a long stream in small batches stays linear.
  RecordVec<zc_record> recs;  // resize leaves new records to be written; grid records may be written ahead
  // the resolver's per-stream lists, kept here for their capacity (Resolver):
  // a list built fresh per stream is new pages, and an incremental backup's
  // candidate lists are megabytes
  std::vector<uint64_t> fin_gq, fin_fresh;
  std::vector<uint32_t> fin_gslot, fin_frec;
  std::vector<CandPos> res_acands, res_hcands, res_sort_tmp;
  std::vector<std::pair<uint64_t, uint64_t>> res_spec_hist;
  std::vector<uint64_t> res_ha, res_hidx;
  std::vector<uint8_t> res_ok;
  std::vector<uint32_t> res_cls, res_cnext, res_ccur, res_ctail;
  // the probe's candidates, read back into pinned memory: a large copy into
  // pageable memory is staged by pinning the caller's pages, and freeing such
  // pages later (the list's destructor) stalled the next call's first
  // submission by 8-28 ms on the GPU box
  HostBuf<Cand> h_cand;
  // the candidates' device split and ordering (launch_cand_order)
  DevBuf<uint32_t> co_bcnt, co_boff, co_bsum, co_rank;
  DevBuf<Cand> co_out0, co_out;
  DevBuf<unsigned long long> co_hc;
  // the epoch tables (ckeys, tab, gfilt) are empty: cleared at the end of the
  // last stream; the next first epoch inserts without clearing (fused)
  bool tables_clean = false;
  HostBuf<unsigned long long> h_co_hc;
  HostBuf<Cand> h_hist_cand;  // the historic candidates, key-checked and in position order
  HostBuf<uint32_t> h_cls;  // the epoch's content classes (likewise)
  HostBuf<Run> h_runs;      // the screen's runs (likewise)
  size_t nrec_done = 0;
  size_t rec_head = 0;
  // every entry point holds this: calls on one context from several threads
  // are serialized (a bundle compressor thread and the feeding thread, say)
  mutable std::recursive_mutex mu;
  zc_stats stats{};

  LzoScratch* lzo = nullptr;  // bundle compression (zc_lzo.hip), made on first use
  DevBuf<uint8_t> lzo_in, lzo_out;  // zc_lzo_compress_host's device copies

  // scratch
  DevBuf<uint64_t> hm_key, hm_fp, hm_rkey;  // metadata of chunks joining the historic index
  DevBuf<uint32_t> hm_anc, hm_g, gidx;
  DevBuf<uint64_t> blk, ftile_off;
  DevBuf<uint32_t> ftile_cnt;
  DevBuf<uint32_t> dbase, dcnt;      // anchor directory per wave-tile
  DevBuf<uint32_t> prel, pg, srel, sg;  // anchor pool and side pool
  DevBuf<uint32_t> otiles, obase;
  DevBuf<unsigned long long> counters;
  // the scan's own two counters (anchors pooled, wave-tiles overflowed), zero
  // between scans: the first epoch's chunk-metadata kernel hands them to
  // h_scnt and clears them (no copy behind the scan, no fill before the next)
  DevBuf<unsigned long long> scnt;
  bool scnt_dirty = true;  // unknown contents (new, or a stream that failed): clear first
  DevBuf<uint8_t> gsha;  // SHA-1 of the first epoch's grid chunks (ZC_FLAG_SHA1)
  HostBuf<uint2> h_pairs;  // an epoch's pairs of grid chunks joined by speculation
  HostBuf<uint8_t> h_gsha;  // ... copied back on the SHA-1 stream right behind the kernel
  HostBuf<uint64_t> h_hmkey;  // pinned staging of the keys and anchors of new historic entries
  HostBuf<uint32_t> h_hmanc;
  DevBuf<uint64_t> c_start, c_key, c_fp, c_vis;
  DevBuf<uint32_t> c_anc, c_g;
  DevBuf<uint8_t> c_dead;
  DevBuf<uint64_t> ckeys;
  DevBuf<uint32_t> c_cls;
  DevBuf<uint64_t> tab;     // anchor table: 16-byte slots {gear | ref << 32, fingerprint}
  DevBuf<uint32_t> gfilt;   // its key filter
  DevBuf<Cand> cand;
  DevBuf<uint64_t> va, vb, dout;
  DevBuf<uint32_t> vlen;
  DevBuf<uint8_t> vok, sha_out;
  DevBuf<uint32_t> f32, fbits, fbits17;
  DevBuf<uint64_t> fwt_off;
  DevBuf<uint32_t> fwt_cnt;
  DevBuf<Run> runs;
  DevBuf<uint32_t> ancless;
  DevBuf<uint2> cpairs;  // content-class pairs to byte-check
  HostBuf<unsigned long long> h_cnt;
  HostBuf<unsigned long long> h_scnt;  // the scan's counters, read back with the first epoch's batch
  HostBuf<uint64_t> h_pre;             // digests of the predicted tail pieces (written by the device)
  HostBuf<uint64_t> h_key;  // grid-chunk keys of the current epoch
  HostBuf<uint64_t> h_ra, h_rb, h_rout;  // pinned staging of range-digest batches
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    HCK(hipSetDevice(dev));
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <class T>
void h2d(zc_ctx& c, T* dst, const T* src, size_t n) {
  if (n) HCK(hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyHostToDevice, c.stream));
}
template <class T>
void d2h(zc_ctx& c, T* dst, const T* src, size_t n) {
  if (n) HCK(hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyDeviceToHost, c.stream));
}
// Waits for a stream by polling it: a blocking wait returned 10-20 us after
// the work had ended (its wake-up), and the epoch's batch is waited for on
// every stream's critical path.  Past kSpinMaxMs it blocks.
constexpr double kSpinMaxMs = 4.0;
void wait_stream(hipStream_t s) {
  const auto t0 = Clock::now();
  for (unsigned i = 1;; ++i) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) HCK(e);
    if ((i & 255) == 0 && ms_since(t0) > kSpinMaxMs) {
      HCK(hipStreamSynchronize(s));
      return;
    }
    _mm_pause();
  }
}
void sync(zc_ctx& c) { wait_stream(c.stream); }
// the same for an event
void wait_event(hipEvent_t ev) {
  const auto t0 = Clock::now();
  for (unsigned i = 1;; ++i) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) HCK(e);
    if ((i & 255) == 0 && ms_since(t0) > kSpinMaxMs) {
      HCK(hipEventSynchronize(ev));
      return;
    }
    _mm_pause();
  }
}

// ---------------------------------------------------------------------------
// the context's index beyond the stream being resolved

void add_static(zc_ctx& c, uint64_t key, const uint8_t* sha, uint8_t seeded) {
  StaticEntry e;
  e.key = key;
  memcpy(e.sha, sha, 16);
  e.seeded = seeded;
  c.smap[key].push_back((uint32_t)c.statics.size());
  c.statics.push_back(e);
  ++c.statics_ver;
}

// the large-set screen structures of the by-value set, rebuilt when it changed
void statics_screen(zc_ctx& c) {
  if (c.sc_ver == c.statics_ver) return;
  std::vector<uint64_t> keys;
  keys.reserve(c.smap.size());
  for (const auto& kv : c.smap) keys.push_back(kv.first);
  c.sc_fbits.assign(1u << 14, 0);
  c.bloom_bits = bloom_bits_for(keys.size() + 64);
  std::vector<uint32_t> bloom(bloom_words(c.bloom_bits), 0);
  uint32_t* const pf = bloom.data() + (2u << c.bloom_bits);
  uint32_t bits = 10;
  while ((1ull << bits) < 2ull * keys.size() + 2) ++bits;
  std::vector<uint64_t> set(1ull << bits, 0);
  c.kset_zero = 0;
  for (uint64_t k : keys) {
    const uint32_t h = (uint32_t)k;
    c.sc_fbits[h >> 18] |= 1u << ((h >> 13) & 31);
    const uint32_t b = bloom_block(k, c.bloom_bits), g = bloom_seed(k);
    bloom[2 * b] |= bloom_lo(g);
    bloom[2 * b + 1] |= bloom_hi(g);
    const uint32_t f = bloom_pf(k);
    pf[f >> 5] |= 1u << (f & 31);
    if (k == 0) {
      c.kset_zero = 1;
      continue;
    }
    for (uint64_t s = (k * 0x9E3779B97F4A7C15ull) >> (64 - bits);; s = (s + 1) & ((1ull << bits) - 1))
      if (set[s] == 0) {
        set[s] = k;
        break;
      }
  }
  c.bloom_s.ensure(bloom.size());
  c.bloom_one = keys.size() + 64 >= kBloomOneLevelMin;
  if (c.bloom_one) {
    // room for the epochs' own keys too (launch_chk_add: chk_room of them, more
    // after an epoch overflowed it); a chain that would reach the last bucket
    // makes the table twice as large.  (ZC_TEST_CHK_BITS: tests start the
    // search from a table too small for any epoch keys, to force that overflow.)
    // (the hook's value is used only inside [10, 30]; anything else is ignored)
    const char* tb = c.chk_room == kChkRoomDefault ? getenv("ZC_TEST_CHK_BITS") : nullptr;
    const long tbv = tb ? strtol(tb, nullptr, 10) : 0;
    const bool test_bits = tbv >= 10 && tbv <= 30;
    for (c.chk_bits = test_bits ? (uint32_t)tbv : chk_bits_for(keys.size() + c.chk_room);; ++c.chk_bits) {
      const uint64_t nb = (1ull << c.chk_bits) + kChkPad;
      std::vector<uint16_t> chk(nb * 4, 0);
      bool fits = true;
      for (uint64_t k : keys) {
        const uint16_t cw = (uint16_t)chk_word(k);
        uint64_t sl = (uint64_t)chk_bucket(k, c.chk_bits) * 4;
        while (sl < (nb - 1) * 4 && chk[sl] != 0 && chk[sl] != cw) ++sl;
        if (sl == (nb - 1) * 4) {
          fits = false;
          break;
        }
        chk[sl] = cw;
      }
      if (!fits) continue;
      c.chk_s.ensure(chk.size());
      h2d(c, c.chk_s.p, chk.data(), chk.size());
      c.chk_ovf.ensure(1);
      break;
    }
  }
  c.kset.ensure(set.size());
  c.kset_bits = bits;
  h2d(c, c.bloom_s.p, bloom.data(), bloom.size());
  h2d(c, c.kset.p, set.data(), set.size());
  sync(c);
  c.sc_ver = c.statics_ver;
}

// historic table: 2^hbits >= 2 max(nhist, room) slots; grows by a rebuild
// (or is rebuilt at its size with `clear`), otherwise entries [from, nhist)
// are inserted
void hist_table(zc_ctx& c, uint32_t from, uint64_t room = 0, bool clear = false) {
  const uint64_t want = std::max<uint64_t>(c.nhist, room);
  if (clear) c.hist_dirty = true;
  if (!want) return;  // (an empty index is not probed: cleared when it is next filled)
  uint32_t bits = std::max<uint32_t>(c.hbits, 12);
  while ((1ull << bits) < 2ull * want) ++bits;
  c.hfilt.ensure(probe_filter_words());
  if (bits != c.hbits || !c.htab.p || c.hist_dirty) {
    c.hist_dirty = false;
    sync(c);  // a probe may still read the old table
    c.htab.ensure(2ull << bits);
    c.hbits = bits;
    from = 0;
    HCK(hipMemsetAsync(c.htab.p, 0xFF, (2ull << bits) * sizeof(uint64_t), c.stream));
    HCK(hipMemsetAsync(c.hfilt.p, 0, probe_filter_words() * sizeof(uint32_t), c.stream));
  }
  if (c.nhist > from)
    HCK(launch_hist_insert(c.hg.p, c.hfp.p, c.hanc.p, from, c.nhist - from, c.htab.p, c.hbits, c.hfilt.p, c.stream));
}

// Room for `total` historic entries, made before a stream queues any work:
// the device arrays and the table are grown now, since growing them when the
// stream's new chunks register at its end frees the old buffers, and hipFree
// waits for the whole device -- the grid SHA-1 on its side stream included
// (the registration's cost then followed the history's size: 1.70 ms with
// 131,072 entries, 0.23 with none).  Grown geometrically, so a
// long series of backups on one context rebuilds its table O(log) times.
void hist_reserve(zc_ctx& c, uint64_t total) {
  if (total > 0xFFFFFFF0ull || total <= c.nhist) return;
  if (total > c.hanc.cap) total = std::max<uint64_t>(total, 2ull * c.nhist);
  c.hanc.grow_keep(total, c.nhist, c.stream);
  c.hg.grow_keep(total, c.nhist, c.stream);
  c.hfp.grow_keep(total, c.nhist, c.stream);
  c.hkey_d.grow_keep(total, c.nhist, c.stream);
  c.hkey.reserve(total);
  c.hsha.reserve(16 * total);
  hist_table(c, c.nhist, total);
}

// the anchor definition metadata carries (zc_anchor_def): 'ZA', definition 2
// (two packed 16-bit parity gears tested at every byte, the first anchor at
// offset >= ZC_ANCHOR_MIN_OFF, the 8-byte fingerprint ending at it: round 5),
// and log2 of the anchor rate chosen for W
uint32_t anchor_def_of(uint32_t W) { return 0x5A410000u | (2u << 8) | (uint32_t)__builtin_ctz(anchor_rate_inv(W)); }

// a by-value entry unless (key, SHA-1) is indexed already (registerNewChunkId,
// chunk_index.cc:163-182)
void add_static_once(zc_ctx& c, uint64_t key, const uint8_t* sha, uint8_t seeded) {
  auto it = c.smap.find(key);
  if (it != c.smap.end())
    for (uint32_t i : it->second)
      if (memcmp(c.statics[i].sha, sha, 16) == 0) return;
  add_static(c, key, sha, seeded);
}

// keep the first nh historic entries and the first ns by-value entries
void index_truncate(zc_ctx& c, uint32_t nh, size_t ns, bool force = false) {
  if (!force && c.nhist == nh && c.statics.size() == ns) return;
  c.nhist = std::min(c.nhist, nh);
  c.hkey.resize(c.nhist);
  c.hsha.resize(16 * (size_t)c.nhist);
  if (ns < c.statics.size()) c.statics.resize(ns);
  c.smap.clear();
  for (uint32_t i = 0; i < c.statics.size(); ++i) c.smap[c.statics[i].key].push_back(i);
  ++c.statics_ver;
  hist_table(c, 0, 0, true);  // rebuilt at its size (the next stream needs the room again)
}

// ---------------------------------------------------------------------------
class Resolver {
 public:
  // A stream of the context.  Whole-stream mode (zc_chunk_device /
  // zc_chunk_host / an unbounded feed): the n bytes sit at `d`, and run()
  // does everything.  Window mode (bounded feed): the stream arrives in the
  // context's window; each full window half is resolved by run_segment()
  // up to its last scanned tile, the window slides (rebase), and
  // run_final() resolves the rest at finish().  All positions are absolute
  // stream offsets: the device arrays indexed by position (the bytes, the
  // span digests, the anchor directory, the screen's per-tile lists) are
  // passed as pointers biased by the window base, so the kernels never see
  // the window.
  Resolver(zc_ctx& c, const uint8_t* d, uint64_t n, bool windowed)
      : c_(c), dphys_(d), n_(n), cap_(windowed ? c.win_cap + ZC_STILE : n), windowed_(windowed), W_(c.W),
        indexable_(c.W >= 128) {
    d_ = dphys_;
  }
  // An error thrown out of the pipeline leaves no device work behind: the
  // side streams (SHA-1 of the grid chunks, copies, tail digests) may still be
  // reading the caller's buffer, which the caller may free once the call
  // has returned its error.
  ~Resolver() {
    if (std::uncaught_exceptions() > 0) {
      drain();
      c_.scnt_dirty = true;  // a scan's counters may not have been handed over
    }
  }
  void drain() {
    (void)hipStreamSynchronize(c_.sha_stream);
    (void)hipStreamSynchronize(c_.copy_stream);
    (void)hipStreamSynchronize(c_.stream);
  }

  // whole pipeline over a stream already in HBM
  void run() {
    begin();
    run_final();
  }

  // Stream start: statistics, records, the resolver state and the scan's
  // buffers (sized for the window, or for the whole stream).
  void begin() {
    t_begin_ = Clock::now();
    c_.recs.clear();
    c_.nrec_done = 0;
    c_.rec_head = 0;
    if (!windowed_) c_.recs.reserve(std::min<uint64_t>(n_ / W_ + 16, 1u << 24));
    c_.stats = zc_stats{};
    c_.stats.bytes = n_;
    c_.stats.window_bytes = windowed_ ? c_.win_cap : 0;
    hist0_ = c_.nhist;
    statics0_ = c_.statics.size();
    // the stream's new W-byte chunks (at most n / W of them) join the index at
    // its end: room for them now, before anything of the stream is queued
    if (!windowed_ && indexable_ && (c_.flags & ZC_FLAG_SHA1) && n_ >= W_) hist_reserve(c_, c_.nhist + n_ / W_ + 2);
    r_ = s_ = x_resume_ = hspan_ = 0;
    gruns_.clear();
    fresh_.clear();
    spec_hist_.clear();
    acands_.clear();
    hcands_.clear();
    // the scan writes the first epoch's grid keys (W a multiple of the lane
    // span dividing the wave-tile; the whole stream resident): their arrays
    // sized now, before it is queued
    bool kok = false;
    key_lshift_ = scan_key_lshift_or_none(W_, kok);
    scan_keys_ = kok && !windowed_ && indexable_ && n_ >= W_ && n_ / W_ < 0xFFFFFFF0ull;
    if (scan_keys_) {
      c_.c_key.ensure(n_ / W_ + 2);
      c_.h_key.ensure(n_ / W_ + 2);
    }
    scan_setup();
  }
  // bytes [0, n) of the stream are (being) copied to the device, in order on
  // the context's stream
  void set_avail(uint64_t n) {
    n_ = n;
    c_.stats.bytes = n;
  }
  // the epoch tables emptied on the context's stream (whole capacities)
  void clear_tables() {
    if (c_.tables_clean || (!c_.ckeys.p && !c_.tab.p)) return;
    if (c_.ckeys.cap % 2 || c_.tab.cap % 2 || c_.gfilt.cap % 4) return;  // (not whole 16-byte units: left dirty)
    HCK(launch_tables_clear(c_.ckeys.p, c_.ckeys.p ? c_.ckeys.cap : 0, c_.tab.p, c_.tab.p ? c_.tab.cap : 0,
                            c_.gfilt.p, c_.gfilt.p ? c_.gfilt.cap : 0, c_.stream));
    c_.tables_clean = true;
  }
  // the event that marks the end of the stream's scan (scan_finish)
  hipEvent_t scan_end_event() const { return (c_.flags & ZC_FLAG_TIMING) ? c_.ev1 : c_.ev_idx; }
  // launch the scan of the full 2 MiB tiles below m; `last`: no scan kernel
  // follows this one, so it records the scan-end event itself
  void scan_upto(uint64_t m, bool last = false) {
    const uint64_t t1 = std::min(m, n_) / ZC_STILE;
    if (t1 > tiles_done_) {
      hipEvent_t start = nullptr;
      if (!scan_open_) {
        if (c_.flags & ZC_FLAG_TIMING) start = c_.ev0;
        scan_open_ = true;
      }
      scnt_pending_ = true;
      const GridKeysOut gko = scan_keys_ ? GridKeysOut{c_.c_key.p, c_.h_key.p, pow257(W_), key_lshift_}
                                         : GridKeysOut{nullptr, nullptr, 0, 0};
      hipEvent_t stop = last ? scan_end_event() : nullptr;
      HCK(launch_scan_tiles(d_, n_, tiles_done_, t1 - tiles_done_, anchor_lo_, blk_v(), pool_out(), c_.scnt.p,
                            c_.stream, gko, start, stop));
      scan_end_recorded_ = stop != nullptr;
      tiles_done_ = t1;
    }
  }
  uint64_t scanned_end() const { return tiles_done_ * ZC_STILE; }

  // window mode: resolve every probe below lim (the scanned end), cut the
  // records up to there and complete them (digests, chunk ids)
  void run_segment(uint64_t lim) {
    const auto t0 = Clock::now();
    scan_upto(lim);
    lim = std::min(lim, scanned_end());
    if (lim <= x0()) return;
    scan_finish();
    lim_ = lim;
    final_ = false;
    while (epoch()) {
    }
    if (!scan_checked_) {
      sync(c_);
      scan_check();
    }
    finalize_records();
    c_.stats.segments++;
    c_.stats.total_ms += ms_since(t0);
  }

  // the end of the stream (n_ bytes): the partial last tile, every probe,
  // finish(), the records completed; with ZC_FLAG_SHA1 the stream's new
  // W-byte chunks join the context's index (Writer::add ->
  // ChunkIndex::addChunk), without it the index is left as the stream found it
  void run_final() {
    const auto t0 = Clock::now();
    if (n_ > 0) {
      const bool tail = n_ % ZC_STILE != 0;
      scan_upto(n_, !tail);
      if (tail) {
        hipEvent_t start = nullptr;
        if (!scan_open_) {
          if (c_.flags & ZC_FLAG_TIMING) start = c_.ev0;
          scan_open_ = true;
        }
        scnt_pending_ = true;
        HCK(launch_scan_tail(d_, n_, anchor_lo_, blk_v(), pool_out(), c_.scnt.p, c_.stream, start, scan_end_event()));
        scan_end_recorded_ = true;
      }
      if (!windowed_) pre_sha();
      scan_finish();
      lim_ = n_;
      final_ = true;
      while (epoch()) {
      }
      if (!scan_checked_) {  // no epoch synchronised (no refs): for the statistics
        sync(c_);
        scan_check();
      }
    }
    finalize_records(true);
    clear_tables();  // (normally done after the last epoch's probe already)
    const double ms = ms_since(t0);
    c_.stats.total_ms += ms;
    // the resolver's work overlaps the scan's tail (nothing waits for the scan
    // alone), so the part after the scan is the whole minus the scan
    c_.stats.resolve_ms = (c_.flags & ZC_FLAG_TIMING) ? std::max(0.0, c_.stats.total_ms - c_.stats.scan_ms)
                                                      : c_.stats.total_ms;
    c_.stats.hist_entries = c_.nhist;
  }

  // window mode: the first stream position the resolver will read again
  // (the next epoch's pending bytes and grid chunks from s_, the screen's
  // and the probe's first windows from x0 - W + 1, plus one scan tile of
  // halo for the next tile's warm-up bytes), a multiple of the 2 MiB tile
  uint64_t keep_from() const {
    const uint64_t xs = x0();
    uint64_t lo = s_;
    const uint64_t ws = xs >= W_ ? xs - W_ + 1 : 0;
    lo = std::min(lo, (ws >> ZC_WT_SHIFT) << ZC_WT_SHIFT);
    const uint64_t fw = xs / ZC_FWT * ZC_FWT;
    lo = std::min(lo, fw >= (uint64_t)W_ + 4096 ? fw - W_ - 4096 : 0);
    uint64_t keep = lo / ZC_STILE * ZC_STILE;
    keep = keep >= ZC_STILE ? keep - ZC_STILE : 0;
    return std::max(keep, wbase_);
  }

  // window mode: the refs that start before `keep` lose their bytes: they
  // join the historic index (key, SHA-1, first anchor), computed now while
  // their bytes are still resident
  void evict_before(uint64_t keep) {
    size_t k = 0;
    while (k < cstart_.size() && cstart_[k] < keep) ++k;
    if (!k) return;
    std::vector<uint64_t> starts(cstart_.begin(), cstart_.begin() + k);
    hist_add(starts, nullptr);
    cstart_.erase(cstart_.begin(), cstart_.begin() + k);
    ckey_.erase(ckey_.begin(), ckey_.begin() + k);
    cfp_.erase(cfp_.begin(), cfp_.begin() + k);
    cg_.erase(cg_.begin(), cg_.begin() + k);
    canc_.erase(canc_.begin(), canc_.begin() + k);
    nconf_ = (uint32_t)cstart_.size();
  }

  // window mode: the window moved; stream byte wbase is at dphys[0]
  void rebase(const uint8_t* dphys, uint64_t wbase) {
    dphys_ = dphys;
    wbase_ = wbase;
    d_ = dphys_ - wbase_;
  }
  uint64_t wbase() const { return wbase_; }
  uint64_t chk_wt() const { return chk_wt_; }  // wave-tiles below have been checked

  // New index entries from this context's chunks [starts[i], starts[i] + W)
  // (resident): all of them join the historic index (key and SHA-1 on the
  // host, first anchor on the device; those with an anchor enter its table),
  // those without an anchor also the by-value set of the exact screen.
  // sha16: the chunks' SHA-1 prefixes when known (16 bytes each), else
  // computed here.
  void hist_add(const std::vector<uint64_t>& starts, const uint8_t* sha16) {
    const HistPending hp = hist_add_meta(starts);
    if (!hp.k) return;
    std::vector<uint8_t> sha;
    if (!sha16) {
      std::vector<uint32_t> len(hp.k, W_);
      const std::vector<uint8_t> sha20 = sha1s(starts, len);
      sha.resize(16 * (size_t)hp.k);
      for (uint32_t i = 0; i < hp.k; ++i) memcpy(&sha[16 * (size_t)i], &sha20[20 * (size_t)i], 16);
      sha16 = sha.data();
    }
    hist_add_sha(hp, sha16);
  }

  // The part of hist_add that needs no SHA-1: the entries' key, first anchor,
  // gear and fingerprint (device), their table insert, the keys on the host.
  // hist_add_sha completes the entries once their SHA-1 prefixes are known.
  struct HistPending {
    uint32_t e0 = 0, k = 0;
    const uint32_t* anc = nullptr;  // the entries' first anchors (host), complete after a sync
  };
  HistPending hist_add_meta(const std::vector<uint64_t>& starts) {
    HistPending hp;
    const uint32_t k = (uint32_t)starts.size();
    if (!k || !indexable_) return hp;
    const uint32_t e0 = c_.nhist;
    c_.va.ensure(k);
    c_.hanc.grow_keep(e0 + k, e0, c_.stream);
    c_.hg.grow_keep(e0 + k, e0, c_.stream);
    c_.hfp.grow_keep(e0 + k, e0, c_.stream);
    c_.hkey_d.grow_keep(e0 + k, e0, c_.stream);
    c_.h_hmanc.ensure(k);
    // a leading run of consecutive grid chunks of the epoch whose metadata the
    // device arrays hold (a whole stream's new chunks, but for the last one or
    // two that finish() cuts) is copied as it is, its keys from the host's
    // copy of the epoch's; the rest is gathered by index lists
    uint32_t run = 0;
    const int64_t ref0 = epoch_ref_at(starts[0]);
    if (ref0 >= (int64_t)dev_nconf_) {
      const uint64_t lim = std::min<uint64_t>(k, (uint64_t)dev_nconf_ + dev_nspec_ - (uint64_t)ref0);
      while (run < lim && starts[run] == starts[0] + (uint64_t)run * W_) ++run;
    }
    c_.hkey.resize((size_t)e0 + k);
    if (run) {
      const uint32_t r0 = (uint32_t)ref0;
      HCK(hipMemcpyAsync(c_.hanc.p + e0, c_.c_anc.p + r0, run * sizeof(uint32_t), hipMemcpyDeviceToDevice, c_.stream));
      HCK(hipMemcpyAsync(c_.hg.p + e0, c_.c_g.p + r0, run * sizeof(uint32_t), hipMemcpyDeviceToDevice, c_.stream));
      HCK(hipMemcpyAsync(c_.hfp.p + e0, c_.c_fp.p + r0, run * sizeof(uint64_t), hipMemcpyDeviceToDevice, c_.stream));
      HCK(hipMemcpyAsync(c_.hkey_d.p + e0, c_.c_key.p + r0, run * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                         c_.stream));
      memcpy(c_.hkey.data() + e0, c_.h_key.p + (r0 - dev_nconf_), run * sizeof(uint64_t));
    }
    if (run < k) {
      const uint32_t kr = k - run;  // entries e0 + run + t, t < kr
      c_.hm_key.ensure(kr);
      // chunks that are refs of the current epoch take the metadata it
      // computed (its grid chunks, its confirmed refs); the rest is computed
      // from the bytes
      std::vector<uint32_t> gsrc, gdst;
      std::vector<uint64_t> rest;
      std::vector<uint32_t> rdst;
      for (uint32_t t = 0; t < kr; ++t) {
        const int64_t ref = epoch_ref_at(starts[run + t]);
        if (ref >= 0) {
          gsrc.push_back((uint32_t)ref);
          gdst.push_back(t);
        } else {
          rest.push_back(starts[run + t]);
          rdst.push_back(t);
        }
      }
      const uint32_t eb = e0 + run;
      c_.gidx.ensure(2ull * kr);  // both lists' index pairs, allocated before either launch
      if (!gsrc.empty()) {
        const uint32_t m = (uint32_t)gsrc.size();
        h2d(c_, c_.gidx.p, gsrc.data(), m);
        h2d(c_, c_.gidx.p + m, gdst.data(), m);
        HCK(launch_ref_gather(c_.gidx.p, c_.gidx.p + m, m, c_.c_key.p, c_.c_anc.p, c_.c_g.p, c_.c_fp.p, c_.hm_key.p,
                              c_.hanc.p + eb, c_.hg.p + eb, c_.hfp.p + eb, c_.stream));
      }
      if (!rest.empty()) {
        // computed into the staging slots after the gathered ones, then moved
        const uint32_t m = (uint32_t)rest.size();
        c_.hm_anc.ensure(m);
        c_.hm_g.ensure(m);
        c_.hm_fp.ensure(m);
        c_.hm_rkey.ensure(m);
        h2d(c_, c_.va.p, rest.data(), m);
        HCK(launch_ref_meta(d_, blk_v(), av(), c_.va.p, m, W_, pow257(W_), c_.hm_rkey.p, c_.hm_anc.p, c_.hm_g.p,
                            c_.hm_fp.p, c_.stream));
        std::vector<uint32_t> src(m);
        for (uint32_t t = 0; t < m; ++t) src[t] = t;
        uint32_t* gi = c_.gidx.p + 2ull * gsrc.size();
        h2d(c_, gi, src.data(), m);
        h2d(c_, gi + m, rdst.data(), m);
        HCK(launch_ref_gather(gi, gi + m, m, c_.hm_rkey.p, c_.hm_anc.p, c_.hm_g.p, c_.hm_fp.p, c_.hm_key.p,
                              c_.hanc.p + eb, c_.hg.p + eb, c_.hfp.p + eb, c_.stream));
      }
      c_.h_hmkey.ensure(kr);
      HCK(hipMemcpyAsync(c_.hkey_d.p + eb, c_.hm_key.p, kr * sizeof(uint64_t), hipMemcpyDeviceToDevice, c_.stream));
      d2h(c_, c_.h_hmkey.p, c_.hm_key.p, kr);
      sync(c_);
      memcpy(c_.hkey.data() + eb, c_.h_hmkey.p, kr * sizeof(uint64_t));
    }
    // the entries' anchors, for hist_add_sha (it synchronises first)
    d2h(c_, c_.h_hmanc.p, c_.hanc.p + e0, k);
    hp.anc = c_.h_hmanc.p;
    c_.nhist = e0 + k;
    hist_table(c_, e0);
    hp.e0 = e0;
    hp.k = k;
    return hp;
  }
  // sha16: the entries' SHA-1 prefixes, 16 bytes each; entries without an
  // anchor also join the by-value set of the exact screen
  // (sha16 null: already in place in c_.hsha)
  // (ancless: the entries without an anchor when already known, see
  // ancless_of; else found here)
  void hist_add_sha(const HistPending& hp, const uint8_t* sha16, const std::vector<uint32_t>* ancless = nullptr) {
    if (!hp.k) return;
    std::vector<uint32_t> own;
    if (!ancless) {
      own = ancless_of(hp);
      ancless = &own;
    }
    c_.hsha.resize(16 * ((size_t)hp.e0 + hp.k));
    uint8_t* hs = c_.hsha.data() + 16 * (size_t)hp.e0;
    if (sha16) memcpy(hs, sha16, 16 * (size_t)hp.k);
    for (uint32_t i : *ancless) add_static_once(c_, c_.hkey[hp.e0 + i], hs + 16 * (size_t)i, 0);
  }
  // the pending entries without an anchor (they join the by-value set too)
  std::vector<uint32_t> ancless_of(const HistPending& hp) {
    std::vector<uint32_t> v;
    if (!hp.k) return v;
    sync(c_);  // hp.anc has landed
    for (uint32_t i = 0; i < hp.k; ++i)
      if (hp.anc[i] == ZC_NO_ANCHOR) v.push_back(i);
    return v;
  }

 private:
  zc_ctx& c_;
  const uint8_t* dphys_;  // stream byte wbase_ is at dphys_[0]
  const uint8_t* d_;      // dphys_ - wbase_: indexed by absolute stream offset
  uint64_t wbase_ = 0;
  uint64_t n_;            // bytes of the stream on the device (so far)
  const uint64_t cap_;    // bytes the position-indexed device arrays cover
  const bool windowed_;
  bool final_ = true;     // this resolution reaches the end of the stream
  uint64_t lim_ = 0;      // probes below lim_ are resolved by this call
  const uint32_t W_;
  const bool indexable_;
  // x / W and x % W without a 64-bit division when W is a power of two (the
  // per-candidate loops run 100 K+ times per stream)
  const int wsh_ = (W_ & (W_ - 1)) == 0 ? __builtin_ctz(W_) : -1;
  uint64_t wdiv(uint64_t x) const { return wsh_ >= 0 ? x >> wsh_ : x / W_; }
  uint64_t wmod(uint64_t x) const { return wsh_ >= 0 ? x & (W_ - 1) : x % W_; }
  uint64_t npool_ = 0;
  const int32_t anchor_lo_ = anchor_lo_for(W_);
  const uint32_t wcap_ = wave_tile_cap(W_);
  Clock::time_point t_begin_;
  uint64_t tiles_done_ = 0;  // full scan tiles launched
  bool scan_open_ = false;   // scan launches queued since the last scan_finish
  bool scan_end_recorded_ = false;  // the last scan launch records the scan-end event itself
  uint64_t chk_wt_ = 0;      // wave-tiles below are checked for overflow
  uint64_t side_used_ = 0;   // entries of the side pool in use
  uint32_t hist0_ = 0;       // historic entries when the stream began
  size_t statics0_ = 0;

  // position-indexed device arrays, biased by the window base
  uint64_t* blk_v() const { return c_.blk.p - wbase_ / ZC_SPAN; }
  uint32_t* dbase_v() const { return c_.dbase.p - (wbase_ >> ZC_WT_SHIFT); }
  uint32_t* dcnt_v() const { return c_.dcnt.p - (wbase_ >> ZC_WT_SHIFT); }
  PoolOut pool_out() const {
    return PoolOut{dbase_v(), dcnt_v(), c_.prel.p, c_.pg.p, wcap_, wbase_ >> ZC_WT_SHIFT};
  }
  AnchorView av() const { return AnchorView{dbase_v(), dcnt_v(), c_.prel.p, c_.pg.p, c_.srel.p, c_.sg.p}; }
  HistTab hist_tab() const {
    return c_.nhist ? HistTab{c_.htab.p, c_.hbits, c_.hfilt.p, c_.hanc.p} : HistTab{nullptr, 0, nullptr, nullptr};
  }
  // wave-tiles of the stream the scan has written (a partial last tile only
  // at the end)
  uint64_t nwt_done() const { return final_ ? wave_tiles(n_) : tiles_done_ * (ZC_SCAN_TPB / 64); }

  // resolver state: reset point r_, bytes saved up to s_, grid origin r_e_ of
  // the epoch (on r_'s grid: its first chunk not yet saved), its probes
  // [x_resume_ or r_ + W - 1, h_end_), and the next horizon length hspan_
  // (0 = to the end of the stream)
  uint64_t r_ = 0, s_ = 0, r_e_ = 0;
  uint64_t x_resume_ = 0, h_end_ = 0, hspan_ = 0;
  uint64_t x0() const { return std::max<uint64_t>(r_ + W_ - 1, x_resume_); }

  // refs = indexable W-byte chunks that can be matched: [0, nconf_) saved in
  // earlier epochs (visible to every later probe), [nconf_, nref_) this
  // epoch's grid chunks, start r_e + k * W, visible from start + 2W - 1.
  // The grid chunks' metadata lives on the device; the host holds their keys.
  std::vector<uint64_t> cstart_, ckey_, cfp_;  // cfp_: anchor fingerprint
  std::vector<uint32_t> canc_, cg_;            // cg_: anchor gear value
  std::vector<uint8_t> dead_;
  uint64_t ndead_ = 0;  // refs of this epoch consumed by same-grid matches
  bool scan_keys_ = false;    // the scan writes the first epoch's grid keys (begin)
  hipEvent_t grec_ev_ = nullptr;  // the grid records' keys are in once this event is
  uint32_t key_lshift_ = 0;   // log2 of the lane spans per grid chunk
  static constexpr uint64_t kParallelRecords = 32768;
  uint32_t nconf_ = 0, nspec_ = 0, nref_ = 0;
  uint64_t ks_ = 0;  // next grid chunk of this epoch to save

  // The grid ref of the epoch whose metadata sits in the device arrays that is
  // chunk [start, start + W), or -1.  The arrays keep the layout of that
  // epoch's start (confirmed refs, then grid chunk k at dev_nconf_ + k), which
  // keep_saved / evict_before change on the host side only afterwards.
  uint64_t dev_r_e_ = 0;
  uint32_t dev_nconf_ = 0, dev_nspec_ = 0;
  bool dev_valid_ = false;
  int64_t epoch_ref_at(uint64_t start) const {
    if (!dev_valid_ || start < dev_r_e_ || (start - dev_r_e_) % W_) return -1;
    const uint64_t k = (start - dev_r_e_) / W_;
    return k < dev_nspec_ ? (int64_t)(dev_nconf_ + k) : -1;
  }

  uint64_t ref_start(uint32_t ref) const {
    return ref < nconf_ ? cstart_[ref] : r_e_ + (uint64_t)(ref - nconf_) * W_;
  }
  uint64_t ref_vis(uint32_t ref) const { return ref < nconf_ ? 0 : ref_start(ref) + 2ull * W_ - 1; }
  uint64_t ref_key(uint32_t ref) const { return ref < nconf_ ? ckey_[ref] : c_.h_key[ref - nconf_]; }

  // content classes of this epoch as linked lists in ascending ref order (so
  // in start and visibility order): cls_[r] = leader, cnext_[r] = next member,
  // ccur_[leader] = first member not consumed.  Empty: every ref leads its
  // own class.
  static constexpr uint32_t kNone = 0xFFFFFFFFu;
  std::vector<uint32_t>& cls_ = c_.res_cls;
  std::vector<uint32_t>& cnext_ = c_.res_cnext;
  std::vector<uint32_t>& ccur_ = c_.res_ccur;

  void load_classes() {
    c_.h_cls.ensure(nref_);
    d2h(c_, c_.h_cls.p, c_.c_cls.p, nref_);
    sync(c_);
    cls_.assign(c_.h_cls.p, c_.h_cls.p + nref_);
    cnext_.assign(nref_, kNone);
    ccur_.resize(nref_);
    std::vector<uint32_t>& tail = c_.res_ctail;
    tail.resize(nref_);
    for (uint32_t r = 0; r < nref_; ++r) {
      ccur_[r] = r;
      tail[r] = r;
      const uint32_t l = cls_[r];
      if (l != r) {
        cnext_[tail[l]] = r;
        tail[l] = r;
      }
    }
  }

  // is some ref of the class led by `lead` in the index at probe p (cut by
  // then and not consumed by a same-grid match)?
  bool class_alive_visible(uint32_t lead, uint64_t p) {
    if (cls_.empty()) return ref_vis(lead) <= p && !dead_[lead];
    uint32_t& c = ccur_[lead];
    while (c != kNone && dead_[c]) c = cnext_[c];
    return c != kNone && ref_vis(c) <= p;
  }

  std::unordered_map<uint64_t, std::vector<uint32_t>> fmap_;  // key -> anchorless refs (start order)
  std::unordered_map<uint64_t, std::vector<uint32_t>>::iterator fmemo_it_;  // last fmap_ lookup
  uint64_t fmemo_key_ = 0;
  bool fmemo_valid_ = false;
  std::vector<Run> runs_;
  uint32_t flist_n_ = 0;
  uint64_t f_min_vis_ = kInf;
  bool has_f_ = false;

  using ACand = CandPos;
  std::vector<ACand>& acands_ = c_.res_acands;
  std::vector<ACand>& hcands_ = c_.res_hcands;  // confirmed candidates of historic entries (ref = entry)

  // F verification batch (positions ascending)
  struct FBatch {
    std::vector<uint64_t> pos, h;
    std::vector<int64_t> vref;     // ref verified against, -1 none
    std::vector<uint8_t> vok;      // content equal to vref
    std::vector<uint8_t> sha;      // 20 bytes per position (statics only)
    std::vector<uint8_t> has_sha;
    size_t cur = 0;
  } fb_;

  struct Piece {
    size_t rec;
    uint64_t a, b;
  };
  std::vector<Piece> need_digest_;

  // ---------------------------------------------------------------- scan
  void scan_setup() {
    const uint64_t nwt = wave_tiles(cap_);
    if (nwt * wcap_ >= ZC_SIDE_POOL) throw ZcError{ZC_ERR_NOMEM, "stream too large for the anchor pool"};
    c_.blk.ensure((cap_ + ZC_SPAN - 1) / ZC_SPAN);
    c_.dbase.ensure(nwt);
    c_.dcnt.ensure(nwt);
    c_.prel.ensure(nwt * wcap_);
    c_.pg.ensure(nwt * wcap_);
    c_.srel.ensure(1);
    c_.sg.ensure(1);
    if (!c_.counters.p) {  // (every user clears what it counts in; zeroed once when made)
      c_.counters.ensure(CNT_LAST);
      HCK(hipMemsetAsync(c_.counters.p, 0, CNT_LAST * sizeof(unsigned long long), c_.stream));
    }
    c_.h_cnt.ensure(CNT_LAST);
    c_.scnt.ensure(2);
    c_.h_scnt.ensure(CNT_LAST);
    if (c_.scnt_dirty) {
      HCK(hipMemsetAsync(c_.scnt.p, 0, 2 * sizeof(unsigned long long), c_.stream));
      c_.scnt_dirty = false;
    }
  }

  // The scan's counters are read back with the first epoch's batch (no
  // synchronisation between the scan and the epoch): that epoch's device work
  // is queued assuming no wave-tile overflowed, and redone in the rare case
  // one did (scan_check).  Overflowed wave-tiles read as empty until then.
  void scan_finish() {
    meta_from_scan_ = scan_open_;
    // the side stream's work of the next epoch (tail digests) needs the scan's
    // span digests only: it waits for the scan-end event, not for one inside
    // the epoch's batch.  The last scan launch records it itself when it is
    // known to be the last (scan_upto / run_final); else it is a marker here.
    if (scan_open_) {
      if (!scan_end_recorded_) HCK(hipEventRecord(scan_end_event(), c_.stream));
      side_wait_ = scan_end_event();
      scan_end_ev_ = side_wait_;
    }
    scan_end_recorded_ = false;
    scan_checked_ = false;
  }
  // the scan's counters to h_scnt (and cleared) unless the next batch's
  // chunk-metadata kernel does it; the caller synchronises before reading
  void scan_counters_readback() {
    if (!scnt_pending_) return;
    scnt_pending_ = false;
    d2h(c_, c_.h_scnt.p, c_.scnt.p, 2);
    HCK(hipMemsetAsync(c_.scnt.p, 0, 2 * sizeof(unsigned long long), c_.stream));
  }

  // after a synchronisation that covers the scan: anchor count, scan timing,
  // and the exact rescan of overflowed wave-tiles; true if the anchors changed
  // (work queued on the provisional pool must be redone)
  bool scan_check() {
    if (scan_checked_) return false;
    if (scnt_pending_) {  // no batch took the scan's counters: read them now
      scan_counters_readback();
      sync(c_);
    }
    scan_checked_ = true;
    if ((c_.flags & ZC_FLAG_TIMING) && scan_open_) {
      float ms = 0;
      HCK(hipEventElapsedTime(&ms, c_.ev0, c_.ev1));
      c_.stats.scan_ms += ms;
    }
    scan_open_ = false;
    const uint64_t wt_lo = chk_wt_, wt_hi = nwt_done();
    chk_wt_ = wt_hi;
    const uint64_t found = c_.h_scnt[CNT_POOL];
    npool_ += found;
    c_.stats.anchors += found;
    // (the next scan launch counts from zero: the hand-off cleared them)
    if (c_.h_scnt[CNT_OVERFLOW] && wt_hi > wt_lo) {
      // wave-tiles whose anchors overflowed the scan's LDS list or their pool
      // share (dense data): count them exactly, then rescan into a side pool
      const uint64_t nw = wt_hi - wt_lo;
      std::vector<uint32_t> cnt(nw), tiles, sbase;
      d2h(c_, cnt.data(), dcnt_v() + wt_lo, nw);
      sync(c_);
      for (uint64_t t = 0; t < nw; ++t)
        if (cnt[t] == 0xFFFFFFFFu) tiles.push_back((uint32_t)(wt_lo + t));
      const uint32_t nt = (uint32_t)tiles.size();
      if (!nt) return false;
      c_.otiles.ensure(nt);
      c_.obase.ensure(nt);
      h2d(c_, c_.otiles.p, tiles.data(), nt);
      HCK(launch_anchor_rescan(d_, n_, anchor_lo_, c_.otiles.p, nullptr, nt, 0, dbase_v(), dcnt_v(), nullptr, nullptr,
                               c_.stream));
      std::vector<uint32_t> cnt2(nw);
      d2h(c_, cnt2.data(), dcnt_v() + wt_lo, nw);
      sync(c_);
      uint64_t total = 0;
      for (uint32_t t : tiles) {
        sbase.push_back((uint32_t)(side_used_ + total));
        total += cnt2[t - wt_lo];
      }
      if (side_used_ + total >= ZC_SIDE_POOL) throw ZcError{ZC_ERR_NOMEM, "anchor side pool too large"};
      npool_ += total;
      c_.stats.anchors += total;
      c_.srel.grow_keep(side_used_ + total, side_used_, c_.stream);
      c_.sg.grow_keep(side_used_ + total, side_used_, c_.stream);
      h2d(c_, c_.obase.p, sbase.data(), nt);
      HCK(launch_anchor_rescan(d_, n_, anchor_lo_, c_.otiles.p, c_.obase.p, nt, 1, dbase_v(), dcnt_v(), c_.srel.p,
                               c_.sg.p, c_.stream));
      side_used_ += total;
      return true;
    }
    return false;
  }
  bool scan_checked_ = true;
  bool scnt_pending_ = false;  // scans queued whose counters are still on the device
  bool meta_from_scan_ = false;  // ev1 marks the end of scan launches queued for this batch
  hipEvent_t side_wait_ = nullptr;  // the copy stream's next work waits for this scan end
  hipEvent_t scan_end_ev_ = nullptr;  // recorded at the last scan's end (scan_finish)

  // ---------------------------------------------------------------- epoch
  // One epoch = one grid origin r_e.  Device work is queued back to back
  // (grid-chunk metadata, anchor table, probe, anchorless compaction) and read
  // back with one synchronisation.
  bool epoch() {
    if (!scan_checked_ && c_.stats.epochs > 0) {
      sync(c_);
      scan_check();
    }
    c_.stats.epochs++;
    r_e_ = s_;
    ks_ = 0;
    grec_ = grec_valid_ = false;
    const uint64_t xs = x0();
    h_end_ = hspan_ ? std::min<uint64_t>(lim_, xs + hspan_) : lim_;
    // grid chunks cut in the rotate phase (the last W bytes are the ring at
    // finish), and before the horizon only those cut by a probe below it
    nspec_ = (n_ >= r_e_ + 2ull * W_) ? (uint32_t)((n_ - r_e_ - 2ull * W_) / W_ + 1) : 0;
    if (h_end_ < n_) {
      const uint64_t kh = h_end_ - r_e_ >= 2ull * W_ ? (h_end_ - r_e_) / W_ - 1 : 0;  // cut at r_e + (k+2)W - 1 < h_end
      nspec_ = (uint32_t)std::min<uint64_t>(nspec_, kh);
    }
    const uint32_t nsref = indexable_ ? nspec_ : 0;
    nref_ = nconf_ + nsref;
    dead_.assign(nref_, 0);
    ndead_ = 0;
    cls_.clear();
    acands_.clear();
    hcands_.clear();
    runs_.clear();
    fmap_.clear();
    fmemo_valid_ = false;
    fb_ = FBatch{};
    fb_next_ = kInf;
    has_f_ = false;
    f_min_vis_ = kInf;
    uint64_t ncand = 0, nancless = 0;
    const HistTab ht = hist_tab();
    if (nref_ || ht.tab) {
      auto tm = Clock::now();
      EpochIndex ix{};
      const bool anchors = !scan_checked_ || npool_ > 0;  // unchecked: assume some
      // sized for every ref having an anchor, at most a quarter full: the
      // inserts' CAS chains and the probe's walks stay short (at a half,
      // zc_index_insert took 36 us per 131,072 refs, at a quarter 26, and the
      // probe 69 -> 59 us; an eighth saves no more than its larger clear costs)
      uint32_t tbits = 10;
      while ((1u << tbits) < 4u * nref_) ++tbits;
      const void* const tabs0[3] = {c_.tab.p, c_.gfilt.p, c_.ckeys.p};
      if (anchors) {
        c_.cand.ensure(std::max<uint64_t>(1u << 16, nref_));
        if (nref_) {
          c_.tab.ensure(2u << tbits);
          c_.gfilt.ensure(probe_filter_words());
        }
      }
      c_.h_cnt.ensure(CNT_LAST);
      // the first epoch's grid chunks inside the scanned full tiles have their
      // keys from the scan (begin: scan_keys_), if the arrays still hold them
      const uint32_t key_from =
          scan_keys_ && r_e_ == 0 && nconf_ == 0 && c_.c_key.cap >= nref_ && c_.h_key.cap >= nsref
              ? (uint32_t)std::min<uint64_t>(nsref, tiles_done_ * ZC_STILE / W_)
              : 0u;
      if (nref_) {
        c_.c_start.ensure(nref_);
        c_.c_key.ensure(nref_);
        c_.c_fp.ensure(nref_);
        c_.c_vis.ensure(nref_);
        c_.c_anc.ensure(nref_);
        c_.c_g.ensure(nref_);
        c_.c_dead.ensure(nref_);
        c_.ancless.ensure(nref_);
        c_.h_key.ensure(nsref);
        if (nconf_) {
          h2d(c_, c_.c_start.p, cstart_.data(), nconf_);
          h2d(c_, c_.c_key.p, ckey_.data(), nconf_);
          h2d(c_, c_.c_fp.p, cfp_.data(), nconf_);
          h2d(c_, c_.c_anc.p, canc_.data(), nconf_);
          h2d(c_, c_.c_g.p, cg_.data(), nconf_);
          HCK(hipMemsetAsync(c_.c_vis.p, 0, nconf_ * sizeof(uint64_t), c_.stream));
          HCK(hipMemsetAsync(c_.c_dead.p, 0, nconf_, c_.stream));
        }
        // content classes: identical refs share one leader in the table
        c_.ckeys.ensure(1u << tbits);
        if (c_.tab.p != tabs0[0] || c_.gfilt.p != tabs0[1] || c_.ckeys.p != tabs0[2]) c_.tables_clean = false;
        c_.c_cls.ensure(nref_);
        c_.cpairs.ensure(nref_);
        ix = EpochIndex{c_.c_start.p, c_.c_vis.p, c_.c_dead.p, c_.c_key.p,
                        c_.c_g.p,     c_.c_fp.p,  c_.c_anc.p,  c_.c_cls.p,
                        c_.ckeys.p,   tbits,      anchors ? c_.tab.p : nullptr, tbits,
                        c_.gfilt.p,   c_.ancless.p, c_.counters.p, c_.cpairs.p,
                        pre_sha_n_ ? c_.h_gsha.p : nullptr, pre_sha_n_, nsref ? c_.h_key.p : nullptr};
        ix.key_from = key_from;
        ix.tables_clean = c_.tables_clean;
        c_.tables_clean = false;  // this epoch fills them
        if (scnt_pending_) {  // the chunk-metadata kernel hands the scan's counters over
          ix.scnt = c_.scnt.p;
          ix.h_scnt = c_.h_scnt.p;
          scnt_pending_ = false;
        }
        grec_valid_ = false;
        grec_ = !windowed_ && indexable_ && nsref >= kGridRecordsMin;
        // every grid key from the scan: the records can be written once the
        // scan is in (no marker inside the batch: one costs it ~6 us)
        grec_ev_ = key_from == nsref && scan_end_ev_ ? scan_end_ev_ : c_.ev_grec;
        HCK(launch_epoch_index(d_, n_, blk_v(), av(), r_e_, nconf_, nsref, W_, pow257(W_), ix, c_.stream,
                               grec_ && grec_ev_ == c_.ev_grec ? c_.ev_grec : nullptr));
        dev_r_e_ = r_e_;
        dev_nconf_ = nconf_;
        dev_nspec_ = nsref;
        dev_valid_ = true;
      } else {
        HCK(hipMemsetAsync(c_.counters.p, 0, CNT_LAST * sizeof(unsigned long long), c_.stream));
        scan_counters_readback();
      }
      const uint64_t* tab = nref_ && anchors ? c_.tab.p : nullptr;
      // ZC_FLAG_SHA1, speculative (spec_): equal-key grid pairs are joined
      // before the probe (a no-op without pairs; the count is on the device),
      // so the probe runs once, on the classes as joined
      const bool early_join = spec_ && nref_ && pre_sha_n_;
      if (early_join) HCK(launch_class_sha(nullptr, pre_sha_n_, n_, W_, ix, nref_, c_.stream));
      if (anchors)
        HCK(launch_probe(d_, av(), pwt0(), pwt1() - pwt0(), tab, tbits, c_.gfilt.p, c_.c_anc.p, c_.c_cls.p,
                         c_.c_vis.p, c_.c_dead.p, r_, h_end_, W_, ht, r_e_, nconf_, nsref, c_.cand.p, c_.cand.cap, c_.counters.p,
                         c_.stream));
      // (the grid chunks' keys reach the host from the metadata kernel itself;
      // the tail digests below need the scan's span digests)
      if (side_wait_) {
        HCK(hipStreamWaitEvent(c_.copy_stream, side_wait_, 0));
        side_wait_ = nullptr;
      }
      predict_tail();
      // what the copy stream holds now (the tail digests): waited for by this
      // event, not by querying the stream, which reported it busy ~17 us
      // after its last kernel had ended
      HCK(hipEventRecord(c_.ev_copy, c_.copy_stream));
      // the walk writes this many grid records at once: have the record team
      // spinning by the time the batch is in
      if (nsref >= kParallelRecordsMin) SpinTeam::get().arm();
      const bool first = !scan_checked_ && meta_from_scan_;  // this batch also waits for the scan
      HCK(launch_counters_out(c_.counters.p, c_.h_cnt.p, c_.stream));
      // the batch's end, waited for by this event (after the read-back kernel:
      // a marker between two kernels costs ~6 us); with timing it is ev_meta
      hipEvent_t batch_ev = c_.ev_batch;
      if (first && (c_.flags & ZC_FLAG_TIMING)) batch_ev = c_.ev_meta;
      HCK(hipEventRecord(batch_ev, c_.stream));
      // the grid SHA-1 behind the batch's read-back too: that copy runs alone
      // (beside the SHA-1 it took 14 us instead of 6), the SHA-1 a few us later
      sha_launch();
      // While the rest of the batch runs, the host writes the epoch's grid
      // records ahead, past the end of the record array, as the walk will
      // when no match comes first (it then adopts them): they need only the
      // grid keys, which the chunk-metadata kernel stores into pinned memory.
      // (Written by the device instead -- a kernel beside the batch storing
      // 5 MB into pinned memory -- they took 109 us of PCIe writes and slowed
      // the index insert from 23 to 119 us; the host has this time idle.)
      if (grec_) {
        const size_t o_e = c_.recs.size();
        c_.recs.reserve(o_e + nsref + 64);
        wait_event(grec_ev_);
        fill_grid_records(c_.recs.data() + o_e, nsref, r_e_, 0, W_, ZC_CHUNK_NEW, c_.h_key.p);
        grec_valid_ = true;
        grec_o_ = o_e;
        grec_n_ = nsref;
      }
      wait_event(batch_ev);
      wait_event(c_.ev_copy);
      if (scan_check()) {  // the pool changed under this epoch: queue it again
        c_.stats.epochs--;
        return true;
      }
      if (nref_ && c_.h_cnt[CNT_SPAIRS]) {
        // ZC_FLAG_SHA1: equal-key grid chunks whose SHA-1 the side stream
        // computes are decided by key + SHA-1 prefix, as ChunkIndex::findChunk
        // decides (chunk_index.cc:119-143) -- no byte comparison.
        // Speculatively (early_join): joined before the probe, the walk runs
        // while the SHA-1 does, and finalize_records checks every such pair's
        // prefixes once they are in (a pair that differs -- equal 64-bit keys
        // of different bytes -- redoes the stream without speculation:
        // Respeculate); else joined after the SHA-1 kernel, and the probe runs
        // again on the final classes
        const uint64_t nsp = c_.h_cnt[CNT_SPAIRS];
        if (early_join) {
          c_.h_pairs.ensure(nsp);
          d2h(c_, c_.h_pairs.p, c_.cpairs.p + (nref_ - nsp), nsp);
          sync(c_);
        } else {
          HCK(hipStreamWaitEvent(c_.stream, c_.ev_sha, 0));
          HCK(launch_class_sha(c_.h_gsha.p, pre_sha_n_, n_, W_, ix, nref_, c_.stream));
          if (anchors) {
            HCK(hipMemsetAsync(c_.counters.p + CNT_CAND, 0, sizeof(unsigned long long), c_.stream));
            HCK(launch_probe(d_, av(), pwt0(), pwt1() - pwt0(), tab, tbits, c_.gfilt.p, c_.c_anc.p, c_.c_cls.p,
                             c_.c_vis.p, c_.c_dead.p, r_, h_end_, W_, ht, r_e_, nconf_, nsref, c_.cand.p,
                             c_.cand.cap, c_.counters.p, c_.stream));
          }
          d2h(c_, c_.h_cnt.p, c_.counters.p, CNT_LAST);
          sync(c_);
        }
        if (early_join)  // the pairs to check, as grid chunk numbers
          for (uint64_t t = 0; t < nsp; ++t) {
            const uint2 pr = c_.h_pairs.p[t];
            spec_pairs_.push_back({ref_start(pr.x) / W_, ref_start(pr.y) / W_});
          }
      }
      ncand = anchors ? c_.h_cnt[CNT_CAND] : 0;
      nancless = nref_ ? c_.h_cnt[CNT_ANCLESS] : 0;
      if (nref_ && c_.h_cnt[CNT_CLASS]) load_classes();
      if (ncand > c_.cand.cap) {  // rare: rerun the probe into a buffer that fits
        c_.cand.ensure(ncand + 1024);
        HCK(hipMemsetAsync(c_.counters.p + CNT_CAND, 0, sizeof(unsigned long long), c_.stream));
        HCK(launch_probe(d_, av(), pwt0(), pwt1() - pwt0(), tab, tbits, c_.gfilt.p, c_.c_anc.p, c_.c_cls.p,
                         c_.c_vis.p, c_.c_dead.p, r_, h_end_, W_, ht, r_e_, nconf_, nsref, c_.cand.p, c_.cand.cap, c_.counters.p,
                         c_.stream));
        d2h(c_, c_.h_cnt.p, c_.counters.p, CNT_LAST);
        sync(c_);
        ncand = c_.h_cnt[CNT_CAND];
        if (ncand > c_.cand.cap) throw ZcError{ZC_ERR_NOMEM, "candidate buffer overflow persisted"};
      }
      // no probe of this epoch follows: empty the tables now, on the device
      // while the host walks (the next stream's first epoch then inserts
      // without clearing them; later epochs clear them in their own batch).
      // Not beside the grid SHA-1 (ZC_FLAG_SHA1): there the clear delayed
      // the historic registration queued behind it (hist_ms 0.26 -> 1-2.8 ms,
      // profiles/r06_sha1_clear_ab.txt); run_final clears after the SHA-1.
      if (!(c_.flags & ZC_FLAG_SHA1)) clear_tables();
      if (first && (c_.flags & ZC_FLAG_TIMING)) {  // device time from the scan's end
        float ms = 0;
        HCK(hipEventElapsedTime(&ms, c_.ev1, c_.ev_meta));
        c_.stats.meta_ms += ms;
      } else {
        c_.stats.meta_ms += ms_since(tm);
      }
    }
    if (ncand) {
      auto tp = Clock::now();
      verify_candidates(ncand);
      c_.stats.probe_ms += ms_since(tp);
    }
    // keys without an anchor, and the static index, go through the exact screen
    if (nancless) {
      std::vector<uint32_t> refs(nancless);
      d2h(c_, refs.data(), c_.ancless.p, nancless);
      sync(c_);
      std::sort(refs.begin(), refs.end());  // start order within each key
      for (uint32_t ref : refs) {
        fmap_[ref_key(ref)].push_back(ref);
        f_min_vis_ = std::min(f_min_vis_, ref_vis(ref));
      }
    }
    if (!c_.smap.empty()) f_min_vis_ = 0;
    has_f_ = !fmap_.empty() || !c_.smap.empty();
    fs_ready_ = false;
    fs_hi_ = x0();
    // by-value keys (the static index) can match anywhere: the whole epoch at
    // once; the epoch's own anchorless chunks mostly match at the grid (the
    // walk's shortcut), so their screen grows from a short first block
    fs_len_ = c_.smap.empty() ? std::max<uint64_t>(4ull << 20, 16ull * W_) : h_end_;
    grid_shortcuts();
    auto tw = Clock::now();
    bool again = walk();
    c_.stats.walk_ms += ms_since(tw);
    return again;
  }

  // An epoch that reaches the end of the stream ends, if no match comes, with
  // finish() cutting [s, n) after the last grid chunk s = r_e + nspec W: the
  // digests of those pieces are computed on the side stream with the epoch's
  // batch, so the common case needs no round trip in finalize()
  std::vector<uint64_t> pre_a_, pre_b_;
  bool pre_ready_ = false;
  void predict_tail() {
    pre_a_.clear();
    pre_b_.clear();
    pre_ready_ = false;
    if (!final_ || h_end_ < n_) return;
    const uint64_t s = nspec_ ? r_e_ + (uint64_t)nspec_ * W_ : r_e_;
    if (s >= n_) return;
    const uint64_t L = n_ - s;
    auto add = [&](uint64_t a, uint64_t b) {
      if (b - a >= 128) {
        pre_a_.push_back(a);
        pre_b_.push_back(b);
      }
    };
    if (L > W_) {
      add(s, s + W_);
      add(s + W_, n_);
    } else {
      add(s, n_);
    }
    if (pre_a_.empty()) return;
    const uint32_t nr = (uint32_t)pre_a_.size();
    // the digests go straight into pinned host memory: a copy behind the
    // kernel ran beside the batch's index insert and slowed it (18-26 us)
    c_.h_pre.ensure(nr);
    HCK(launch_range_digest_small(d_, n_, blk_v(), pre_a_.data(), pre_b_.data(), nr, c_.h_pre.p, c_.copy_stream));
    pre_ready_ = true;  // read after the epoch's copy-stream synchronisation
  }

  // wave-tiles holding the anchors of windows ending in [x0, h_end)
  uint64_t pwt0() const {
    const uint64_t xs = x0();
    return std::min<uint64_t>(nwt_done(), (xs >= W_ ? xs - W_ + 1 : 0) >> ZC_WT_SHIFT);
  }
  uint64_t pwt1() const { return std::max(pwt0(), std::min<uint64_t>(nwt_done(), ((h_end_ - 1) >> ZC_WT_SHIFT) + 1)); }

  // every probe candidate: windows of this epoch's refs byte-exact against
  // the ref's bytes; windows of historic entries by key and SHA-1 prefix,
  // as ChunkIndex::findChunk confirms them (chunk_index.cc:119-143)
  void verify_candidates(uint64_t nc) {
    c_.stats.candidates += nc;
    if (c_.nhist) {
      verify_candidates_dev(nc);
      return;
    }
    c_.h_cand.ensure(nc);
    d2h(c_, c_.h_cand.p, c_.cand.p, nc);
    sync(c_);
    verify_epoch_cands(c_.h_cand.p, nc);
  }

  // candidates of this epoch's refs (hc[0, m), all pad 0) -> acands_
  void verify_epoch_cands(const Cand* hc, uint64_t m) {
    // a window that is exactly a grid chunk of this epoch in the candidate's
    // class is already known equal (the class was byte-verified)
    std::vector<uint64_t> wa, ra;
    std::vector<uint64_t> idx;
    std::vector<uint8_t>& ok = c_.res_ok;
    ok.assign(m, 1);
    for (uint64_t i = 0; i < m; ++i) {
      const uint64_t ws = hc[i].p - W_ + 1;
      if (!cls_.empty() && ws >= r_e_ && wmod(ws - r_e_) == 0 && wdiv(ws - r_e_) < nref_ - nconf_) {
        const uint32_t r = nconf_ + (uint32_t)wdiv(ws - r_e_);
        if (cls_[r] == hc[i].ref) continue;
      }
      wa.push_back(ws);
      ra.push_back(ref_start(hc[i].ref));
      idx.push_back(i);
    }
    std::vector<uint8_t> vok = verify_pairs(wa, ra, W_);
    for (size_t j = 0; j < idx.size(); ++j) ok[idx[j]] = vok[j];
    acands_.reserve(acands_.size() + m);
    for (uint64_t i = 0; i < m; ++i)
      if (ok[i]) acands_.push_back({hc[i].p, hc[i].ref});
    sort_by_position(acands_);
  }

  // With a historic index the candidates are split on the device: the epoch's
  // come back as a list of their own, the historic ones key-checked and in
  // position order (launch_cand_order), so the host reads each once, in order
  void verify_candidates_dev(uint64_t nc) {
    if (nc > 0xFFFFFFF0ull) throw ZcError{ZC_ERR_NOMEM, "too many probe candidates"};
    // buckets of ~n / (2 nc) positions: a few candidates each at most
    // (at most 2^20 buckets: the scan's block sums fit one workgroup)
    uint32_t bshift = 0;
    const uint64_t nb_max = std::min<uint64_t>(std::max<uint64_t>(2 * nc, 1024), 1u << 20);
    while (bshift < 63 && (n_ >> bshift) + 1 > nb_max) ++bshift;
    const uint32_t nb = (uint32_t)((n_ >> bshift) + 1);
    // the bucket counts and the call counters stay zero between calls (the
    // kernels clear them): filled only when (re)made
    if (c_.co_bcnt.cap < nb || !c_.co_bcnt.p) {
      c_.co_bcnt.ensure(std::max<uint64_t>(nb, 1u << 16));
      HCK(hipMemsetAsync(c_.co_bcnt.p, 0, c_.co_bcnt.cap * sizeof(uint32_t), c_.stream));
    }
    if (!c_.co_hc.p) {
      c_.co_hc.ensure(4);
      HCK(hipMemsetAsync(c_.co_hc.p, 0, 4 * sizeof(unsigned long long), c_.stream));
    }
    c_.co_boff.ensure((uint64_t)nb + 1);
    c_.co_bsum.ensure((uint64_t)nb / 1024 + 2);
    c_.co_rank.ensure(nc);
    c_.co_out0.ensure(nc);
    c_.co_out.ensure(nc);
    c_.h_co_hc.ensure(4);
    c_.h_cand.ensure(nc);
    c_.h_hist_cand.ensure(nc);
    const CandOrderBufs b{bshift,       nb,          c_.co_bcnt.p,  c_.co_boff.p,       c_.co_bsum.p,
                          c_.co_rank.p, c_.co_out0.p, c_.co_out.p, c_.co_hc.p,         c_.h_cand.p,
                          c_.h_hist_cand.p, c_.h_co_hc.p};
    HCK(launch_cand_order(d_, blk_v(), c_.cand.p, (uint32_t)nc, c_.hkey_d.p, pow257(W_), W_, n_,
                          pre_sha_n_ ? pre_sha_n_ : 0, b, c_.stream));
    sync(c_);
    const uint64_t n0 = c_.h_co_hc[3], nk = c_.h_co_hc[1];
    const bool unsorted = c_.h_co_hc[2] != 0;
    if (n0) verify_epoch_cands(c_.h_cand.p, n0);
    if (!nk) return;
    Cand* const hk = c_.h_hist_cand.p;
    if (unsorted) std::stable_sort(hk, hk + nk, [](const Cand& x, const Cand& y) { return x.p < y.p; });
    // the windows that are no grid chunk of the side stream's SHA-1 pass
    // (pad 2) are hashed here, in batches; the rest are grid chunks: joined on
    // the key now and checked when the digests land (speculation, whole-stream
    // SHA-1 mode), or compared with the grid digests
    std::vector<uint64_t> sa;
    std::vector<uint32_t> sl;
    for (uint64_t i = 0; i < nk; ++i)
      if (hk[i].pad == 2) sa.push_back(hk[i].p + 1 - W_);
    std::vector<uint8_t> sh;
    if (!sa.empty()) {
      sh.resize(20 * sa.size());
      for (size_t off = 0; off < sa.size(); off += kFBatchMax) {
        const size_t m = std::min(sa.size() - off, kFBatchMax);
        const std::vector<uint64_t> pa(sa.begin() + off, sa.begin() + off + m);
        sl.assign(m, W_);
        const std::vector<uint8_t> part = sha1s(pa, sl);
        memcpy(&sh[20 * off], part.data(), part.size());
      }
    }
    hcands_.reserve(hcands_.size() + nk);
    if (spec_) spec_hist_.reserve(spec_hist_.size() + nk);
    size_t js = 0;
    for (uint64_t i = 0; i < nk; ++i) {
      const Cand& k = hk[i];
      const uint8_t* pre = &c_.hsha[16 * (size_t)k.ref];
      if (k.pad == 2) {
        if (memcmp(&sh[20 * js++], pre, 16) == 0) hcands_.push_back({k.p, k.ref});
        continue;
      }
      const uint64_t ws = k.p + 1 - W_;
      if (spec_ && grid_sha_pending(ws)) {
        hcands_.push_back({k.p, k.ref});
        spec_hist_.push_back({wdiv(ws), k.ref});
      } else if (const uint8_t* g = grid_sha_of(ws)) {
        if (memcmp(g, pre, 16) == 0) hcands_.push_back({k.p, k.ref});
      }
    }
  }

  // LSD radix sort by window end (11-bit digits, stable).  Candidates with the
  // same end are windows equal to refs of equal content, so their relative
  // order does not change the walk.
  void sort_by_position(std::vector<ACand>& v) {
    const size_t m = v.size();
    if (m < 2) return;
    std::vector<ACand>& tmp = c_.res_sort_tmp;
    tmp.resize(m);
    uint32_t bits = 1;
    while (bits < 64 && (n_ >> bits)) ++bits;
    std::vector<uint32_t> cnt(2048);
    for (uint32_t shift = 0; shift < bits; shift += 11) {
      std::fill(cnt.begin(), cnt.end(), 0u);
      for (const ACand& a : v) ++cnt[(a.p >> shift) & 2047];
      uint32_t sum = 0;
      for (uint32_t& c : cnt) {
        const uint32_t t = c;
        c = sum;
        sum += t;
      }
      for (const ACand& a : v) tmp[cnt[(a.p >> shift) & 2047]++] = a;
      v.swap(tmp);
    }
  }

  std::vector<uint8_t> verify_pairs(const std::vector<uint64_t>& wa, const std::vector<uint64_t>& ra,
                                    uint32_t len) {
    const size_t np = wa.size();
    std::vector<uint8_t> ok(np, 0);
    if (!np) return ok;
    c_.va.ensure(np);
    c_.vb.ensure(np);
    c_.vok.ensure(np);
    h2d(c_, c_.va.p, wa.data(), np);
    h2d(c_, c_.vb.p, ra.data(), np);
    HCK(launch_verify_pairs(d_, c_.va.p, c_.vb.p, len, (uint32_t)np, c_.vok.p, c_.stream));
    d2h(c_, ok.data(), c_.vok.p, np);
    sync(c_);
    return ok;
  }

  std::vector<uint64_t> range_digests(const std::vector<uint64_t>& a, const std::vector<uint64_t>& b) {
    const size_t nr = a.size();
    std::vector<uint64_t> out(nr);
    if (!nr) return out;
    c_.va.ensure(nr);
    c_.vb.ensure(nr);
    c_.dout.ensure(nr);
    c_.h_ra.ensure(nr);
    c_.h_rb.ensure(nr);
    c_.h_rout.ensure(nr);
    memcpy(c_.h_ra.p, a.data(), nr * sizeof(uint64_t));
    memcpy(c_.h_rb.p, b.data(), nr * sizeof(uint64_t));
    h2d(c_, c_.va.p, c_.h_ra.p, nr);
    h2d(c_, c_.vb.p, c_.h_rb.p, nr);
    HCK(launch_range_digest(d_, n_, blk_v(), c_.va.p, c_.vb.p, (uint32_t)nr, c_.dout.p, c_.stream));
    d2h(c_, c_.h_rout.p, c_.dout.p, nr);
    sync(c_);
    memcpy(out.data(), c_.h_rout.p, nr * sizeof(uint64_t));
    return out;
  }

  // RollingHash digests of the W-byte windows [a[i], a[i] + W), in pinned
  // memory (valid until the next range digest)
  const uint64_t* window_digests(const std::vector<uint64_t>& a) {
    const size_t nr = a.size();
    c_.va.ensure(nr);
    c_.vb.ensure(nr);
    c_.dout.ensure(nr);
    c_.h_ra.ensure(nr);
    c_.h_rb.ensure(nr);
    c_.h_rout.ensure(nr);
    for (size_t i = 0; i < nr; ++i) {
      c_.h_ra.p[i] = a[i];
      c_.h_rb.p[i] = a[i] + W_;
    }
    h2d(c_, c_.va.p, c_.h_ra.p, nr);
    h2d(c_, c_.vb.p, c_.h_rb.p, nr);
    HCK(launch_range_digest(d_, n_, blk_v(), c_.va.p, c_.vb.p, (uint32_t)nr, c_.dout.p, c_.stream));
    d2h(c_, c_.h_rout.p, c_.dout.p, nr);
    sync(c_);
    return c_.h_rout.p;
  }

  std::vector<uint8_t> sha1s(const std::vector<uint64_t>& a, const std::vector<uint32_t>& len) {
    const size_t nr = a.size();
    std::vector<uint8_t> out(nr * 20);
    if (!nr) return out;
    c_.va.ensure(nr);
    c_.vlen.ensure(nr);
    c_.sha_out.ensure(nr * 20);
    h2d(c_, c_.va.p, a.data(), nr);
    h2d(c_, c_.vlen.p, len.data(), nr);
    HCK(launch_sha1(d_, c_.va.p, c_.vlen.p, (uint32_t)nr, c_.sha_out.p, c_.stream));
    d2h(c_, out.data(), c_.sha_out.p, nr * 20);
    sync(c_);
    return out;
  }

  // ---------------------------------------------------------------- F screen
  // Key sets beyond the LDS (kLdsKeys) take the Bloom mode: the staged
  // screen tests a 4 MiB Bloom filter in L2 at every position, and its runs
  // are trimmed on the device to positions whose exact 64-bit key is in the
  // set before they come back (the filter's false hits never reach the walk)
  static constexpr size_t kLdsKeys = 2048;
  void fscan_setup() {
    keys32_.clear();
    std::vector<uint32_t>& keys32 = keys32_;
    for (auto& kv : fmap_) keys32.push_back((uint32_t)kv.first);
    bloom_ = W_ >= 32 && n_ >= 64 && !(c_.flags & ZC_FLAG_NO_STAGED_SCREEN) &&
                       c_.smap.size() + fmap_.size() > kLdsKeys;
    const bool bloom = bloom_;
    if (!bloom)
      for (auto& kv : c_.smap) keys32.push_back((uint32_t)kv.first);
    std::sort(keys32.begin(), keys32.end());
    keys32.erase(std::unique(keys32.begin(), keys32.end()), keys32.end());
    nf_ = bloom ? (uint32_t)(c_.smap.size() + keys32.size()) : (uint32_t)keys32.size();
    const uint32_t nf = nf_;
    c_.f32.ensure(std::max<size_t>(keys32.size(), 1));
    h2d(c_, c_.f32.p, keys32.data(), keys32.size());
    c_.fbits.ensure(1u << 14);
    bloom_p_ = nullptr;
    chk_p_ = nullptr;
    if (bloom) {
      statics_screen(c_);
      std::vector<uint32_t> bits = c_.sc_fbits;
      for (uint32_t h : keys32) bits[h >> 18] |= 1u << ((h >> 13) & 31);
      h2d(c_, c_.fbits.p, bits.data(), bits.size());
      bloom_p_ = c_.bloom_s.p;
      chk_p_ = c_.bloom_one ? c_.chk_s.p : nullptr;
      std::vector<uint64_t> fk;
      for (auto& kv : fmap_) fk.push_back(kv.first);
      std::sort(fk.begin(), fk.end());
      c_.flist.ensure(std::max<size_t>(fk.size(), 1));
      h2d(c_, c_.flist.p, fk.data(), fk.size());
      flist_n_ = (uint32_t)fk.size();
      if (!fk.empty()) {  // the epoch's keys join a copy of the set's filter
        c_.bloom_w.ensure(bloom_words(c_.bloom_bits));
        HCK(hipMemcpyAsync(c_.bloom_w.p, c_.bloom_s.p, sizeof(uint32_t) * bloom_words(c_.bloom_bits),
                           hipMemcpyDeviceToDevice, c_.stream));
        HCK(launch_bloom_add(c_.bloom_w.p, c_.bloom_bits, c_.flist.p, (uint32_t)fk.size(), c_.stream));
        bloom_p_ = c_.bloom_w.p;
        if (c_.bloom_one) {  // and a copy of the check table
          for (;;) {
            const size_t nw = ((1ull << c_.chk_bits) + kChkPad) * 4;
            c_.chk_w.ensure(nw);
            HCK(hipMemcpyAsync(c_.chk_w.p, c_.chk_s.p, sizeof(uint16_t) * nw, hipMemcpyDeviceToDevice, c_.stream));
            HCK(hipMemsetAsync(c_.chk_ovf.p, 0, sizeof(unsigned int), c_.stream));
            HCK(launch_chk_add(c_.chk_w.p, c_.chk_bits, c_.flist.p, (uint32_t)fk.size(), c_.chk_ovf.p, c_.stream));
            unsigned int ovf = 0;
            d2h(c_, &ovf, c_.chk_ovf.p, 1);
            sync(c_);
            if (!ovf) break;
            // the epoch's keys did not fit: rebuild the set's table with room
            // for them (the one-level screen stays: the two-level one's filter
            // is sized for other key counts) and add them again
            c_.chk_room = std::max<uint64_t>(2 * c_.chk_room, 2 * fk.size());
            c_.sc_ver = 0;
            statics_screen(c_);
            ++c_.stats.chk_rebuilds;
          }
          chk_p_ = c_.chk_w.p;
        }
      }
    } else if (nf > 16) {
      std::vector<uint32_t> bits(1u << 14, 0);
      for (uint32_t h : keys32) bits[h >> 18] |= 1u << ((h >> 13) & 31);
      h2d(c_, c_.fbits.p, bits.data(), bits.size());
    }
  }

  // screen positions [p_start, p_end) and append their runs to runs_
  void fscan_range(uint64_t p_start, uint64_t p_end) {
    const std::vector<uint32_t>& keys32 = keys32_;
    const bool bloom = bloom_;
    const uint32_t nf = nf_;
    const uint32_t* bloom_p = bloom_p_;
    if (p_start >= p_end) return;
    const uint32_t pw32 = (uint32_t)pow257(W_);
    const uint64_t ntiles = (p_end + ZC_TILE - 1) / ZC_TILE;  // zc_fscan tiles up to the horizon
    // the staged kernel screens wave-tiles [wt_lo, wt_hi) (the whole range
    // from p_start to the end); zc_fscan redoes wave-tiles whose runs
    // overflowed, or everything when the staged kernel does not apply
    const uint64_t t_first = p_start / ZC_TILE;
    // the staged kernel's wave walks a 512 KiB wave-tile (~0.5 ms); short
    // ranges (the walk's first blocks) take the lane-per-KiB kernel
    const bool staged = W_ >= 32 && n_ >= 64 && !(c_.flags & ZC_FLAG_NO_STAGED_SCREEN) &&
                        p_end - p_start > (64ull << 20);
    const uint64_t wt_lo = staged ? p_start / ZC_FWT : 0;
    const uint64_t wt_hi = staged ? (p_end + ZC_FWT - 1) / ZC_FWT : 0;
    constexpr uint64_t kTpw = ZC_FWT / ZC_TILE;  // zc_fscan tiles per screen wave-tile
    // the per-tile lists are indexed by absolute tile, biased by the window base
    const uint64_t tb = wbase_ / ZC_TILE, wb = wbase_ / ZC_FWT;
    c_.ftile_off.ensure(ntiles - tb + 1);
    c_.ftile_cnt.ensure(ntiles - tb + 1);
    c_.fwt_off.ensure(std::max<uint64_t>(wt_hi, wb + 1) - wb);
    c_.fwt_cnt.ensure(std::max<uint64_t>(wt_hi, wb + 1) - wb);
    uint64_t* const ftile_off_v = c_.ftile_off.p - tb;
    uint32_t* const ftile_cnt_v = c_.ftile_cnt.p - tb;
    uint64_t* const fwt_off_v = c_.fwt_off.p - wb;
    uint32_t* const fwt_cnt_v = c_.fwt_cnt.p - wb;
    if (staged && nf > 4) {
      std::vector<uint32_t> map17(1u << 12, 0);
      for (uint32_t h : keys32) map17[(h >> 15) >> 5] |= 1u << ((h >> 15) & 31);
      c_.fbits17.ensure(map17.size());
      h2d(c_, c_.fbits17.p, map17.data(), map17.size());
    }
    uint64_t cap = std::max<uint64_t>((ntiles - t_first) * 4, 1u << 16);
    unsigned long long cnt[CNT_LAST];
    auto old_screen = [&](uint64_t t0, uint64_t t1) {
      t0 = std::max(t0, t_first);
      t1 = std::min(t1, ntiles);
      if (t1 > t0)
        HCK(launch_fscan(d_, n_, blk_v(), W_, pw32, p_start, p_end, t0, t1 - t0, c_.f32.p, nf, c_.fbits.p,
                         bloom_p, c_.bloom_bits, c_.runs.p, c_.runs.cap, ftile_off_v, ftile_cnt_v, c_.counters.p, c_.stream));
    };
    std::vector<uint32_t> wcnt(wt_hi - wt_lo);
    for (int attempt = 0; attempt < 3; ++attempt) {
      c_.runs.ensure(cap);
      HCK(hipMemsetAsync(c_.counters.p, 0, CNT_LAST * sizeof(unsigned long long), c_.stream));
      if (staged && bloom) {
        HCK(launch_fscan_staged_bloom(d_, n_, blk_v(), W_, pw32, p_start, p_end, wt_lo, wt_hi - wt_lo, bloom_p,
                                      c_.bloom_bits, chk_p_, c_.chk_bits, c_.runs.p, c_.runs.cap, fwt_off_v,
                                      fwt_cnt_v, c_.counters.p, c_.stream));
      } else if (staged) {
        HCK(launch_fscan_staged(d_, n_, blk_v(), W_, pw32, p_start, p_end, wt_lo, wt_hi - wt_lo, keys32.data(),
                                c_.f32.p, nf, c_.fbits17.p, c_.runs.p, c_.runs.cap, fwt_off_v, fwt_cnt_v,
                                c_.counters.p, c_.stream));
      }
      if (staged) {
        d2h(c_, wcnt.data(), fwt_cnt_v + wt_lo, wcnt.size());
        sync(c_);
        // wave-tiles whose runs overflowed the lane slots: redo with zc_fscan,
        // one launch per stretch of consecutive ones; a launch costs about the
        // same for any number of tiles (a lane walks 1 KiB), so past 64
        // stretches everything from the first to the last overflowed
        // wave-tile is redone in one launch
        std::vector<std::pair<uint64_t, uint64_t>> st;
        for (uint64_t i = 0; i < wcnt.size();) {
          if (wcnt[i] != ZC_FWT_OVERFLOW) {
            ++i;
            continue;
          }
          uint64_t j = i + 1;
          while (j < wcnt.size() && wcnt[j] == ZC_FWT_OVERFLOW) ++j;
          st.push_back({i, j});
          i = j;
        }
        if (st.size() > 64) {
          for (uint64_t i = st.front().first; i < st.back().second; ++i) wcnt[i] = ZC_FWT_OVERFLOW;
          st = {{st.front().first, st.back().second}};
        }
        for (const auto& r : st) old_screen((wt_lo + r.first) * kTpw, (wt_lo + r.second) * kTpw);
      } else {
        old_screen(t_first, ntiles);
      }
      d2h(c_, cnt, c_.counters.p, CNT_LAST);
      sync(c_);
      if (!cnt[CNT_FOVF]) break;
      cap = cnt[CNT_RUNS] + 1024;
      if (attempt == 2) throw ZcError{ZC_ERR_NOMEM, "screen-run buffer overflow persisted"};
    }
    const uint64_t nruns = cnt[CNT_RUNS];
    c_.stats.fscan_runs += nruns;
    if (bloom)
      HCK(launch_key64_filter(d_, blk_v(), W_, pow257(W_), c_.runs.p, nruns, c_.kset.p, c_.kset_bits, c_.kset_zero,
                              c_.flist.p, flist_n_, c_.stream));
    // zc_fscan's per-tile lists are read only where it ran
    bool old_ran = !staged;
    for (uint32_t c : wcnt) old_ran |= c == ZC_FWT_OVERFLOW;
    c_.h_runs.ensure(nruns);
    const Run* const raw = c_.h_runs.p;
    std::vector<uint64_t> toff(old_ran ? ntiles - t_first : 0), woff(wcnt.size());
    std::vector<uint32_t> tcnt(old_ran ? ntiles - t_first : 0);
    d2h(c_, c_.h_runs.p, c_.runs.p, nruns);
    if (old_ran) {
      d2h(c_, toff.data(), ftile_off_v + t_first, ntiles - t_first);
      d2h(c_, tcnt.data(), ftile_cnt_v + t_first, ntiles - t_first);
    }
    d2h(c_, woff.data(), fwt_off_v + wt_lo, woff.size());
    sync(c_);
    auto take = [&](const Run* q, uint64_t k) {
      for (uint64_t i = 0; i < k; ++i) {
        if (q[i].end <= q[i].start) continue;  // emptied by the 64-bit filter
        if (!runs_.empty() && runs_.back().end == q[i].start)
          runs_.back().end = q[i].end;
        else
          runs_.push_back(q[i]);
      }
    };
    auto take_tiles = [&](uint64_t t0, uint64_t t1) {
      for (uint64_t t = std::max(t0, t_first); t < std::min(t1, ntiles); ++t)
        take(&raw[toff[t - t_first]], tcnt[t - t_first]);
    };
    if (!staged) take_tiles(t_first, ntiles);
    for (uint64_t i = 0; i < wcnt.size(); ++i) {
      if (wcnt[i] == ZC_FWT_OVERFLOW)
        take_tiles((wt_lo + i) * kTpw, (wt_lo + i + 1) * kTpw);
      else
        take(&raw[woff[i]], wcnt[i]);
    }
  }
  std::vector<uint32_t> keys32_;
  bool bloom_ = false;
  uint32_t nf_ = 0;
  const uint32_t* bloom_p_ = nullptr;
  const uint16_t* chk_p_ = nullptr;  // the one-level screen's check table, or none
  // the screen runs lazily: positions [x0, fs_hi_) are screened so far, in
  // blocks of fs_len_ bytes (doubling) as the walk needs them
  bool fs_ready_ = false;
  uint64_t fs_hi_ = 0, fs_len_ = 0;
  static constexpr uint64_t kFewPositions = 8;  // one fbatch (its first 8 positions per run)

  // first position p >= from inside the screen runs, or kInf
  size_t irun_ = 0;
  uint64_t next_run_pos(uint64_t from) {
    while (irun_ < runs_.size() && runs_[irun_].end <= from) ++irun_;
    if (irun_ == runs_.size()) return kInf;
    return std::max(from, runs_[irun_].start);
  }

  // is window [ws, ws + W) known to equal ref without reading it?  It is when
  // the window is a grid chunk of this epoch in ref's content class (classes
  // are byte-verified on the device)
  bool known_equal(uint64_t ws, uint32_t ref) const {
    if (!indexable_ || ws < r_e_ || (ws - r_e_) % W_) return false;
    const uint64_t j = (ws - r_e_) / W_;
    if (j >= nspec_) return false;
    const uint32_t g = nconf_ + (uint32_t)j;
    if (g == ref) return true;
    return !cls_.empty() && cls_[g] == cls_[ref];
  }

  // first alive ref with key h visible at p (start order; vis grows with start)
  int64_t first_alive_ref(uint64_t h, uint64_t p) {
    // consecutive screen hits mostly share one key (runs of repeated content)
    if (!fmemo_valid_ || fmemo_key_ != h) {
      fmemo_it_ = fmap_.find(h);
      fmemo_key_ = h;
      fmemo_valid_ = true;
    }
    auto it = fmemo_it_;
    if (it == fmap_.end()) return -1;
    for (uint32_t ref : it->second) {
      if (ref_vis(ref) > p) break;
      if (class_alive_visible(ref, p)) return ref;
    }
    return -1;
  }

  uint64_t fb_take_ = 8, fb_next_ = kInf;
  void build_fbatch(uint64_t p0) {
    const auto t0 = Clock::now();
    FBatch b;
    // predicted positions: the first 8 positions of every screen run from p0
    // on (p0, p0+1.. in case p0 fails; and every later run when the runs are
    // many short false hits of a large static index: one batch for all of
    // them), then the success chain p0+W, p0+2W, ... restricted to the runs
    size_t save = irun_;
    std::vector<uint64_t> pos;
    uint64_t q = p0;
    {
      size_t ir = irun_;
      while (ir < runs_.size() && runs_[ir].end <= p0) ++ir;
      // a run whose positions keep failing (content with no live match, e.g.
      // a long repeated run whose refs were consumed) takes 8x more of its
      // positions per batch each time the walk comes back right after them
      fb_take_ = p0 == fb_next_ ? std::min<uint64_t>(fb_take_ * 8, 1u << 16) : 8;
      fb_next_ = kInf;
      for (; ir < runs_.size() && pos.size() < kFBatchMax / 2; ++ir) {
        const uint64_t a = std::max(p0, runs_[ir].start);
        const uint64_t b = std::min(runs_[ir].end, a + (fb_next_ == kInf ? fb_take_ : 8));
        if (fb_next_ == kInf) fb_next_ = b;
        for (uint64_t x = a; x < b; ++x) pos.push_back(x);
      }
    }
    q = p0 + W_;
    while (pos.size() < kFBatchMax) {
      q = next_run_pos(q);
      if (q == kInf) break;
      pos.push_back(q);
      q += W_;
    }
    irun_ = save;
    // two ascending lists (the neighbours of p0, then the success chain):
    // merge them, dropping duplicates
    {
      size_t k = 0;
      while (k + 1 < pos.size() && pos[k] < pos[k + 1]) ++k;
      std::vector<uint64_t> m;
      m.reserve(pos.size());
      std::merge(pos.begin(), pos.begin() + k + 1, pos.begin() + k + 1, pos.end(), std::back_inserter(m));
      m.erase(std::unique(m.begin(), m.end()), m.end());
      pos.swap(m);
    }
    const size_t np = pos.size();
    std::vector<uint64_t> a(np), e(np);
    for (size_t i = 0; i < np; ++i) {
      a[i] = pos[i] - W_ + 1;
      e[i] = pos[i] + 1;
    }
    b.h = range_digests(a, e);
    b.pos = std::move(pos);
    b.vref.assign(np, -1);
    b.vok.assign(np, 0);
    const bool statics = !c_.smap.empty();
    b.has_sha.assign(statics ? np : 0, 0);
    b.sha.assign(statics ? np * 20 : 0, 0);
    std::vector<uint64_t> wa, ra;
    std::vector<size_t> widx;
    std::vector<uint64_t> sa;
    std::vector<uint32_t> sl;
    std::vector<size_t> sidx;
    for (size_t i = 0; i < np; ++i) {
      int64_t ref = first_alive_ref(b.h[i], b.pos[i]);
      if (ref >= 0) {
        b.vref[i] = ref;
        if (known_equal(a[i], (uint32_t)ref)) {
          b.vok[i] = 1;
        } else {
          wa.push_back(a[i]);
          ra.push_back(ref_start(ref));
          widx.push_back(i);
        }
      }
      if (statics && c_.smap.count(b.h[i])) {
        sa.push_back(a[i]);
        sl.push_back(W_);
        sidx.push_back(i);
      }
    }
    std::vector<uint8_t> ok = verify_pairs(wa, ra, W_);
    for (size_t j = 0; j < widx.size(); ++j) b.vok[widx[j]] = ok[j];
    std::vector<uint8_t> sh = sha1s(sa, sl);
    for (size_t j = 0; j < sidx.size(); ++j) {
      b.has_sha[sidx[j]] = 1;
      memcpy(&b.sha[sidx[j] * 20], &sh[j * 20], 20);
    }
    fb_ = std::move(b);
    c_.stats.fbatch_ms += ms_since(t0);
  }

  // Is p an F match?  Returns the matched key via *key.
  bool eval_f(uint64_t p, uint64_t* key) {
    while (fb_.cur < fb_.pos.size() && fb_.pos[fb_.cur] < p) ++fb_.cur;
    if (fb_.cur == fb_.pos.size() || fb_.pos[fb_.cur] != p) build_fbatch(p);
    const size_t i = fb_.cur;
    const uint64_t h = fb_.h[i];
    *key = h;
    // the batch's witness is still in the index: the common case
    if (fb_.vref[i] >= 0 && fb_.vok[i] && class_alive_visible((uint32_t)fb_.vref[i], p)) return true;
    // in-stream anchorless chunks: content equality with an alive visible ref
    auto it = fmap_.find(h);
    if (it != fmap_.end()) {
      for (uint32_t ref : it->second) {
        if (ref_vis(ref) > p) break;
        if (!class_alive_visible(ref, p)) continue;
        bool ok;
        if (fb_.vref[i] == (int64_t)ref) {
          ok = fb_.vok[i];
        } else if (known_equal(p - W_ + 1, ref)) {
          ok = true;
        } else {
          std::vector<uint64_t> wa{p - W_ + 1}, ra{ref_start(ref)};
          ok = verify_pairs(wa, ra, W_)[0];
        }
        if (ok) return true;
      }
    }
    // static index entries: SHA-1 prefix of the window (chunk_index.cc:130-139)
    auto st = c_.smap.find(h);
    if (st != c_.smap.end()) {
      if (!fb_.has_sha[i]) {
        std::vector<uint64_t> sa{p - W_ + 1};
        std::vector<uint32_t> sl{W_};
        std::vector<uint8_t> sh = sha1s(sa, sl);
        memcpy(&fb_.sha[i * 20], sh.data(), 20);
        fb_.has_sha[i] = 1;
      }
      for (uint32_t si : st->second)
        if (memcmp(c_.statics[si].sha, &fb_.sha[i * 20], 16) == 0) return true;
    }
    return false;
  }

  // the first screen position in [x, limit) that matches, or kInf; screens
  // further as it goes (the runs below fs_hi_ are known)
  uint64_t next_f(uint64_t x, uint64_t limit, uint64_t* key) {
    if (!has_f_) return kInf;
    uint64_t p = std::max(x, f_min_vis_);
    limit = std::min(limit, h_end_);
    for (;;) {
      if (p >= limit) return kInf;
      const uint64_t q = next_run_pos(p);
      if (q != kInf) {
        if (q >= limit) return kInf;
        if (eval_f(q, key)) return q;
        p = q + 1;
        continue;
      }
      if (fs_hi_ >= limit) return kInf;
      const uint64_t lo = std::max(fs_hi_, p);
      if (limit - lo <= kFewPositions) {
        // a few positions (the walk's next candidate is close): each one is
        // checked by eval_f's exact 64-bit key instead of a screen launch
        runs_.push_back(Run{lo, limit});
        fs_hi_ = limit;
        continue;
      }
      auto tf = Clock::now();
      if (!fs_ready_) {
        fscan_setup();
        fs_ready_ = true;
      }
      const uint64_t hi = std::min(h_end_, lo + fs_len_);
      fscan_range(lo, hi);
      fs_hi_ = hi;
      fs_len_ *= 4;
      c_.stats.fscan_ms += ms_since(tf);
    }
  }

  // Grid chunks of this epoch that are not the leader of their content class:
  // the window that IS such a chunk matches at its end whenever a member of
  // its class is in the index by then (cut earlier, or confirmed) and not
  // consumed -- the earliest probe there, found without the probe's or the
  // screen's candidates (the probe leaves those candidates out).  The walk
  // takes them in order.
  std::vector<uint32_t> sc_list_;
  size_t isc_ = 0;
  void grid_shortcuts() {
    sc_list_.clear();
    isc_ = 0;
    if (cls_.empty()) return;
    for (uint32_t j = 0; j < nspec_; ++j)
      if (cls_[nconf_ + j] != nconf_ + j) sc_list_.push_back(j);
  }
  // the next grid window end >= x that matches (its grid chunk via *g), or kInf
  uint64_t next_grid(uint64_t x, uint32_t* g) {
    while (isc_ < sc_list_.size()) {
      const uint32_t j = sc_list_[isc_];
      const uint64_t pg = r_e_ + (uint64_t)(j + 1) * W_ - 1;
      if (pg >= h_end_) return kInf;
      if (pg >= x) {
        const uint32_t gr = nconf_ + j;
        // (gr itself may be consumed -- then x is past pg -- or abandoned by a
        // grid shift: its window still equals its class.)  Consumption only
        // grows, so a class not in the index at pg now never will be
        if (class_alive_visible(cls_[gr], pg)) {
          *g = gr;
          return pg;
        }
      }
      ++isc_;
    }
    return kInf;
  }

  // ---------------------------------------------------------------- walk

  // the runs of records fill_grid_records wrote since the last finalize:
  // records rec0 .. rec0 + n - 1 are [off0 + j W, off0 + (j + 1) W), one kind;
  // finalize_records classifies them without reading them back
  struct GridRun {
    size_t rec0;
    uint64_t n, off0;
    uint32_t kind;
  };
  std::vector<GridRun> gruns_;

  void push(uint64_t off, uint32_t size, uint32_t kind, uint64_t rolling) {
    zc_record r;
    memset(&r, 0, sizeof r);
    r.offset = off;
    r.size = size;
    r.kind = kind;
    r.rolling = rolling;
    c_.recs.push_back(r);
  }

  // a cut piece [a, b) saved via saveChunkToSave (digest filled in later)
  void piece(uint64_t a, uint64_t b) {
    const uint32_t len = (uint32_t)(b - a);
    if (len < 128) {
      push(a, len, ZC_BYTES, 0);
    } else {
      need_digest_.push_back({c_.recs.size(), a, b});
      push(a, len, ZC_CHUNK_NEW, 0);
    }
  }

  // the grid records of this epoch written ahead (epoch()): grid chunk k's
  // record at index grec_o_ + k, k < grec_n_
  static constexpr uint32_t kGridRecordsMin = 16384;
  bool grec_ = false;  // this epoch's grid records are written ahead
  bool grec_valid_ = false;
  size_t grec_o_ = 0;
  uint32_t grec_n_ = 0;

  // save the grid chunks of this epoch whose cut happens at or before probe m
  // (chunk k is cut at r_e + (k+2)W - 1); the records are written in place,
  // the common case being every grid chunk of the stream at once
  void save_grid_until(uint64_t m) {
    if (ks_ >= nspec_ || r_e_ + 2ull * W_ - 1 > m) return;
    const uint64_t kmax = std::min<uint64_t>(nspec_, (m - (r_e_ + 2ull * W_ - 1)) / W_ + 1);
    if (ks_ >= kmax) return;
    size_t o = c_.recs.size();
    c_.recs.resize(o + (kmax - ks_));
    zc_record* rec = c_.recs.data();
    const uint32_t kind = indexable_ ? (uint32_t)ZC_CHUNK_NEW : (uint32_t)ZC_BYTES;
    const uint8_t* dead = indexable_ ? dead_.data() + nconf_ : nullptr;
    if (ndead_ == 0 && r_e_ + ks_ * W_ >= s_ && kmax - ks_ >= kParallelRecords) {
      // every chunk of the run is saved: record o + j is grid chunk ks_ + j --
      // as written ahead, when record o is where chunk ks_ was put
      if (!(grec_valid_ && o == grec_o_ + ks_ && kmax <= grec_n_))
        fill_grid_records(rec + o, kmax - ks_, r_e_, ks_, W_, kind, indexable_ ? c_.h_key.p : nullptr);
      gruns_.push_back({o, kmax - ks_, r_e_ + ks_ * W_, kind});
      s_ = r_e_ + kmax * W_;
      ks_ = kmax;
      return;
    }
    for (uint64_t k = ks_; k < kmax; ++k) {
      const uint64_t ck = r_e_ + k * W_;
      if ((dead && dead[k]) || ck < s_) continue;
      zc_record& r = rec[o++];
      r.offset = ck;
      r.size = W_;
      r.kind = kind;
      r.rolling = indexable_ ? c_.h_key[k] : 0;
      memset(r.sha1, 0, sizeof r.sha1);
      s_ = ck + W_;
    }
    c_.recs.resize(o);
    ks_ = kmax;
  }

  void finish() {
    save_grid_until(kInf);
    const uint64_t L = n_ - s_;
    if (L > W_) {
      piece(s_, s_ + W_);
      piece(s_ + W_, n_);
    } else if (L > 0) {
      piece(s_, n_);
    }
    s_ = n_;
  }

  // the horizon reached without a grid-shifting match: the chunks cut by
  // then become confirmed refs; the next epoch resumes at the horizon
  bool horizon_stop() {
    save_grid_until(h_end_ - 1);
    keep_saved(h_end_ - 1);
    x_resume_ = h_end_;
    hspan_ *= 2;
    return true;
  }

  // After a grid shortcut match of grid chunk j: the following grid chunks
  // in a row that match at their own ends too (x is each one's end, so nothing
  // can come first) -- a duplicated or constant stretch -- as one run of DUP
  // records, written in parallel when long
  void chain(uint64_t j) {
    uint32_t jn = (uint32_t)j + 1;
    while (isc_ + 1 < sc_list_.size() && sc_list_[isc_ + 1] == jn) {
      const uint64_t pn = r_e_ + (uint64_t)(jn + 1) * W_ - 1;
      if (pn >= h_end_) break;
      const uint32_t gn = nconf_ + jn;
      if (!class_alive_visible(cls_[gn], pn)) break;
      ++isc_;
      dead_[gn] = 1;
      ++ndead_;
      ++jn;
    }
    const uint64_t nchain = jn - (j + 1);
    if (!nchain) return;
    const size_t o = c_.recs.size();
    c_.recs.resize(o + nchain);
    fill_grid_records(c_.recs.data() + o, nchain, r_e_, j + 1, W_, ZC_CHUNK_DUP, c_.h_key.p);
    gruns_.push_back({o, nchain, r_e_ + (j + 1) * W_, (uint32_t)ZC_CHUNK_DUP});
    r_ = r_e_ + (uint64_t)jn * W_;
    s_ = r_;
    if (jn > ks_) ks_ = jn;
  }

  // the probes of this epoch are done up to h_end_: go on at a horizon, stop
  // at the end of a window segment (the state carries over to the next one),
  // or finish the stream
  bool stop() {
    if (h_end_ < lim_) return horizon_stop();
    if (!final_) {
      save_grid_until(h_end_ - 1);
      keep_saved(h_end_ - 1);
      x_resume_ = h_end_;
      return false;
    }
    finish();
    return false;
  }

  // Grid shifts without a new epoch.  A match that moves the grid (the window
  // starts off the epoch's grid) ends the epoch's grid: its chunks not cut by
  // then leave the index (abandoned: marked dead), and a new grid starts at
  // r_g_.  The walk goes on with this epoch's candidates -- they cover every
  // index entry but the new grid's chunks -- for as long as no chunk of the
  // new grid gets cut: matches on it (an edited copy re-synchronising after
  // each insertion) consume its chunks, and pieces under W never match.  The
  // first time one would be cut (a match at or past s_ + 2W - 1, or the end
  // of the epoch's probes), a real epoch starts from the current position:
  // its index then holds the new grid's chunks.
  bool lazy_ = false;
  uint64_t r_g_ = 0;
  void abandon(uint64_t m) {
    for (uint32_t k = 0; k < nspec_; ++k) {
      const uint32_t g = nconf_ + k;
      if (ref_vis(g) > m && !dead_[g]) {
        dead_[g] = 1;
        ++ndead_;
      }
    }
  }
  bool lazy_exit(uint64_t x) {
    keep_saved(x);
    x_resume_ = x;
    hspan_ = std::max<uint64_t>(kHorizon0, 64ull * W_);
    return true;
  }

  bool walk() {
    uint64_t x = x0();
    size_t ia = 0, ih = 0;
    irun_ = 0;
    lazy_ = false;
    for (;;) {
      if (x >= h_end_) return lazy_ ? lazy_exit(x) : stop();
      uint32_t gref = 0;
      const uint64_t pg = next_grid(x, &gref);
      uint64_t pa = kInf;
      uint32_t refa = 0;
      while (ia < acands_.size()) {
        const ACand& a = acands_[ia];
        if (a.p >= x && class_alive_visible(a.ref, a.p)) {
          pa = a.p;
          refa = a.ref;
          break;
        }
        ++ia;
      }
      // historic entries are always in the index
      while (ih < hcands_.size() && hcands_[ih].p < x) ++ih;
      const uint64_t ph = ih < hcands_.size() ? hcands_[ih].p : kInf;
      const uint64_t pe = std::min(std::min(pa, ph), pg);
      uint64_t fkey = 0;
      // nothing precedes a match at x itself
      // lazily on a shifted grid, no match at or past s_ + 2W - 1 is taken
      // (lazy_exit first): the screen search stops there
      uint64_t flim = pe == kInf ? h_end_ : pe + 1;
      if (lazy_) flim = std::min<uint64_t>(flim, s_ + 2ull * W_ - 1);
      uint64_t pf = pe == x ? kInf : next_f(x, flim, &fkey);
      if (pe == kInf && pf == kInf) return lazy_ ? lazy_exit(x) : stop();
      uint64_t m, key;
      if (pf != kInf && (pe == kInf || pf < pe)) {
        m = pf;
        key = fkey;
      } else if (pg <= pa && pg <= ph) {
        m = pg;
        key = ref_key(gref);
      } else if (pa <= ph) {
        m = pa;
        key = ref_key(refa);
      } else {
        m = ph;
        key = c_.hkey[hcands_[ih].ref];
      }
      // the new grid's next chunk [s_, s_ + W) would be cut first
      if (lazy_ && m >= s_ + 2ull * W_ - 1) return lazy_exit(x);
      // the match at m
      save_grid_until(m);
      const uint64_t ws = m - W_ + 1;
      if (ws > s_) piece(s_, ws);
      push(ws, W_, ZC_CHUNK_DUP, key);
      r_ = m + 1;
      s_ = r_;
      const bool hist_match = m == ph && m != pg && m != pa && m != pf;
      if (lazy_) {
        // on the new grid: its chunk under the window is consumed; off it: the
        // grid moves again (back onto this epoch's grid: a real epoch)
        if ((r_ - r_g_) % W_ != 0) {
          r_g_ = r_;
          if ((r_g_ - r_e_) % W_ == 0) return lazy_exit(r_ + W_ - 1);
        }
        x = r_ + W_ - 1;
        if (hist_match) x = hist_run(ih, x, std::min(pa, pg), false);
        continue;
      }
      if ((r_ - r_e_) % W_ == 0) {
        // same grid: the grid chunk the window covered is consumed, not saved
        const uint64_t j = (ws - r_e_) / W_;
        if (indexable_ && j < nspec_) {
          dead_[nconf_ + j] = 1;
          ++ndead_;
        }
        if (j >= ks_) ks_ = j + 1;
        if (m == pg) chain(j);
        x = r_ + W_ - 1;
        if (hist_match) x = hist_run(ih, x, std::min(pa, pg), true);
        continue;
      }
      // grid shift: this epoch's grid ends at m; the walk goes on lazily
      abandon(m);
      lazy_ = true;
      r_g_ = r_;
      x = r_ + W_ - 1;
    }
  }

  // After a historic match whose window ended at x - W (the walk now at x):
  // the historic candidates that follow at x, x + W, x + 2W, ... -- an
  // unchanged stretch of an earlier backup, found window after window -- are
  // taken as one run of DUP records, written like the grid runs (in parallel
  // when long, classified by finalize_records from the run alone).  Each is a
  // match exactly where the walk stands (nothing can precede it: no flush
  // piece, no other candidate before `bound`, no by-value key to screen), so
  // the state after the run is what the walk would reach one match at a time:
  // r = s = the run's end, and on this epoch's grid (same_grid) the grid
  // chunks under the windows consumed.  Returns the walk's next position.
  std::vector<uint64_t> run_keys_;
  uint64_t hist_run(size_t& ih, uint64_t x, uint64_t bound, bool same_grid) {
    if (has_f_) return x;
    run_keys_.clear();
    const uint64_t x0r = x;
    size_t k = ih;
    while (k < hcands_.size()) {
      while (k < hcands_.size() && hcands_[k].p < x) ++k;  // (entries of a key chain at the window just taken)
      if (k == hcands_.size() || hcands_[k].p != x || x >= h_end_ || x >= bound) break;
      run_keys_.push_back(c_.hkey[hcands_[k].ref]);
      x += W_;
    }
    const uint64_t nrun = run_keys_.size();
    if (!nrun) return x0r;
    ih = k;
    const uint64_t ws0 = x0r - W_ + 1;
    if (same_grid && indexable_) {
      const uint64_t j0 = (ws0 - r_e_) / W_;
      for (uint64_t j = j0; j < j0 + nrun && j < nspec_; ++j)
        if (!dead_[nconf_ + j]) {
          dead_[nconf_ + j] = 1;
          ++ndead_;
        }
      if (j0 + nrun > ks_) ks_ = j0 + nrun;
    }
    const size_t o = c_.recs.size();
    c_.recs.resize(o + nrun);
    fill_grid_records(c_.recs.data() + o, nrun, ws0, 0, W_, ZC_CHUNK_DUP, run_keys_.data());
    gruns_.push_back({o, nrun, ws0, (uint32_t)ZC_CHUNK_DUP});
    r_ = x - W_ + 1;
    s_ = r_;
    return x;
  }

  // the grid chunks of this epoch saved by probe m become confirmed refs
  // (saved before the new origin: visible to every later probe)
  void keep_saved(uint64_t m) {
    if (!indexable_ || !nspec_) return;
    uint32_t nk = 0;
    while (nk < nspec_ && ref_vis(nconf_ + nk) <= m) ++nk;  // vis grows with k
    if (!nk) return;
    std::vector<uint64_t> fp(nk);
    std::vector<uint32_t> g(nk), anc(nk);
    d2h(c_, fp.data(), c_.c_fp.p + nconf_, nk);
    d2h(c_, g.data(), c_.c_g.p + nconf_, nk);
    d2h(c_, anc.data(), c_.c_anc.p + nconf_, nk);
    sync(c_);
    const uint32_t base = nconf_;
    for (uint32_t k = 0; k < nk; ++k) {
      const uint32_t ref = base + k;
      if (dead_[ref]) continue;
      cstart_.push_back(ref_start(ref));
      ckey_.push_back(c_.h_key[k]);
      cfp_.push_back(fp[k]);
      cg_.push_back(g[k]);
      canc_.push_back(anc[k]);
    }
    nconf_ = (uint32_t)cstart_.size();
  }

  // With chunk ids, the grid chunks [k W, min((k + 1) W, n)) -- the
  // stream's chunks unless matches move the grid -- are hashed on a side
  // stream as soon as the bytes are in HBM (ev_in), beside the scan (the
  // SHA-1 kernel needs no LDS, so it shares the CUs with the scan's
  // workgroups); finalize() takes every record that is one of them from there
  uint64_t pre_sha_n_ = 0;
  bool gsha_ready_ = false;
  // speculative SHA-1 class joins (whole-stream runs): the pairs of grid
  // chunks joined before their digests existed
  std::vector<std::pair<uint64_t, uint64_t>> spec_pairs_;
  // speculative historic joins: {grid chunk, historic entry} whose keys are
  // equal, joined before the chunk's digest existed
  std::vector<std::pair<uint64_t, uint64_t>>& spec_hist_ = c_.res_spec_hist;
 public:
  bool spec_ = false;
 private:
  const uint8_t* grid_sha() {
    if (!gsha_ready_) {
      sha_launch();  // (if no epoch batch queued it)
      if (pre_sha_n_) wait_stream(c_.sha_stream);  // the kernel and the copy behind it  // the kernel and the copy behind it
      gsha_ready_ = true;
    }
    return c_.h_gsha.p;
  }
  // window [ws, ws + W) is a grid chunk whose SHA-1 the side stream computes
  bool grid_sha_pending(uint64_t ws) const {
    return pre_sha_n_ && wmod(ws) == 0 && wdiv(ws) < pre_sha_n_ && ws + W_ <= n_;
  }
  // grid chunk q's SHA-1 when window [ws, ws + W) is that chunk, else null
  const uint8_t* grid_sha_of(uint64_t ws) {
    if (!pre_sha_n_ || wmod(ws)) return nullptr;
    const uint64_t q = wdiv(ws);
    if (q >= pre_sha_n_ || ws + W_ > n_) return nullptr;
    return grid_sha() + 20 * q;
  }
  // The grid SHA-1 is VALU work (~630 instructions per 64-byte block, 2.6 ms
  // per 8 GiB alone) and runs on its own stream behind the first epoch's
  // batch (sha_launch, queued right after the batch's last kernel): beside
  // the scan it only got the cycles the older scan waves left (scan + SHA-1
  // as concurrent kernels 4.1 ms, fused into the scan 4.3 ms, one after the
  // other 4.2 ms), and the batch's latency-bound kernels beside it starved
  // (chunk metadata 1.2 ms instead of 25 us, the probe 3.9 ms instead of
  // 0.1).  After the batch the walk, the records and the index registration
  // run on the host while the SHA-1 does.
  bool sha_pending_ = false;
  void pre_sha() {
    pre_sha_n_ = 0;
    gsha_ready_ = false;
    sha_pending_ = false;
    if (!(c_.flags & ZC_FLAG_SHA1) || !indexable_ || n_ < W_) return;
    const uint64_t k = (n_ + W_ - 1) / W_;
    if (k > 0xFFFFFFFFull) return;
    c_.h_gsha.ensure(k * 20);
    pre_sha_n_ = k;
    sha_pending_ = true;
  }
  void sha_launch() {
    if (!sha_pending_) return;
    sha_pending_ = false;
    const uint64_t k = pre_sha_n_;
    HCK(hipEventRecord(c_.ev_sha, c_.stream));  // behind the batch (and the scan)
    HCK(hipStreamWaitEvent(c_.sha_stream, c_.ev_sha, 0));
    // the digests go straight to pinned host memory (dword stores from the
    // kernel's lanes as they finish): no copy behind the kernel; the few
    // device reads of them (class joins after the kernel) cross the bus
    HCK(launch_sha1_grid(d_, n_, W_, (uint32_t)k, c_.h_gsha.p, c_.sha_stream));
    HCK(hipEventRecord(c_.ev_sha, c_.sha_stream));
  }

  // ---------------------------------------------------------------- finalize
  // Records [nrec_done, size) are complete once their pieces have digests
  // and (ZC_FLAG_SHA1) every chunk record its SHA-1 prefix.
  // finalize_records' per-record lists and the stream's new chunks live in the
  // context, so their capacity carries over from stream to stream (a fresh
  // 1 MB vector per stream is new pages, whose first touch faulted in ~0.5 ms)
  std::vector<uint64_t>& gq_ = c_.fin_gq;
  std::vector<uint32_t>& gslot_ = c_.fin_gslot;
  std::vector<uint32_t>& frec_ = c_.fin_frec;
  std::vector<uint64_t>& fresh_ = c_.fin_fresh;  // NEW W-byte chunks of the stream still resident: offset,
  std::vector<uint8_t, DefaultInit<uint8_t>> fresh_sha_;  // and SHA-1 prefix (ZC_FLAG_SHA1)
  // stream_end: the stream's end (run_final): with ZC_FLAG_SHA1 its new W-byte
  // chunks join the context's index here, their device metadata queued before
  // the wait for the grid SHA-1, so that wait ends the call with little after it
  void finalize_records(bool stream_end = false) {
    auto t0 = Clock::now();
    struct Done {
      zc_stats& st;
      Clock::time_point t;
      ~Done() {
        st.finalize_ms += ms_since(t);
        SpinTeam::disarm_any();  // the segment's parallel jobs are over
      }
    } done{c_.stats, t0};
    std::vector<uint64_t> a, b;
    std::vector<size_t> rest;
    for (size_t i = 0; i < need_digest_.size(); ++i) {
      const Piece& pc = need_digest_[i];
      size_t k = 0;
      while (pre_ready_ && k < pre_a_.size() && !(pre_a_[k] == pc.a && pre_b_[k] == pc.b)) ++k;
      if (pre_ready_ && k < pre_a_.size()) {
        c_.recs[pc.rec].rolling = c_.h_pre[k];
      } else {
        a.push_back(pc.a);
        b.push_back(pc.b);
        rest.push_back(i);
      }
    }
    std::vector<uint64_t> h = range_digests(a, b);
    for (size_t j = 0; j < rest.size(); ++j) c_.recs[need_digest_[rest[j]].rec].rolling = h[j];
    need_digest_.clear();
    const size_t r0 = c_.nrec_done, r1 = c_.recs.size();
    const bool sha1 = c_.flags & ZC_FLAG_SHA1;
    struct ClearRuns {
      std::vector<GridRun>& v;
      ~ClearRuns() { v.clear(); }
    } clear_runs{gruns_};
    if (!sha1) {
      c_.nrec_done = r1;
      if (stream_end) stream_end_index(nullptr);
      return;
    }
    // the fill team, awake by the time the digests land
    if (r1 - r0 >= kParallelRecordsMin) SpinTeam::get().arm();
    // records that are a whole grid chunk take their SHA-1 from the side
    // stream's pass; the others are hashed now
    const bool pow2 = (W_ & (W_ - 1)) == 0;
    const int wsh = pow2 ? __builtin_ctzll(W_) : 0;
    auto grid_q = [&](const zc_record& r) -> uint64_t {  // grid chunk of the record, or kInf
      const uint64_t q = pow2 ? r.offset >> wsh : r.offset / W_;
      return q * W_ == r.offset && q < pre_sha_n_ && r.size == std::min<uint64_t>(W_, n_ - r.offset) ? q : kInf;
    };
    std::vector<uint64_t> sa;
    std::vector<uint32_t> sl;
    std::vector<size_t> idx;
    std::vector<uint64_t>& gq = gq_;        // grid-chunk records: record index << 32 | chunk (both < 2^32)
    std::vector<uint32_t>& gslot = gslot_;  // per gq entry: its fresh_ entry (from f0), or kNoSlot
    std::vector<uint32_t>& frec = frec_;    // record (from r0) of each new fresh_ entry
    gq.clear();
    gslot.clear();
    frec.clear();
    std::vector<uint32_t> fsh;   // fresh_ entries (from f0) hashed here (not grid chunks): their idx entry
    constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
    const size_t f0 = fresh_.size();
    gq.reserve(r1 - r0);
    gslot.reserve(r1 - r0);
    frec.reserve(r1 - r0);
    if (fresh_.capacity() < fresh_.size() + (r1 - r0)) fresh_.reserve(2 * (fresh_.size() + (r1 - r0)));
    size_t gr = 0;
    while (gr < gruns_.size() && gruns_[gr].rec0 < r0) ++gr;
    for (size_t i = r0; i < r1; ++i) {
      if (gr < gruns_.size() && gruns_[gr].rec0 == i) {
        // a run of grid-aligned records written by fill_grid_records: its
        // chunks, fresh entries and index slots follow from the run alone
        const GridRun& g = gruns_[gr++];
        const bool on_grid = g.off0 % W_ == 0 && g.kind != ZC_BYTES;
        const uint64_t q0 = g.off0 / W_;
        for (uint64_t j = 0; j < g.n; ++j) {
          uint32_t slot = kNoSlot;
          if (g.kind == ZC_CHUNK_NEW) {
            slot = (uint32_t)frec.size();
            fresh_.push_back(g.off0 + j * W_);
            frec.push_back((uint32_t)(i + j - r0));
          }
          if (on_grid && q0 + j < pre_sha_n_ && g.off0 + (j + 1) * W_ <= n_) {
            gq.push_back((uint64_t)(i + j - r0) << 32 | (q0 + j));
            gslot.push_back(slot);
          } else if (g.kind != ZC_BYTES) {
            if (slot != kNoSlot) fsh.push_back((uint32_t)idx.size());
            sa.push_back(g.off0 + j * W_);
            sl.push_back(W_);
            idx.push_back(i + j);
          }
        }
        i += g.n - 1;
        continue;
      }
      const zc_record& r = c_.recs[i];
      if (r.kind == ZC_BYTES) continue;
      uint32_t slot = kNoSlot;
      if (r.kind == ZC_CHUNK_NEW && r.size == W_) {
        slot = (uint32_t)frec.size();
        fresh_.push_back(r.offset);
        frec.push_back((uint32_t)(i - r0));
      }
      const uint64_t q = grid_q(r);
      if (q != kInf) {
        gq.push_back((uint64_t)(i - r0) << 32 | q);
        gslot.push_back(slot);
        continue;
      }
      if (slot != kNoSlot) fsh.push_back((uint32_t)idx.size());
      sa.push_back(r.offset);
      sl.push_back(r.size);
      idx.push_back(i);
    }
    std::vector<uint8_t> sh = sha1s(sa, sl);
    HistPending hp;
    auto th = Clock::now();
    std::vector<uint32_t> hp_ancless;
    if (stream_end) {
      hp = hist_add_meta(fresh_);
      hp_ancless = ancless_of(hp);  // (its work ran beside the SHA-1 kernel: done by now)
    }
    c_.stats.hist_ms += ms_since(th);
    // the new W-byte chunks' SHA-1 prefixes, in record order as fresh_: at
    // the stream's end straight into the historic index (their entries
    // hp.e0 + j), else kept with fresh_ until they join it.  Sized before
    // the wait (no value-initialisation: every byte is written below).
    uint8_t* fs;
    const bool in_place = stream_end && f0 == 0 && hp.k > 0 && hp.k == frec.size();
    if (in_place) {
      c_.hsha.resize(16 * ((size_t)hp.e0 + hp.k));
      fs = c_.hsha.data() + 16 * (size_t)hp.e0;
    } else {
      fresh_sha_.resize(16 * fresh_.size());
      fs = fresh_sha_.data() + 16 * f0;
    }
    const bool team = gq.size() >= kParallelRecordsMin;
    auto tw = Clock::now();
    const uint8_t* gsha = pre_sha_n_ ? grid_sha() : nullptr;  // waits for the side stream
    c_.stats.sha_wait_ms += ms_since(tw);
    auto tf = Clock::now();
    {
      // the speculated joins (epoch): every pair's prefixes must agree
      std::atomic<bool> refuted{false};
      auto check = [&](size_t a, size_t b) {
        for (size_t j = a; j < b; ++j)
          if (memcmp(gsha + 20 * spec_pairs_[j].first, gsha + 20 * spec_pairs_[j].second, 16) != 0) {
            refuted.store(true, std::memory_order_relaxed);
            return;
          }
      };
      if (spec_pairs_.size() >= kParallelRecordsMin) SpinTeam::get().run(spec_pairs_.size(), check);
      else check(0, spec_pairs_.size());
      // the speculated historic joins: a window joined on the key to several
      // entries (a key chain, chunk_index.cc:119-143) is right when ANY of them
      // has its prefix; a window with none refutes the speculation
      std::mutex mm;
      std::vector<size_t> miss;
      auto check_hist = [&](size_t a, size_t b) {
        std::vector<size_t> mine;
        for (size_t j = a; j < b; ++j)
          if (memcmp(gsha + 20 * spec_hist_[j].first, &c_.hsha[16 * (size_t)spec_hist_[j].second], 16) != 0)
            mine.push_back(j);
        if (!mine.empty()) {
          std::lock_guard<std::mutex> lk(mm);
          miss.insert(miss.end(), mine.begin(), mine.end());
        }
      };
      if (spec_hist_.size() >= kParallelRecordsMin) SpinTeam::get().run(spec_hist_.size(), check_hist);
      else check_hist(0, spec_hist_.size());
      if (miss.size() > 64) {
        refuted.store(true);  // (many wrong-prefix chain entries: redone exactly rather than searched)
      } else {
        for (size_t j : miss) {
          const uint64_t q = spec_hist_[j].first;
          bool any = false;
          for (const auto& sp : spec_hist_)
            if (sp.first == q && memcmp(gsha + 20 * q, &c_.hsha[16 * (size_t)sp.second], 16) == 0) {
              any = true;
              break;
            }
          if (!any) refuted.store(true);
        }
      }
      spec_hist_.clear();
      if (refuted.load()) throw Respeculate{};
      spec_pairs_.clear();
    }
    zc_record* const rb = c_.recs.data() + r0;
    // one pass: each grid-chunk record's prefix from the side stream's
    // digests, into the record and, for a new chunk, its index slot; the
    // record lines are fetched for writing a few entries ahead
    // (the index slots are written past the caches: nothing reads them soon)
    const bool fs_nt = ((uintptr_t)fs & 15) == 0;
    auto fill = [&](size_t a, size_t b) {
      constexpr size_t kAhead = 32;
      for (size_t j = a; j < std::min(b, a + kAhead); ++j) __builtin_prefetch(rb[gq[j] >> 32].sha1, 1);
      for (size_t j = a; j < b; ++j) {
        if (j + kAhead < b) __builtin_prefetch(rb[gq[j + kAhead] >> 32].sha1, 1);
        const uint8_t* src = gsha + 20 * (uint32_t)gq[j];
        const __m128i v = _mm_loadu_si128((const __m128i*)src);
        _mm_storeu_si128((__m128i*)rb[gq[j] >> 32].sha1, v);
        if (gslot[j] != kNoSlot) {
          uint8_t* d = fs + 16 * (size_t)gslot[j];
          if (fs_nt) _mm_stream_si128((__m128i*)d, v);
          else _mm_storeu_si128((__m128i*)d, v);
        }
      }
      _mm_sfence();
    };
    if (team) SpinTeam::get().run(gq.size(), fill);
    else fill(0, gq.size());
    for (size_t j = 0; j < idx.size(); ++j) memcpy(c_.recs[idx[j]].sha1, &sh[j * 20], 16);
    for (uint32_t t : fsh) {  // new chunks hashed here: their slot is their place among frec
      const uint32_t rec = (uint32_t)(idx[t] - r0);
      const size_t slot = std::lower_bound(frec.begin(), frec.end(), rec) - frec.begin();
      memcpy(fs + 16 * slot, &sh[t * 20], 16);
    }
    c_.nrec_done = r1;
    if (stream_end) stream_end_index(&hp, in_place, &hp_ancless);
    c_.stats.sha_fill_ms += ms_since(tf);
  }

  // The stream's end.  With ZC_FLAG_SHA1 its new W-byte chunks join the
  // context's index (Writer::add -> ChunkIndex::addChunk, chunk_storage.cc:
  // 31-46): a later stream on this context matches them, as a later backup
  // matches a committed one's index (chunk_index.cc:26-79).  Without it the
  // index is left as the stream found it (entries evicted from the window
  // during the stream are dropped again).
  void stream_end_index(const HistPending* hp, bool sha_in_place = false,
                        const std::vector<uint32_t>* ancless = nullptr) {
    if (c_.flags & ZC_FLAG_SHA1) {
      hist_add_sha(*hp, sha_in_place ? nullptr : fresh_sha_.data(), ancless);
    } else {
      index_truncate(c_, hist0_, statics0_);
    }
    fresh_.clear();
    fresh_sha_.clear();
  }

 public:
  // window mode: NEW chunks below `keep` are no longer resident; those that
  // are refs went to the historic index with evict_before()
  void drop_fresh_before(uint64_t keep) {
    size_t k = 0;
    while (k < fresh_.size() && fresh_[k] < keep) ++k;
    fresh_.erase(fresh_.begin(), fresh_.begin() + k);
    fresh_sha_.erase(fresh_sha_.begin(), fresh_sha_.begin() + 16 * k);
  }
};

// every entry point on a context holds its mutex (null-safe)
#define ZC_LOCK(c)                                                                                 \
  std::unique_lock<std::recursive_mutex> zc_lk_ =                                                  \
      (c) ? std::unique_lock<std::recursive_mutex>((c)->mu) : std::unique_lock<std::recursive_mutex>()

int fail(zc_ctx* c, const ZcError& e) {
  if (c) c->err = e.msg;
  return e.code;
}

template <class F>
int guarded(zc_ctx* c, F&& f) {
  try {
    f();
    if (c) c->err.clear();
    return ZC_OK;
  } catch (const ZcError& e) {
    return fail(c, e);
  } catch (const std::bad_alloc&) {
    return fail(c, ZcError{ZC_ERR_NOMEM, "host allocation failed"});
  } catch (const std::exception& e) {
    return fail(c, ZcError{ZC_ERR_STATE, e.what()});
  }
}

void append_device(zc_ctx& c, const void* src, size_t n, hipMemcpyKind kind) {
  if (!n) return;
  if (c.n_stream + n > c.d_stream.cap) {
    size_t want = std::max<size_t>(c.n_stream + n, c.d_stream.cap * 2);
    want = (want + 4095) & ~size_t(4095);
    uint8_t* np = nullptr;
    hipError_t e = hipMalloc(&np, want);
    if (e != hipSuccess) throw ZcError{ZC_ERR_NOMEM, std::string("stream buffer: ") + hipGetErrorString(e)};
    if (c.n_stream)
      HCK(hipMemcpyAsync(np, c.d_stream.p, c.n_stream, hipMemcpyDeviceToDevice, c.stream));
    sync(c);
    c.d_stream.release();
    c.d_stream.p = np;
    c.d_stream.cap = want;
  }
  HCK(hipMemcpyAsync(c.d_stream.p + c.n_stream, src, n, kind, c.stream));
  sync(c);
  c.n_stream += n;
}

// ---------------------------------------------------------------------------
// The bounded feed window (zc_set_window).  The feed writes into the pinned
// host mirror at the window's end (getInputBuffer), each piece is copied to
// the same place in HBM on the copy stream, and once half a window of new
// bytes has arrived the resolver takes every probe up to the last full scan
// tile (run_segment).  Before the next input the window slides down to what
// the resolver will read again (Resolver::keep_from: about 2 W + 4 MiB),
// moving the bytes, their span digests and anchors with it; chunks that
// start below that join the historic index first.  HBM and pinned memory
// stay at the window's size however long the stream is.
constexpr uint64_t kDefaultWindow = 1ull << 30;
constexpr uint64_t kFeedMax = 64ull << 20;  // most bytes one getInputBuffer offers

uint64_t window_for(uint64_t want, uint32_t W) {
  // a window half must hold new tiles beyond what the resolver keeps
  const uint64_t m = std::max<uint64_t>(want, 8ull * W + (16ull << 20));
  return (m + ZC_STILE - 1) / ZC_STILE * ZC_STILE;
}

void window_alloc_join(zc_ctx& c) {
  if (!c.win_alloc.joinable()) return;
  c.win_alloc.join();
  if (!c.win_alloc_err.empty()) {
    std::string e;
    e.swap(c.win_alloc_err);
    throw ZcError{ZC_ERR_NOMEM, "feed window: " + e};
  }
}

// start making the window's buffers on a helper thread
void window_alloc_start(zc_ctx& c) {
  window_alloc_join(c);
  if (!c.win_cap || (c.dwin.cap >= c.win_cap && c.hwin.cap >= c.win_cap && c.dwin.p && c.hwin.p)) return;
  c.win_alloc = std::thread([&c] {
    try {
      DeviceGuard g(c.device);
      c.dwin.ensure(c.win_cap);
      c.hwin.ensure(c.win_cap);
    } catch (const ZcError& e) {
      c.win_alloc_err = e.msg;
    } catch (const std::exception& e) {
      c.win_alloc_err = e.what();
    }
  });
}

void window_open(zc_ctx& c) {
  if (c.res) return;
  window_alloc_join(c);
  c.dwin.ensure(c.win_cap);
  c.hwin.ensure(c.win_cap);
  c.wbase = c.wend = 0;
  c.windowed_last = true;
  c.res = new Resolver(c, c.dwin.p, 0, true);
  c.res->begin();
}

void window_close(zc_ctx& c) {
  delete c.res;
  c.res = nullptr;
  c.slide_pending = false;
}

// buf[shift, shift + len) -> buf[0, len), in stream order, pieces no longer
// than the shift so no piece overlaps its own source
template <class T>
void move_down(hipStream_t s, T* buf, uint64_t shift, uint64_t len) {
  if (!shift || !len) return;
  for (uint64_t off = 0; off < len; off += shift) {
    const uint64_t m = std::min(shift, len - off);
    HCK(hipMemcpyAsync(buf + off, buf + off + shift, m * sizeof(T), hipMemcpyDeviceToDevice, s));
  }
}

void window_slide(zc_ctx& c) {
  c.slide_pending = false;
  Resolver& r = *c.res;
  const uint64_t keep = r.keep_from();
  if (keep <= c.wbase) return;
  r.evict_before(keep);
  r.drop_fresh_before(keep);
  HCK(hipStreamWaitEvent(c.stream, c.ev_in, 0));  // the window's copies have landed
  const uint64_t sh = keep - c.wbase, len = c.wend - keep;
  move_down(c.stream, c.dwin.p, sh, len);
  // span digests and anchors of the scanned tiles above `keep`
  const uint64_t scanned = std::max(r.scanned_end(), keep);
  move_down(c.stream, c.blk.p, sh / ZC_SPAN, (scanned - keep) / ZC_SPAN);
  const uint64_t w0 = sh >> ZC_WT_SHIFT, wl = (scanned - keep) >> ZC_WT_SHIFT;
  const uint64_t wcap = wave_tile_cap(c.W);
  move_down(c.stream, c.dbase.p, w0, wl);
  move_down(c.stream, c.dcnt.p, w0, wl);
  move_down(c.stream, c.prel.p, w0 * wcap, wl * wcap);
  move_down(c.stream, c.pg.p, w0 * wcap, wl * wcap);
  HCK(launch_slide_dir(c.dbase.p, c.dcnt.p, (uint32_t)wl, (uint32_t)(w0 * wcap), c.stream));
  HCK(hipStreamSynchronize(c.copy_stream));
  memmove(c.hwin.p, c.hwin.p + sh, len);
  c.wbase = keep;
  r.rebase(c.dwin.p, keep);
  sync(c);
}

size_t window_room(const zc_ctx& c) {
  return (size_t)std::min<uint64_t>(kFeedMax, c.win_cap - (c.wend - c.wbase));
}

void window_add(zc_ctx& c, size_t added) {
  const uint64_t off = c.wend - c.wbase;
  if (added > c.win_cap - off) throw ZcError{ZC_ERR_ARG, "handleMoreData: more than getInputBufferSize() bytes"};
  if (!added) return;
  HCK(hipMemcpyAsync(c.dwin.p + off, c.hwin.p + off, added, hipMemcpyHostToDevice, c.copy_stream));
  HCK(hipEventRecord(c.ev_in, c.copy_stream));
  HCK(hipStreamWaitEvent(c.stream, c.ev_in, 0));
  c.wend += added;
  c.res->set_avail(c.wend);
  if (c.wend - c.res->scanned_end() >= c.win_cap / 2) {
    c.res->run_segment(c.wend / ZC_STILE * ZC_STILE);
    c.slide_pending = true;
  }
}

size_t ctx_hbm_bytes(const zc_ctx& c) {
  size_t b = c.d_stream.bytes() + c.dwin.bytes() + c.hanc.bytes() + c.hg.bytes() + c.hfp.bytes() + c.htab.bytes() +
             c.hfilt.bytes() + c.hm_key.bytes() + c.hm_fp.bytes() + c.hm_anc.bytes() + c.hm_g.bytes() +
             c.blk.bytes() + c.ftile_off.bytes() + c.ftile_cnt.bytes() + c.dbase.bytes() + c.dcnt.bytes() +
             c.prel.bytes() + c.pg.bytes() + c.srel.bytes() + c.sg.bytes() + c.otiles.bytes() + c.obase.bytes() +
             c.counters.bytes() + c.gsha.bytes() + c.c_start.bytes() + c.c_key.bytes() + c.c_fp.bytes() +
             c.c_vis.bytes() + c.c_anc.bytes() + c.c_g.bytes() + c.c_dead.bytes() + c.ckeys.bytes() +
             c.c_cls.bytes() + c.tab.bytes() + c.gfilt.bytes() + c.cand.bytes() + c.va.bytes() + c.vb.bytes() +
             c.dout.bytes() + c.vlen.bytes() + c.vok.bytes() + c.sha_out.bytes() + c.f32.bytes() + c.fbits.bytes() +
             c.fbits17.bytes() + c.fwt_off.bytes() + c.fwt_cnt.bytes() + c.runs.bytes() + c.ancless.bytes();
  return b;
}

}  // namespace

#ifndef ZC_BUILD_ID
#define ZC_BUILD_ID "unknown"
#endif
// kept in the binary as "zc-build-id:<digest>" so _build.py can read it
// from the file without loading the library
__attribute__((used)) const char kZcBuildTag[] = "zc-build-id:" ZC_BUILD_ID;

extern "C" {

int zc_abi_version(void) { return ZCHUNK_ABI_VERSION; }
const char* zc_build_id(void) { return kZcBuildTag + 12; }

int zc_create(zc_ctx** out, uint32_t chunk_max_size, int device, uint32_t flags) {
  if (!out || chunk_max_size == 0) return ZC_ERR_ARG;
  *out = nullptr;
  zc_ctx* c = new (std::nothrow) zc_ctx;
  if (!c) return ZC_ERR_NOMEM;
  c->device = device;
  c->W = chunk_max_size;
  c->flags = flags;
  c->win_cap = window_for(kDefaultWindow, chunk_max_size);
  int rc = guarded(c, [&] {
    DeviceGuard g(device);
    HCK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HCK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    HCK(hipEventCreate(&c->ev0));
    HCK(hipEventCreate(&c->ev1));
    HCK(hipEventCreate(&c->ev_meta));
    HCK(hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming));
    HCK(hipEventCreateWithFlags(&c->ev_idx, hipEventDisableTiming));
    HCK(hipEventCreateWithFlags(&c->ev_sha, hipEventDisableTiming));
    HCK(hipEventCreateWithFlags(&c->ev_grec, hipEventDisableTiming));
    HCK(hipEventCreateWithFlags(&c->ev_copy, hipEventDisableTiming));
    HCK(hipEventCreateWithFlags(&c->ev_batch, hipEventDisableTiming));
    HCK(hipStreamCreateWithFlags(&c->sha_stream, hipStreamNonBlocking));
    HCK(hipHostMalloc((void**)&c->stage, kFeedChunk, hipHostMallocDefault));
  });
  if (rc != ZC_OK) {
    zc_destroy(c);
    return rc;
  }
  *out = c;
  return ZC_OK;
}

int zc_destroy(zc_ctx* c) {
  if (!c) return ZC_ERR_ARG;
  {
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->win_alloc.joinable()) c->win_alloc.join();
    window_close(*c);
    if (c->stage) (void)hipHostFree(c->stage);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev_meta) (void)hipEventDestroy(c->ev_meta);
    if (c->ev_in) (void)hipEventDestroy(c->ev_in);
    if (c->ev_idx) (void)hipEventDestroy(c->ev_idx);
    if (c->ev_sha) (void)hipEventDestroy(c->ev_sha);
    if (c->ev_grec) (void)hipEventDestroy(c->ev_grec);
    if (c->ev_copy) (void)hipEventDestroy(c->ev_copy);
    if (c->ev_batch) (void)hipEventDestroy(c->ev_batch);
    if (c->sha_stream) (void)hipStreamSynchronize(c->sha_stream);
    if (c->sha_stream) (void)hipStreamDestroy(c->sha_stream);
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    lzo_scratch_free(c->lzo);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  return ZC_OK;
}

int zc_seed_index(zc_ctx* c, const zc_seed* seeds, size_t n) {
  ZC_LOCK(c);
  if (!c || (n && !seeds)) return ZC_ERR_ARG;
  return guarded(c, [&] {
    for (size_t i = 0; i < n; ++i) {
      if (seeds[i].size != c->W) continue;  // only W-byte entries can equal a W-byte window
      add_static_once(*c, seeds[i].rolling, seeds[i].sha1, 1);
    }
  });
}

uint32_t zc_anchor_def(uint32_t chunk_max_size) { return chunk_max_size ? anchor_def_of(chunk_max_size) : 0u; }

// ids with metadata join the historic index (key and SHA-1 prefix on the host,
// first anchor / gear / fingerprint on the device, the anchor in its table),
// the rest the by-value set: what ChunkIndex::loadIndex registers
// (chunk_index.cc:26-79,163-182), split by how the engine can find each id
int zc_seed_index_meta(zc_ctx* c, const zc_seed* seeds, size_t n, const zc_chunk_meta* meta, size_t nm) {
  ZC_LOCK(c);
  if (!c || (n && !seeds) || (nm && !meta)) return ZC_ERR_ARG;
  if (c->nhist != c->nhist_seeded) {
    c->err = "zc_seed_index_meta: the context's streams have added chunks to its index (seed before the first "
             "stream, or after zc_forget_stream_chunks)";
    return ZC_ERR_STATE;
  }
  return guarded(c, [&] {
    DeviceGuard g(c->device);
    // the host arrays hold exactly the entries so far (a call that failed
    // part-way may have appended some without registering them)
    c->hkey.resize(c->nhist);
    c->hsha.resize(16 * (size_t)c->nhist);
    const uint32_t W = c->W, def = anchor_def_of(W);
    // usable metadata by rolling key (then SHA-1 prefix): W-byte chunks of
    // this anchor definition with an anchor where a W-byte chunk can hold one
    std::unordered_map<uint64_t, std::vector<uint32_t>> mk;
    mk.reserve(nm);
    for (size_t j = 0; j < nm; ++j) {
      const zc_chunk_meta& m = meta[j];
      if (m.size != W || m.anchor_def != def || m.anchor == ZC_NO_ANCHOR || m.anchor < ZC_ANCHOR_MIN_OFF ||
          m.anchor >= W || W <= ZC_ANCHOR_MIN_OFF)
        continue;
      mk[m.rolling].push_back((uint32_t)j);
    }
    // historic ids already seeded, for registerNewChunkId's "unless present"
    std::unordered_map<uint64_t, std::vector<uint32_t>> have;
    for (uint32_t e = 0; e < c->nhist; ++e) have[c->hkey[e]].push_back(e);
    const uint32_t e0 = c->nhist;
    std::vector<uint32_t> anc, gv;
    std::vector<uint64_t> fp;
    for (size_t i = 0; i < n; ++i) {
      const zc_seed& sd = seeds[i];
      if (sd.size != W) continue;  // only W-byte entries can equal a W-byte window
      const zc_chunk_meta* m = nullptr;
      auto it = mk.find(sd.rolling);
      if (it != mk.end())
        for (uint32_t j : it->second)
          if (memcmp(meta[j].sha1, sd.sha1, 16) == 0) {
            m = &meta[j];
            break;
          }
      if (!m) {
        add_static_once(*c, sd.rolling, sd.sha1, 1);
        continue;
      }
      auto& hv = have[sd.rolling];
      bool dup = false;
      for (uint32_t e : hv)
        if (memcmp(&c->hsha[16 * (size_t)e], sd.sha1, 16) == 0) dup = true;
      if (dup) continue;
      const uint32_t e = e0 + (uint32_t)anc.size();
      if (e == 0xFFFFFFFFu) throw ZcError{ZC_ERR_NOMEM, "historic index full"};
      hv.push_back(e);
      c->hkey.push_back(sd.rolling);
      c->hsha.insert(c->hsha.end(), sd.sha1, sd.sha1 + 16);
      anc.push_back(m->anchor);
      gv.push_back(m->gear);
      fp.push_back(m->fingerprint);
    }
    const uint32_t k = (uint32_t)anc.size();
    if (!k) return;
    c->hanc.grow_keep((uint64_t)e0 + k, e0, c->stream);
    c->hg.grow_keep((uint64_t)e0 + k, e0, c->stream);
    c->hfp.grow_keep((uint64_t)e0 + k, e0, c->stream);
    c->hkey_d.grow_keep((uint64_t)e0 + k, e0, c->stream);
    h2d(*c, c->hkey_d.p + e0, c->hkey.data() + e0, k);
    h2d(*c, c->hanc.p + e0, anc.data(), k);
    h2d(*c, c->hg.p + e0, gv.data(), k);
    h2d(*c, c->hfp.p + e0, fp.data(), k);
    c->nhist = e0 + k;
    c->nhist_seeded = c->nhist;
    hist_table(*c, e0);
    sync(*c);  // (the host arrays above are freed on return)
  });
}

int zc_export_chunk_meta(const zc_ctx* c, zc_chunk_meta* out, size_t cap, size_t* n_out) {
  ZC_LOCK(c);
  if (!c || !n_out || (cap && !out)) return ZC_ERR_ARG;
  const uint32_t e0 = c->nhist_seeded, k = c->nhist - c->nhist_seeded;
  *n_out = k;
  if (k > cap) return ZC_ERR_ARG;
  if (!k) return ZC_OK;
  std::vector<uint32_t> anc(k), gv(k);
  std::vector<uint64_t> fp(k);
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(c->device) != hipSuccess) return ZC_ERR_HIP;
  hipError_t e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) e = hipMemcpy(anc.data(), c->hanc.p + e0, k * sizeof(uint32_t), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(gv.data(), c->hg.p + e0, k * sizeof(uint32_t), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(fp.data(), c->hfp.p + e0, k * sizeof(uint64_t), hipMemcpyDeviceToHost);
  if (prev >= 0) (void)hipSetDevice(prev);
  if (e != hipSuccess) return ZC_ERR_HIP;
  const uint32_t def = anchor_def_of(c->W);
  for (uint32_t i = 0; i < k; ++i) {
    zc_chunk_meta& m = out[i];
    memcpy(m.sha1, &c->hsha[16 * ((size_t)e0 + i)], 16);
    m.rolling = c->hkey[e0 + i];
    m.size = c->W;
    m.anchor_def = def;
    m.anchor = anc[i];
    m.gear = anc[i] == ZC_NO_ANCHOR ? 0u : gv[i];
    m.fingerprint = anc[i] == ZC_NO_ANCHOR ? 0ull : fp[i];
  }
  return ZC_OK;
}

int zc_set_window(zc_ctx* c, uint64_t bytes) {
  ZC_LOCK(c);
  if (!c) return ZC_ERR_ARG;
  if (c->res || c->n_stream) return ZC_ERR_STATE;
  return guarded(c, [&] {
    window_alloc_join(*c);
    c->win_cap = bytes ? window_for(bytes, c->W) : 0;
    window_alloc_start(*c);  // (joined by the first getInputBuffer)
  });
}

uint64_t zc_get_window(const zc_ctx* c) { return c ? c->win_cap : 0; }

void* zc_get_input_buffer(zc_ctx* c) {
  ZC_LOCK(c);
  if (!c || c->finished) return nullptr;
  if (!c->win_cap) return c->stage;
  void* p = nullptr;
  int rc = guarded(c, [&] {
    DeviceGuard g(c->device);
    window_open(*c);
    if (c->slide_pending) window_slide(*c);
    p = c->hwin.p + (c->wend - c->wbase);
  });
  return rc == ZC_OK ? p : nullptr;
}

size_t zc_get_input_buffer_size(zc_ctx* c) {
  ZC_LOCK(c);
  if (!c || c->finished) return 0;
  if (!c->win_cap) return kFeedChunk;
  size_t n = 0;
  int rc = guarded(c, [&] {
    DeviceGuard g(c->device);
    window_open(*c);
    if (c->slide_pending) window_slide(*c);
    n = window_room(*c);
  });
  return rc == ZC_OK ? n : 0;
}

int zc_handle_more_data(zc_ctx* c, size_t added) {
  ZC_LOCK(c);
  if (!c) return ZC_ERR_ARG;
  if (c->finished) return ZC_ERR_STATE;
  if (!c->win_cap) {
    if (added > kFeedChunk) return ZC_ERR_ARG;
    return guarded(c, [&] {
      DeviceGuard g(c->device);
      append_device(*c, c->stage, added, hipMemcpyHostToDevice);
    });
  }
  if (!c->res) return ZC_ERR_STATE;  // no getInputBuffer() before it
  return guarded(c, [&] {
    DeviceGuard g(c->device);
    window_add(*c, added);
  });
}

int zc_feed(zc_ctx* c, const void* host, size_t n) {
  ZC_LOCK(c);
  if (!c || (n && !host)) return ZC_ERR_ARG;
  if (c->finished) return ZC_ERR_STATE;
  if (!c->win_cap) {
    return guarded(c, [&] {
      DeviceGuard g(c->device);
      append_device(*c, host, n, hipMemcpyHostToDevice);
    });
  }
  const uint8_t* h = (const uint8_t*)host;
  while (n) {
    uint8_t* dst = (uint8_t*)zc_get_input_buffer(c);
    const size_t room = zc_get_input_buffer_size(c);
    if (!dst || !room) return dst ? ZC_ERR_STATE : (c->err.empty() ? ZC_ERR_STATE : ZC_ERR_HIP);
    const size_t m = std::min(room, n);
    memcpy(dst, h, m);
    const int rc = zc_handle_more_data(c, m);
    if (rc != ZC_OK) return rc;
    h += m;
    n -= m;
  }
  return ZC_OK;
}

int zc_finish(zc_ctx* c) {
  ZC_LOCK(c);
  if (!c) return ZC_ERR_ARG;
  if (c->finished) return ZC_ERR_STATE;
  if (c->win_cap) {
    return guarded(c, [&] {
      DeviceGuard g(c->device);
      window_open(*c);
      try {
        c->res->run_final();
      } catch (...) {
        window_close(*c);
        throw;
      }
      window_close(*c);
      c->d_last = c->dwin.p;
      c->n_last = c->wend;
      c->finished = true;
    });
  }
  return guarded(c, [&] {
    DeviceGuard g(c->device);
    c->windowed_last = false;
    Resolver res(*c, c->d_stream.p, c->n_stream, false);
    res.run();
    c->d_last = c->d_stream.p;
    c->n_last = c->n_stream;
    c->finished = true;
  });
}

int zc_chunk_device(zc_ctx* c, const void* d_data, uint64_t n) {
  ZC_LOCK(c);
  if (!c || (n && !d_data) || ((uintptr_t)d_data & 15)) return ZC_ERR_ARG;
  if (c->res) return ZC_ERR_STATE;  // a fed stream is open
  return guarded(c, [&] {
    DeviceGuard g(c->device);
    // the stream may have just been written on the legacy default stream
    // (e.g. torch's): order the context's stream after that work (nothing to
    // order after when that stream is idle: the event and the wait cost ~7 us
    // of host time before the scan is queued)
    const hipError_t q = hipStreamQuery(nullptr);
    if (q != hipSuccess) {
      if (q != hipErrorNotReady) HCK(q);
      HCK(hipEventRecord(c->ev_in, nullptr));
      HCK(hipStreamWaitEvent(c->stream, c->ev_in, 0));
    }
    c->windowed_last = false;
    const uint32_t nh = c->nhist;
    const size_t ns = c->statics.size();
    bool redo = false;
    {
      Resolver res(*c, (const uint8_t*)d_data, n, false);
      res.spec_ = (c->flags & ZC_FLAG_SHA1) != 0;
      try {
        res.run();
      } catch (const Respeculate&) {
        res.drain();
        redo = true;
      }
    }
    if (redo) {  // (equal 64-bit keys of different grid chunks: practically only by construction)
      index_truncate(*c, nh, ns, true);
      Resolver res(*c, (const uint8_t*)d_data, n, false);
      res.run();
      c->stats.respeculations = 1;
    }
    c->d_last = (const uint8_t*)d_data;
    c->n_last = n;
    c->finished = true;
  });
}

int zc_chunk_host(zc_ctx* c, const void* host, uint64_t n) {
  ZC_LOCK(c);
  if (!c || (n && !host)) return ZC_ERR_ARG;
  if (c->res) return ZC_ERR_STATE;
  return guarded(c, [&] {
    DeviceGuard g(c->device);
    if (c->d_stream.cap < n) {
      c->d_stream.release();
      c->d_stream.ensure((n + 4095) & ~uint64_t(4095));
    }
    c->n_stream = n;
    c->windowed_last = false;
    uint8_t* d = c->d_stream.p;
    const uint8_t* h = (const uint8_t*)host;
    // segments land on the copy stream; the scan of each follows on the
    // context's stream as soon as its copy has completed
    Resolver res(*c, d, n, false);
    res.begin();
    for (uint64_t off = 0; off < n; off += kHostSegment) {
      const uint64_t len = std::min<uint64_t>(kHostSegment, n - off);
      HCK(hipMemcpyAsync(d + off, h + off, len, hipMemcpyHostToDevice, c->copy_stream));
      HCK(hipEventRecord(c->ev_in, c->copy_stream));
      HCK(hipStreamWaitEvent(c->stream, c->ev_in, 0));
      res.scan_upto(off + len);
    }
    res.run_final();
    c->d_last = d;
    c->n_last = n;
    c->finished = true;
  });
}

size_t zc_record_count(const zc_ctx* c) {
  if (!c) return 0;
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  return c->nrec_done - c->rec_head;
}

int zc_get_records(const zc_ctx* c, zc_record* out, size_t cap, size_t* n_out) {
  if (!c || (cap && !out)) return ZC_ERR_ARG;
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  size_t n = std::min(cap, c->nrec_done - c->rec_head);
  if (n) memcpy(out, c->recs.data() + c->rec_head, n * sizeof(zc_record));
  if (n_out) *n_out = n;
  return ZC_OK;
}

int zc_take_records(zc_ctx* c, zc_record* out, size_t cap, size_t* n_out) {
  if (!c || (cap && !out)) return ZC_ERR_ARG;
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  const size_t n = std::min(cap, c->nrec_done - c->rec_head);
  if (n) {
    memcpy(out, c->recs.data() + c->rec_head, n * sizeof(zc_record));
    c->rec_head += n;
    // between calls every record cut is complete (nrec_done == size): drop
    // the taken prefix once it is most of the vector (amortised O(1) per record)
    if (c->rec_head >= 65536 && 2 * c->rec_head >= c->recs.size() && c->nrec_done == c->recs.size()) {
      c->recs.erase_front(c->rec_head);
      c->nrec_done -= c->rec_head;
      c->rec_head = 0;
    }
  }
  if (n_out) *n_out = n;
  return ZC_OK;
}

int zc_get_stats(const zc_ctx* c, zc_stats* out) {
  ZC_LOCK(c);
  if (!c || !out) return ZC_ERR_ARG;
  if (c->win_alloc.joinable()) const_cast<zc_ctx*>(c)->win_alloc.join();  // (its error stays for window_open)
  *out = c->stats;
  out->hbm_bytes = ctx_hbm_bytes(*c);
  out->hist_entries = c->nhist;
  out->hist_seeded = c->nhist_seeded;
  out->by_value = c->statics.size();
  out->window_bytes = c->win_cap;
  return ZC_OK;
}

int zc_reset(zc_ctx* c) {
  ZC_LOCK(c);
  if (!c) return ZC_ERR_ARG;
  if (c->res) {
    (void)hipStreamSynchronize(c->stream);
    window_close(*c);
  }
  c->n_stream = 0;
  c->wbase = c->wend = 0;
  c->finished = false;
  c->d_last = nullptr;
  c->n_last = 0;
  c->recs.clear();
  c->nrec_done = 0;
  c->rec_head = 0;
  c->err.clear();
  return ZC_OK;
}

int zc_forget_stream_chunks(zc_ctx* c) {
  ZC_LOCK(c);
  if (!c) return ZC_ERR_ARG;
  return guarded(c, [&] {
    DeviceGuard g(c->device);
    c->statics.erase(std::remove_if(c->statics.begin(), c->statics.end(),
                                    [](const StaticEntry& e) { return !e.seeded; }),
                     c->statics.end());
    index_truncate(*c, c->nhist_seeded, c->statics.size(), true);
  });
}

int zc_read_stream(const zc_ctx* c, uint64_t offset, size_t n, void* host_out) {
  ZC_LOCK(c);
  if (!c || (n && !host_out)) return ZC_ERR_ARG;
  if (c->windowed_last) {
    // the bytes still in the window (the host mirror)
    if (offset < c->wbase || offset > c->wend || n > c->wend - offset) return ZC_ERR_ARG;
    if (n) memcpy(host_out, c->hwin.p + (offset - c->wbase), n);
    return ZC_OK;
  }
  if (offset > c->n_last || n > c->n_last - offset) return ZC_ERR_ARG;
  if (!n) return ZC_OK;
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(c->device) != hipSuccess) return ZC_ERR_HIP;
  hipError_t e = hipMemcpy(host_out, c->d_last + offset, n, hipMemcpyDeviceToHost);
  if (prev >= 0) (void)hipSetDevice(prev);
  return e == hipSuccess ? ZC_OK : ZC_ERR_HIP;
}

const void* zc_stream_data(const zc_ctx* c, uint64_t offset, size_t n) {
  if (!c) return nullptr;
  ZC_LOCK(c);
  if (!c->windowed_last || !c->hwin.p || offset < c->wbase || offset > c->wend || n > c->wend - offset)
    return nullptr;
  return c->hwin.p + (offset - c->wbase);
}

// Message::serialize of BackupInstruction (message.cc:16-23, zbackup.proto:149-159): a
// varint32 length, then field 1 (chunk_to_emit: ChunkId::toBlob, chunk_id.cc:19-27) or field
// 2 (bytes_to_emit), each a tag byte, a varint length and the bytes
static size_t varint_len(uint64_t v) {
  size_t k = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++k;
  }
  return k;
}
static uint8_t* put_varint(uint8_t* p, uint64_t v) {
  while (v >= 0x80) {
    *p++ = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  *p++ = (uint8_t)v;
  return p;
}

int zc_serialize_records(const zc_ctx* c, const zc_record* recs, size_t n, void* out, size_t cap, size_t* n_out) {
  ZC_LOCK(c);
  if (!c || (n && !recs) || !n_out || (cap && !out)) return ZC_ERR_ARG;
  size_t need = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t len = recs[i].kind == ZC_BYTES ? recs[i].size : 24;
    const uint64_t body = 1 + varint_len(len) + len;
    need += varint_len(body) + body;
  }
  *n_out = need;
  if (need > cap) return ZC_ERR_ARG;  // *n_out: the bytes needed
  uint8_t* p = (uint8_t*)out;
  for (size_t i = 0; i < n; ++i) {
    const zc_record& r = recs[i];
    const bool raw = r.kind == ZC_BYTES;
    const uint64_t len = raw ? r.size : 24;
    p = put_varint(p, 1 + varint_len(len) + len);
    *p++ = raw ? 0x12 : 0x0a;
    p = put_varint(p, len);
    if (raw) {
      const int rc = zc_read_stream(c, r.offset, r.size, p);  // the bytes of bytes_to_emit
      if (rc != ZC_OK) return rc;
    } else {
      memcpy(p, r.sha1, 16);  // ChunkId::toBlob: SHA-1 prefix, then the rolling hash LE
      for (int k = 0; k < 8; ++k) p[16 + k] = (uint8_t)(r.rolling >> (8 * k));
    }
    p += len;
  }
  return ZC_OK;
}

const char* zc_last_error(const zc_ctx* c) { return c ? c->err.c_str() : "null context"; }

int zc_fill_splitmix64(void* d_data, uint64_t n, uint64_t seed, int device) {
  if (n && !d_data) return ZC_ERR_ARG;
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return ZC_ERR_HIP;
  hipError_t e = launch_fill_splitmix64((uint8_t*)d_data, n, seed, nullptr);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (prev >= 0) (void)hipSetDevice(prev);
  return e == hipSuccess ? ZC_OK : ZC_ERR_HIP;
}

}  // extern "C"

// ---- bundle writer offload (zc_lzo.hip) ----

int zc_bundle_plan(const uint64_t* sizes, size_t n, uint64_t max_payload, uint32_t* bundle_of, size_t* n_bundles) {
  if ((n && (!sizes || !bundle_of)) || !n_bundles) return ZC_ERR_ARG;
  // Writer::add: getCurrentBundle() makes a bundle before the size test, so a
  // chunk larger than max_payload finishes even an empty current bundle
  size_t nb = 0;
  uint64_t payload = 0;
  bool open = false;
  for (size_t i = 0; i < n; i++) {
    if (!open) {
      open = true;
      payload = 0;
      nb++;
    }
    if (payload + sizes[i] > max_payload) {
      nb++;
      payload = 0;
    }
    bundle_of[i] = (uint32_t)(nb - 1);
    payload += sizes[i];
  }
  *n_bundles = nb;
  return ZC_OK;
}

static int lzo_fail(zc_ctx* c, hipError_t e, const char* what) {
  c->err = std::string(what) + ": " + hipGetErrorString(e);
  return e == hipErrorOutOfMemory ? ZC_ERR_NOMEM : ZC_ERR_HIP;
}

int zc_bundle_gather(zc_ctx* c, const void* d_src, const uint64_t* src_off, const uint64_t* sizes, size_t n,
                     void* d_payload) {
  ZC_LOCK(c);
  if (!c || (n && (!d_src || !src_off || !sizes || !d_payload))) return ZC_ERR_ARG;
  if (!n) return ZC_OK;
  DeviceGuard g(c->device);
  if (!c->lzo) c->lzo = lzo_scratch_new();
  hipError_t e = hipEventRecord(c->ev_in, nullptr);  // after the caller's default-stream work
  if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_in, 0);
  if (e == hipSuccess)
    e = lzo_gather(c->lzo, (const uint8_t*)d_src, src_off, sizes, n, (uint8_t*)d_payload, c->stream);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(c->stream);
    return lzo_fail(c, e, "zc_bundle_gather");
  }
  c->err.clear();
  return ZC_OK;
}

uint64_t zc_lzo_capacity(uint64_t payload_size) { return payload_size + payload_size / 16 + 64 + 3 + 16; }

int zc_lzo_compress(zc_ctx* c, const void* d_payload, const uint64_t* pay_off, const uint64_t* pay_size, size_t n,
                    void* d_out, const uint64_t* out_off, uint64_t* out_size) {
  ZC_LOCK(c);
  if (!c || (n && (!d_payload || !pay_off || !pay_size || !d_out || !out_off || !out_size))) return ZC_ERR_ARG;
  for (size_t i = 0; i < n; i++)
    if (pay_size[i] > 0xffffffffull) {  // compression.cc:437-438
      c->err = "zc_lzo_compress: a payload of 4 GiB or more";
      return ZC_ERR_ARG;
    }
  if (!n) return ZC_OK;
  DeviceGuard g(c->device);
  if (!c->lzo) c->lzo = lzo_scratch_new();
  hipError_t e = hipEventRecord(c->ev_in, nullptr);
  if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_in, 0);
  if (e == hipSuccess)
    e = lzo_compress(c->lzo, (const uint8_t*)d_payload, pay_off, pay_size, n, (uint8_t*)d_out, out_off, out_size,
                     c->stream);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(c->stream);
    return lzo_fail(c, e, "zc_lzo_compress");
  }
  c->err.clear();
  return ZC_OK;
}

int zc_lzo_compress_host(zc_ctx* c, const void* payload, const uint64_t* pay_off, const uint64_t* pay_size,
                         size_t n, void* out, const uint64_t* out_off, uint64_t* out_size) {
  ZC_LOCK(c);
  if (!c || (n && (!payload || !pay_off || !pay_size || !out || !out_off || !out_size))) return ZC_ERR_ARG;
  uint64_t in_end = 0, out_end = 0;
  for (size_t i = 0; i < n; i++) {
    if (pay_size[i] > 0xffffffffull) {
      c->err = "zc_lzo_compress_host: a payload of 4 GiB or more";
      return ZC_ERR_ARG;
    }
    in_end = std::max(in_end, pay_off[i] + pay_size[i]);
    out_end = std::max(out_end, out_off[i] + zc_lzo_capacity(pay_size[i]));
  }
  if (!n) return ZC_OK;
  return guarded(c, [&] {
    DeviceGuard g(c->device);
    if (!c->lzo) c->lzo = lzo_scratch_new();
    c->lzo_in.ensure(in_end);
    c->lzo_out.ensure(out_end);
    HCK(hipMemcpyAsync(c->lzo_in.p, payload, in_end, hipMemcpyHostToDevice, c->stream));
    HCK(lzo_compress(c->lzo, c->lzo_in.p, pay_off, pay_size, n, c->lzo_out.p, out_off, out_size, c->stream));
    for (size_t i = 0; i < n; i++)
      HCK(hipMemcpyAsync((uint8_t*)out + out_off[i], c->lzo_out.p + out_off[i], out_size[i], hipMemcpyDeviceToHost,
                         c->stream));
    HCK(hipStreamSynchronize(c->stream));
  });
}

int zc_adler32(zc_ctx* c, const void* d_base, const uint64_t* off, const uint64_t* len, size_t n, uint32_t* out) {
  ZC_LOCK(c);
  if (!c || (n && (!d_base || !off || !len || !out))) return ZC_ERR_ARG;
  if (!n) return ZC_OK;
  DeviceGuard g(c->device);
  if (!c->lzo) c->lzo = lzo_scratch_new();
  hipError_t e = hipEventRecord(c->ev_in, nullptr);
  if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_in, 0);
  if (e == hipSuccess) e = lzo_adler32(c->lzo, (const uint8_t*)d_base, off, len, n, out, c->stream);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(c->stream);
    return lzo_fail(c, e, "zc_adler32");
  }
  c->err.clear();
  return ZC_OK;
}

int zc_lzo_last_stats(const zc_ctx* c, double* parse_ms, uint64_t* blocks) {
  ZC_LOCK(c);
  if (!c) return ZC_ERR_ARG;
  const LzoTimes t = c->lzo ? *lzo_times(c->lzo) : LzoTimes{};
  if (parse_ms) *parse_ms = t.parse_ms;
  if (blocks) *blocks = t.blocks;
  return ZC_OK;
}
