// zc_oracle.cpp -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
//
// A CPU restatement of zbackup's dedup hot path.  Only tests/, the smoke check
// in __graft_entry__.py and bench.py's cpu_baseline leg may load or run this
// code.  The product path (zbackup_amd/csrc) never links it.
//
// What it restates, and where the reference does it:
//   * RollingHash: base 257, mod 2^64, leading 257^n term
//       /root/reference/rolling_hash.hh:40-79, rolling_hash.cc:11-29
//   * BackupCreator: ring buffer of W + page bytes, fill phase (rollIn),
//     rotate phase (one rotate + one index probe per byte), max-size cut,
//     match handling, 128-byte bytes_to_emit rule, finish rules
//       /root/reference/backup_creator.cc:18-280
//   * ChunkIndex probe: __gnu_cxx::hash_map keyed by the 64-bit rolling hash
//     with the identity hash, chains of 16-byte SHA-1 prefixes, lazy SHA-1 of
//     the window only on a key hit
//       /root/reference/chunk_index.hh:37-45,61-75; chunk_index.cc:119-202
//   * ChunkStorage::Writer::add -> ChunkIndex::addChunk (synchronous, so a
//     chunk is probe-visible from the very next check)
//       /root/reference/chunk_storage.cc:31-46
//
// The code is written from the formal spec in SURVEY.md §3.3, not copied.
// Build with -DZCO_USE_REFERENCE_RH to swap this file's rolling hash for the
// reference's own RollingHash class (compiled from /root/reference/
// rolling_hash.cc by oracle/Makefile into oracle/_ref/); the golden fixtures
// under tests/golden/ are produced by that build.
//
// Third-party arithmetic: SHA-1 from OpenSSL (libcrypto), exactly as the
// reference calls it (backup_creator.cc:130-131,212-229).

#undef __DEPRECATED
#include <ext/hash_map>

#include <openssl/sha.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <string>
#include <vector>

#include "zc_oracle.h"

#ifdef ZCO_USE_REFERENCE_RH
#include "rolling_hash.hh"  // from /root/reference, via -I
typedef RollingHash OracleRH;
#else
// Restated rolling hash.  State after rolling in b_0..b_{n-1}:
//   acc  = sum b_i * 257^(n-1-i)          (mod 2^64)
//   pw   = 257^n,  pw_prev = 257^(n-1)    (pw_prev = 0 when n == 0)
// digest = acc + pw.  rotate(in,out) drops the oldest byte and appends `in`
// without changing n.
class OracleRH {
  uint64_t pw_prev_, pw_, acc_;
  size_t n_;

 public:
  OracleRH() { reset(); }
  void reset() { pw_prev_ = 0; pw_ = 1; acc_ = 0; n_ = 0; }
  void rollIn(char c) {
    pw_prev_ = pw_;
    pw_ *= 257u;
    acc_ = acc_ * 257u + (uint8_t)c;
    ++n_;
  }
  void rotate(char in, char out) {
    acc_ -= (uint64_t)(uint8_t)out * pw_prev_;
    acc_ = acc_ * 257u + (uint8_t)in;
  }
  uint64_t digest() const { return acc_ + pw_; }
  static uint64_t digest(const void* p, unsigned n) {
    OracleRH h;
    const char* b = (const char*)p;
    for (unsigned i = 0; i < n; ++i) h.rollIn(b[i]);
    return h.digest();
  }
};
#endif

namespace {

// ---------------------------------------------------------------------------
// Probe set: identity-hashed map from rolling hash to a chain of SHA-1
// prefixes, the same container and hash the reference uses, so the CPU
// baseline pays the same per-byte probe cost.
struct IdentityHash {
  size_t operator()(uint64_t v) const { return (size_t)v; }
};

struct ChainLink {
  uint8_t sha[16];
  uint32_t size;
  ChainLink* next;
};

class ProbeSet {
  typedef __gnu_cxx::hash_map<uint64_t, ChainLink*, IdentityHash> Map;
  Map map_;
  std::vector<ChainLink*> owned_;
  // Optional exact prefilter (zco_chunk_ex ZCO_OPT_PREFILTER): one bit per
  // key's low 23 bits, set on insert.  A clear bit proves the key absent, so
  // hasKey() returns the same answer with or without it; it only saves the
  // hash_map walk on misses (the parity tests' full-size runs use it; the timed
  // CPU baseline does not, to keep the reference's per-byte probe cost).
  std::vector<uint64_t> bits_;

 public:
  static const unsigned kBits = 23;
  ~ProbeSet() {
    for (size_t i = 0; i < owned_.size(); ++i) delete owned_[i];
  }
  void enablePrefilter() {
    bits_.assign((1u << kBits) / 64, 0);
    for (Map::iterator it = map_.begin(); it != map_.end(); ++it) setBit(it->first);
  }
  void setBit(uint64_t key) {
    const uint32_t b = (uint32_t)key & ((1u << kBits) - 1);
    bits_[b >> 6] |= 1ull << (b & 63);
  }
  bool hasKey(uint64_t key, Map::iterator& it) {
    if (!bits_.empty()) {
      const uint32_t b = (uint32_t)key & ((1u << kBits) - 1);
      if (!((bits_[b >> 6] >> (b & 63)) & 1)) return false;
    }
    it = map_.find(key);
    return it != map_.end();
  }
  static bool chainHas(ChainLink* c, const uint8_t* sha) {
    for (; c; c = c->next)
      if (memcmp(c->sha, sha, 16) == 0) return true;
    return false;
  }
  // Returns true if inserted (the id was new).
  bool add(uint64_t key, const uint8_t* sha, uint32_t size) {
    if (!bits_.empty()) setBit(key);
    std::pair<Map::iterator, bool> r = map_.insert(std::make_pair(key, (ChainLink*)0));
    ChainLink** slot = &r.first->second;
    for (; *slot; slot = &(*slot)->next)
      if (memcmp((*slot)->sha, sha, 16) == 0) return false;
    ChainLink* c = new ChainLink;
    memcpy(c->sha, sha, 16);
    c->size = size;
    c->next = 0;
    owned_.push_back(c);
    *slot = c;
    return true;
  }
  friend class StreamChunker;
};

// ---------------------------------------------------------------------------
// The chunker state machine.  Absolute stream offsets are tracked so every
// record carries {offset, size}; the reference only writes the instruction
// stream, whose order and contents these records determine.
class StreamChunker {
  const unsigned W_;
  ProbeSet& index_;
  std::vector<char> ring_;
  size_t head_, tail_;     // indices into ring_
  unsigned ringFill_;
  std::vector<char> pending_;
  unsigned pendingFill_;
  uint64_t pendingStart_;  // absolute stream offset of pending_[0]
  uint64_t tailPos_;       // absolute stream offset of ring_[tail_]
  OracleRH rh_;
  std::vector<zco_record>& out_;

  bool idCached_;
  uint8_t idSha_[16];

  void emitBytes(uint64_t off, unsigned size) {
    zco_record r;
    memset(&r, 0, sizeof r);
    r.offset = off;
    r.size = size;
    r.kind = ZCO_BYTES;
    out_.push_back(r);
  }

  // backup_creator.cc:110-145 restated: <128 bytes become bytes_to_emit,
  // anything else becomes a chunk {SHA-1[0:16], digest} added to the index.
  void flushPending() {
    uint64_t off = pendingStart_;
    if (pendingFill_ < 128) {
      emitBytes(off, pendingFill_);
    } else {
      zco_record r;
      memset(&r, 0, sizeof r);
      r.offset = off;
      r.size = pendingFill_;
      r.kind = ZCO_CHUNK_NEW;
      r.rolling = OracleRH::digest(pending_.data(), pendingFill_);
      uint8_t full[SHA_DIGEST_LENGTH];
      SHA1((const unsigned char*)pending_.data(), pendingFill_, full);
      memcpy(r.sha1, full, 16);
      index_.add(r.rolling, r.sha1, r.size);
      out_.push_back(r);
    }
    pendingStart_ += pendingFill_;
    pendingFill_ = 0;
  }

  // SHA-1 of the W bytes in the ring, which may wrap (backup_creator.cc:208-240)
  void windowSha(uint8_t* sha16) {
    if (!idCached_) {
      SHA_CTX c;
      SHA1_Init(&c);
      if (tail_ < head_) {
        SHA1_Update(&c, ring_.data() + tail_, head_ - tail_);
      } else {
        SHA1_Update(&c, ring_.data() + tail_, ring_.size() - tail_);
        SHA1_Update(&c, ring_.data(), head_);
      }
      uint8_t full[SHA_DIGEST_LENGTH];
      SHA1_Final(full, &c);
      memcpy(idSha_, full, 16);
      idCached_ = true;
    }
    memcpy(sha16, idSha_, 16);
  }

  // One probe: the window [tail, head) of W bytes (backup_creator.cc:242-265,
  // chunk_index.cc:119-143).
  void probe() {
    idCached_ = false;
    uint64_t key = rh_.digest();
    ProbeSet::Map::iterator it;
    if (!index_.hasKey(key, it)) return;
    uint8_t sha[16];
    windowSha(sha);
    if (!ProbeSet::chainHas(it->second, sha)) return;
    if (pendingFill_) flushPending();
    zco_record r;
    memset(&r, 0, sizeof r);
    r.offset = tailPos_;
    r.size = W_;
    r.kind = ZCO_CHUNK_DUP;
    r.rolling = key;
    memcpy(r.sha1, sha, 16);
    out_.push_back(r);
    // the window is consumed: empty ring, fresh hash, restart the fill phase
    tailPos_ += W_;
    pendingStart_ = tailPos_;
    tail_ = head_;
    ringFill_ = 0;
    rh_.reset();
  }

  void movePending(unsigned n) {
    for (unsigned i = 0; i < n; ++i) {
      pending_[pendingFill_++] = ring_[tail_];
      if (++tail_ == ring_.size()) tail_ = 0;
    }
    tailPos_ += n;
    ringFill_ -= n;
  }

 public:
  StreamChunker(unsigned W, ProbeSet& idx, std::vector<zco_record>& out)
      : W_(W), index_(idx), head_(0), tail_(0), ringFill_(0), pendingFill_(0),
        pendingStart_(0), tailPos_(0), out_(out), idCached_(false) {
    ring_.resize((size_t)W + (size_t)sysconf(_SC_PAGESIZE));
    pending_.resize(W);
  }

  // zero-copy feed contract of backup_creator.cc:40-54
  char* inputBuffer() { return ring_.data() + head_; }
  size_t inputBufferSize() const {
    if (tail_ > head_) return tail_ - head_;
    if (tail_ == head_ && ringFill_) return 0;
    return ring_.size() - head_;
  }

  void consume(unsigned n) {
    while (n) {
      if (ringFill_ < W_) {
        // fill phase: roll in until the window is full, then one probe
        unsigned need = W_ - ringFill_;
        unsigned take = n < need ? n : need;
        for (unsigned i = 0; i < take; ++i) rh_.rollIn(ring_[head_++]);
        if (head_ == ring_.size()) head_ = 0;
        ringFill_ += take;
        n -= take;
        if (ringFill_ == W_) probe();
      } else {
        // rotate phase: the oldest ring byte moves to the pending chunk
        // (cut at exactly W bytes), the hash rotates by one byte, one probe
        pending_[pendingFill_++] = ring_[tail_];
        if (pendingFill_ == W_) flushPending();
        char in = ring_[head_], outb = ring_[tail_];
        rh_.rotate(in, outb);
        if (++head_ == ring_.size()) head_ = 0;
        if (++tail_ == ring_.size()) tail_ = 0;
        tailPos_ += 1;
        probe();
        --n;
      }
    }
  }

  // backup_creator.cc:147-172 restated
  void finish() {
    if (pendingFill_ + ringFill_ > W_) {
      movePending(W_ - pendingFill_);
      flushPending();
    }
    movePending(ringFill_);
    if (pendingFill_) flushPending();
  }
};

}  // namespace

extern "C" {

uint64_t zco_digest(const uint8_t* p, uint64_t n) {
  return OracleRH::digest(p, (unsigned)n);
}

int zco_chunk(const uint8_t* data, uint64_t n, uint32_t W, const zco_seed* seeds,
              size_t nseeds, uint64_t feed_max, zco_record** out, size_t* nout) {
  return zco_chunk_ex(data, n, W, seeds, nseeds, feed_max, 0, out, nout);
}

int zco_chunk_ex(const uint8_t* data, uint64_t n, uint32_t W, const zco_seed* seeds,
                 size_t nseeds, uint64_t feed_max, uint32_t opts, zco_record** out, size_t* nout) {
  if (!out || !nout || W == 0) return -1;
  std::vector<zco_record> recs;
  {
    ProbeSet index;
    if (opts & ZCO_OPT_PREFILTER) index.enablePrefilter();
    for (size_t i = 0; i < nseeds; ++i) index.add(seeds[i].rolling, seeds[i].sha1, seeds[i].size);
    StreamChunker ch(W, index, recs);
    uint64_t pos = 0;
    // mimic zutils.cc:100-124: fread(getInputBuffer(), 1, getInputBufferSize())
    while (pos < n) {
      size_t want = ch.inputBufferSize();
      if (feed_max && want > feed_max) want = feed_max;
      if (want > n - pos) want = (size_t)(n - pos);
      memcpy(ch.inputBuffer(), data + pos, want);
      ch.consume((unsigned)want);
      pos += want;
    }
    ch.finish();
  }
  zco_record* r = (zco_record*)malloc(sizeof(zco_record) * (recs.size() ? recs.size() : 1));
  if (!r) return -2;
  if (!recs.empty()) memcpy(r, recs.data(), sizeof(zco_record) * recs.size());
  *out = r;
  *nout = recs.size();
  return 0;
}

void zco_free(void* p) { free(p); }

void zco_sha1(const uint8_t* p, uint64_t n, uint8_t* out20) { SHA1(p, n, out20); }

// ---------------------------------------------------------------------------
// Seeded synthetic streams (shared recipe with zbackup_amd's device filler,
// which the GPU tests check against this one).  Byte k of the stream is byte
// (k mod 8) of splitmix64 word floor(k / 8), little-endian; word i is the
// splitmix64 output for state seed + (i + 1) * 0x9E3779B97F4A7C15.
static inline uint64_t splitmix64_word(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void zco_fill_splitmix64(uint8_t* out, uint64_t n, uint64_t seed) {
  uint64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w = splitmix64_word(seed, i / 8);
    memcpy(out + i, &w, 8);
  }
  if (i < n) {
    uint64_t w = splitmix64_word(seed, i / 8);
    memcpy(out + i, &w, n - i);
  }
}

}  // extern "C"
