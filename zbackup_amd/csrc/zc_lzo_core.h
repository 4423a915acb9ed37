// LZO1X-1 block parse, encoding and per-bundle assembly, shared by the GPU
// bundle compressor (zc_lzo.hip) and its CPU unit check
// (tests/lzo/lzo_core_check.cpp, which compares it with liblzo2's own
// lzo1x_1_compress; test infrastructure only).
//
// What zbackup runs: Bundle::Creator::write (bundle.cc:96-155) feeds a bundle's
// payload to the selected compression; for "lzo1x_1" that is
// LZO1X_1_Encoder::doProcessNoSize (compression.cc:586-606) = liblzo2 2.10's
// lzo1x_1_compress (third-party, not vendored in the reference; the image has
// liblzo2 2.10 under /opt/conda/lib, which the tests run as the oracle).
//
// lzo1x_1_compress (LZO_DETERMINISTIC build, the default) cuts its input into
// 49152-byte blocks while more than 20 bytes remain, resets its 2^14-entry
// dictionary per block and parses each block greedily; the only state a block
// inherits is the count `ti` of literals still pending from the blocks before
// it.  A block that contains a match ends at least 10 bytes past its last
// match (the match extension stops short of the block's end - 20), and a
// block without one passes on ti + its length, so every block but a payload's
// first starts with ti >= 4: its parse does not depend on the blocks before
// it.  (One more rule of the block loop: a block whose length plus the
// pending literals is under 32 bytes is not parsed at all -- a side effect of
// the loop's pointer-overflow guard -- which only a payload of 21-31 bytes or
// a short last block can meet; chain_bundle applies it.)  Each block is
// therefore parsed on its own lane (the first with ti = 0)
// and encodes itself into a staging area — everything from its first match
// on; the first literal run's header and bytes (which include the inherited
// ti literals) are written by a per-bundle assembly pass (chain_bundle) that
// walks the blocks in order.
#pragma once
#include <stdint.h>

#ifndef ZC_HD
#define ZC_HD
#endif

namespace zclzo {

constexpr uint32_t kBlock = 49152;        // DO_COMPRESS: ll = LZO_MIN(l, 49152)
constexpr uint32_t kMinBlock = 21;        // DO_COMPRESS: while (l > 20)
constexpr uint32_t kDictBits = 14;        // lzo1x_1.c: D_BITS
constexpr uint32_t kDictSize = 1u << kDictBits;
constexpr uint32_t kM2MaxLen = 8, kM3MaxLen = 33, kM4MaxLen = 9;
constexpr uint32_t kM2MaxOffset = 0x0800, kM3MaxOffset = 0x4000;
constexpr uint8_t kM3Marker = 32, kM4Marker = 16;
// staging for one block's encoding: lzo's own bound (in + in/16 + 64 + 3)
// plus slack for the 8-byte literal copies; a multiple of 16
constexpr uint32_t kStageCap = 52320;
static_assert(kStageCap >= kBlock + kBlock / 16 + 64 + 3 + 8 && kStageCap % 16 == 0, "stage");

ZC_HD inline uint32_t ld32(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}
ZC_HD inline uint64_t ld64(const uint8_t* p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}
ZC_HD inline void st64(uint8_t* p, uint64_t v) { __builtin_memcpy(p, &v, 8); }

// DINDEX (lzo1x_1.c): the top D_BITS of a 32-bit multiply
ZC_HD inline uint32_t dindex(uint32_t dv) { return (0x1824429du * dv) >> (32 - kDictBits); }

// ---- token encoding (lzo1x_c.ch) ----

// a run of 255-steps: zero bytes while more than 255 remain, then the rest
ZC_HD inline uint8_t* put_run(uint8_t* op, uint32_t tt) {
  while (tt > 255) {
    tt -= 255;
    *op++ = 0;
  }
  *op++ = (uint8_t)tt;
  return op;
}

// header of a literal run of L >= 4 (runs of 1-3 after a match have none:
// their count is or-ed into the match's second-to-last byte)
ZC_HD inline uint8_t* put_lit_header(uint8_t* op, uint32_t L) {
  if (L <= 18) {
    *op++ = (uint8_t)(L - 3);
    return op;
  }
  *op++ = 0;
  return put_run(op, L - 18);
}

// match encoding (M2 / M3 / M4)
ZC_HD inline uint8_t* put_match(uint8_t* op, uint32_t len, uint32_t off) {
  if (len <= kM2MaxLen && off <= kM2MaxOffset) {
    off -= 1;
    *op++ = (uint8_t)(((len - 1) << 5) | ((off & 7) << 2));
    *op++ = (uint8_t)(off >> 3);
    return op;
  }
  if (off <= kM3MaxOffset) {
    off -= 1;
    if (len <= kM3MaxLen) {
      *op++ = (uint8_t)(kM3Marker | (len - 2));
    } else {
      *op++ = kM3Marker;
      op = put_run(op, len - kM3MaxLen);
    }
  } else {
    off -= 0x4000;
    uint8_t hi = (uint8_t)((off >> 11) & 8);
    if (len <= kM4MaxLen) {
      *op++ = (uint8_t)(kM4Marker | hi | (len - 2));
    } else {
      *op++ = (uint8_t)(kM4Marker | hi);
      op = put_run(op, len - kM4MaxLen);
    }
  }
  *op++ = (uint8_t)(off << 2);
  *op++ = (uint8_t)(off >> 6);
  return op;
}

// ---- one block ----

// per-block result of the parse
struct BlkOut {
  uint32_t ntok;    // matches in the block
  uint32_t lit0;    // literals before the first match, from the block start
  uint32_t tail;    // literals after the last match (the block's length if none)
  uint32_t staged;  // bytes of the staged encoding (first match onwards)
};

// Parse one block (do_compress in lzo1x_c.ch, the LZO_DETERMINISTIC path) and
// stage its encoding.  `in` points at the block, `ll` is its length
// (21 .. 49152), `ti` the literals pending before it (only min(ti, 4)
// matters).  Dict provides `uint32_t exchange(uint32_t index, uint32_t pos)`:
// the position last stored at index (0 if none), storing pos.  `op` receives
// the staged bytes (kStageCap).
template <class Dict>
ZC_HD inline BlkOut parse_block(const uint8_t* in, uint32_t ll, uint32_t ti, Dict& dict, uint8_t* const stage) {
  const uint32_t ip_end = ll - 20;
  uint32_t ip = ti < 4 ? 4 - ti : 0;
  uint32_t ii = 0;
  uint8_t* op = stage;
  BlkOut r{0, 0, 0, 0};
  ip += 1 + ((ip - ii) >> 5);  // the first probe (the loop's "literal" step)
  uint32_t dv = ip < ip_end ? ld32(in + ip) : 0;
  for (;;) {
    if (ip >= ip_end) break;
    const uint32_t m = dict.exchange(dindex(dv), ip);
    // the next probe of a literal run and its bytes, loaded while the
    // dictionary entry's bytes are (the step depends on ip and ii only)
    const uint32_t ip_lit = ip + 1 + ((ip - ii) >> 5);
    const uint32_t dv_lit = ip_lit < ip_end ? ld32(in + ip_lit) : 0;
    if (dv != ld32(in + m)) {
      ip = ip_lit;
      dv = dv_lit;
      continue;
    }
    // a match: extend it 8 bytes at a time, stopping once past ip_end
    uint32_t m_len = 4;
    uint64_t v = ld64(in + ip + m_len) ^ ld64(in + m + m_len);
    if (v == 0) {
      do {
        m_len += 8;
        v = ld64(in + ip + m_len) ^ ld64(in + m + m_len);
        if (ip + m_len >= ip_end) goto m_len_done;
      } while (v == 0);
    }
    m_len += (uint32_t)__builtin_ctzll(v) / 8;
  m_len_done:
    {
      const uint32_t lit = ip - ii;
      if (r.ntok == 0) {
        r.lit0 = lit;  // written by chain_bundle with the inherited literals
      } else if (lit) {
        if (lit <= 3) {
          op[-2] |= (uint8_t)lit;
        } else {
          op = put_lit_header(op, lit);
        }
        // 8-byte copies; the overrun (< 8 bytes, inside the block: a match
        // of >= 4 bytes follows and ip < ll - 20) is overwritten next
        for (uint32_t k = 0; k < lit; k += 8) st64(op + k, ld64(in + ii + k));
        op += lit;
      }
      op = put_match(op, m_len, ip - m);
      r.ntok++;
    }
    ip += m_len;
    ii = ip;
    if (ip < ip_end) dv = ld32(in + ip);
  }
  r.tail = ll - ii;
  r.staged = (uint32_t)(op - stage);
  return r;
}

// ---- one bundle ----

// zbackup's framing of an lzo1x_1 payload (NoStreamAndUnknownSizeEncoder::
// doProcess, compression.cc:435-466): the template "ABCDEFGHIJKLMNOP", its
// first 4 bytes overwritten with the uncompressed size (LE32), bytes 8-11 with
// the compressed size (LE32); the LZO stream follows.
constexpr uint32_t kFrame = 16;
ZC_HD inline void put_frame(uint8_t* out, uint32_t n, uint32_t csize) {
  const char tmpl[17] = "ABCDEFGHIJKLMNOP";
  for (int i = 0; i < 16; i++) out[i] = (uint8_t)tmpl[i];
  for (int i = 0; i < 4; i++) out[i] = (uint8_t)(n >> (8 * i));
  for (int i = 0; i < 4; i++) out[8 + i] = (uint8_t)(csize >> (8 * i));
}

// output capacity zbackup reserves for a payload (LZO1X_1_Encoder::
// suggestOutputSize + the framing, compression.cc:566-583)
ZC_HD inline uint64_t frame_capacity(uint64_t n) { return n + n / 16 + 64 + 3 + kFrame; }

// blocks of a payload of n bytes
ZC_HD inline uint32_t block_count(uint64_t n) {
  uint32_t k = 0;
  if (n <= 20) return 0;
  k = (uint32_t)(n / kBlock);
  uint64_t rem = n - (uint64_t)k * kBlock;
  return rem > 20 ? k + 1 : k;
}

// copies chain_bundle asks for (literal runs from the payload, staged
// encodings): at most 2 per block + 1; split into pieces of at most kPiece
// bytes, at most one more piece per kPiece of output
constexpr uint64_t kPiece = 1u << 16;
ZC_HD inline uint64_t copies_cap(uint32_t nblk, uint64_t n) { return 2ull * nblk + 1 + frame_capacity(n) / kPiece + 1; }

// Assemble one bundle (DO_COMPRESS in lzo1x_c.ch after the block loop, and the
// framing): writes the frame, every block's first literal-run header, the final
// literal run's header and the end marker (M4_MARKER | 1, 0, 0) into `out`, and
// asks `copy(src_is_stage, src_index_or_offset, dst_offset, n)` for the
// literal runs (from the payload, offsets relative to the payload's start) and
// the staged block encodings.  A final run of 1-3 literals after a match is
// or-ed into the last match's second-to-last byte: *or_at / *or_val (0: none)
// for after the copies.  Returns the framed size.
template <class Copy>
ZC_HD inline uint64_t chain_bundle(uint64_t n, const BlkOut* bo, uint8_t* out, Copy& copy, uint64_t* or_at,
                                   uint32_t* or_val) {
  uint64_t pos = kFrame, start = 0, rem = n, ti = 0;
  uint32_t k = 0;
  bool any = false;
  uint64_t last_or = 0;
  *or_at = 0;
  *or_val = 0;
  while (rem > 20) {
    const uint32_t ll = rem < kBlock ? (uint32_t)rem : kBlock;
    // DO_COMPRESS's overflow guard `(ll_end + ((t + ll) >> 5)) <= ll_end` also
    // holds when the pending literals and the block are under 32 bytes: the
    // block is not parsed and everything left is literals (only a payload of
    // 21-31 bytes, or a short last block, meets it; its parse is ignored)
    if (((ti + ll) >> 5) == 0) break;
    const BlkOut o = bo[k];
    if (o.ntok) {
      const uint64_t L0 = ti + o.lit0;
      pos = (uint64_t)(put_lit_header(out + pos, (uint32_t)L0) - out);
      copy(false, start - ti, pos, L0);
      pos += L0;
      copy(true, k, pos, o.staged);
      pos += o.staged;
      last_or = pos - 2;
      any = true;
      ti = o.tail;
    } else {
      ti += ll;
    }
    start += ll;
    rem -= ll;
    k++;
  }
  const uint64_t T = ti + rem;
  if (T) {
    if (any && T <= 3) {
      *or_at = last_or;
      *or_val = (uint32_t)T;
    } else {
      if (!any && T <= 238)
        out[pos++] = (uint8_t)(17 + T);
      else
        pos = (uint64_t)(put_lit_header(out + pos, (uint32_t)T) - out);
      copy(false, n - T, pos, T);
      pos += T;
    }
  }
  out[pos++] = kM4Marker | 1;
  out[pos++] = 0;
  out[pos++] = 0;
  put_frame(out, (uint32_t)n, (uint32_t)(pos - kFrame));
  return pos;
}

}  // namespace zclzo
