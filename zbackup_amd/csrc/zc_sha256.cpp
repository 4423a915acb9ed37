// Whole-stream SHA-256 of a backup's input (host side of the feed loop).
//
// The reference hashes every buffer it feeds to BackupCreator with OpenSSL's
// SHA256_Update (zutils.cc:94,119 -> sha256.cc:13-16) and stores the digest in
// BackupInfo.sha256 (zutils.cc:134); restore re-hashes and compares it
// (zutils.cc:225-232,252-264). OpenSSL is not a dependency here, so this file
// restates FIPS 180-4 SHA-256: a scalar compression function plus, on x86 hosts
// with the SHA extensions (the GPU box's EPYC has them), the sha256rnds2 /
// sha256msg1/2 form, chosen once by cpuid. It is one serial chain over the whole
// stream, so it stays on the host CPU beside the device's chunking; the GPU has no
// parallel form of it to offer.
#include <cpuid.h>
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "zchunk.h"

namespace {

alignas(16) const uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void blocks_scalar(uint32_t s[8], const uint8_t* p, size_t nblk) {
  for (; nblk; --nblk, p += 64) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 |
             p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
      uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
    for (int i = 0; i < 64; ++i) {
      uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
  }
}

// The state travels as {A,B,E,F} / {C,D,G,H} lanes, the layout sha256rnds2 takes;
// the message schedule advances four words per step with sha256msg1/msg2.
__attribute__((target("sha,sse4.1,ssse3")))
void blocks_shani(uint32_t s[8], const uint8_t* p, size_t nblk) {
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i t = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&s[0]), 0xB1);  // C D A B
  __m128i st1 = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&s[4]), 0x1B);  // E F G H
  __m128i st0 = _mm_alignr_epi8(t, st1, 8);                                     // A B E F
  st1 = _mm_blend_epi16(st1, t, 0xF0);                                          // C D G H
  for (; nblk; --nblk, p += 64) {
    const __m128i save0 = st0, save1 = st1;
    __m128i w[4];
    for (int g = 0; g < 16; ++g) {
      __m128i m;
      if (g < 4) {
        m = w[g] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * g)), bswap);
      } else {
        __m128i& w0 = w[g & 3];                       // words 4g-16 .. 4g-13
        const __m128i& w1 = w[(g + 1) & 3];           // 4g-12 ..
        const __m128i& w2 = w[(g + 2) & 3];           // 4g-8 ..
        const __m128i& w3 = w[(g + 3) & 3];           // 4g-4 ..
        w0 = _mm_sha256msg2_epu32(
            _mm_add_epi32(_mm_sha256msg1_epu32(w0, w1), _mm_alignr_epi8(w3, w2, 4)), w3);
        m = w0;
      }
      m = _mm_add_epi32(m, _mm_load_si128((const __m128i*)&K[4 * g]));
      st1 = _mm_sha256rnds2_epu32(st1, st0, m);
      st0 = _mm_sha256rnds2_epu32(st0, st1, _mm_shuffle_epi32(m, 0x0E));
    }
    st0 = _mm_add_epi32(st0, save0);
    st1 = _mm_add_epi32(st1, save1);
  }
  t = _mm_shuffle_epi32(st0, 0x1B);                    // F E B A
  st1 = _mm_shuffle_epi32(st1, 0xB1);                  // D C H G
  _mm_storeu_si128((__m128i*)&s[0], _mm_blend_epi16(t, st1, 0xF0));  // D C B A
  _mm_storeu_si128((__m128i*)&s[4], _mm_alignr_epi8(st1, t, 8));     // H G F E
}

bool have_shani() {
  unsigned a, b, c, d;
  if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
  if (!(b & (1u << 29))) return false;  // SHA
  __get_cpuid(1, &a, &b, &c, &d);
  return (c & (1u << 19)) && (c & (1u << 9));  // SSE4.1, SSSE3
}

using blocks_fn = void (*)(uint32_t*, const uint8_t*, size_t);

blocks_fn pick() {
  const char* force = getenv("ZC_SHA256_SCALAR");
  if (force && *force == '1') return blocks_scalar;
  return have_shani() ? blocks_shani : blocks_scalar;
}

}  // namespace

struct zc_sha256 {
  uint32_t h[8];
  uint64_t total;
  uint8_t buf[64];
  uint32_t fill;
  bool done;
  blocks_fn blocks;
};

extern "C" {

int zc_sha256_create(zc_sha256** out) {
  if (!out) return ZC_ERR_ARG;
  zc_sha256* c = (zc_sha256*)calloc(1, sizeof(zc_sha256));
  if (!c) return ZC_ERR_NOMEM;
  static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(c->h, iv, sizeof iv);
  c->blocks = pick();
  *out = c;
  return ZC_OK;
}

int zc_sha256_add(zc_sha256* c, const void* data, size_t n) {
  if (!c || (!data && n) || c->done) return ZC_ERR_ARG;
  const uint8_t* p = (const uint8_t*)data;
  c->total += n;
  if (c->fill) {
    size_t take = 64 - c->fill < n ? 64 - c->fill : n;
    memcpy(c->buf + c->fill, p, take);
    c->fill += (uint32_t)take; p += take; n -= take;
    if (c->fill < 64) return ZC_OK;
    c->blocks(c->h, c->buf, 1);
    c->fill = 0;
  }
  if (n >= 64) {
    c->blocks(c->h, p, n / 64);
    p += n & ~(size_t)63; n &= 63;
  }
  memcpy(c->buf, p, n);
  c->fill = (uint32_t)n;
  return ZC_OK;
}

int zc_sha256_finish(zc_sha256* c, uint8_t out[32]) {
  if (!c || !out || c->done) return ZC_ERR_ARG;
  uint64_t bits = c->total * 8;
  uint8_t pad[72] = {0x80};
  size_t padlen = (c->fill < 56 ? 56 : 120) - c->fill;
  for (int i = 0; i < 8; ++i) pad[padlen + i] = (uint8_t)(bits >> (56 - 8 * i));
  uint64_t keep = c->total;
  zc_sha256_add(c, pad, padlen + 8);
  c->total = keep;
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(c->h[i] >> 24); out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(c->h[i] >> 8); out[4 * i + 3] = (uint8_t)c->h[i];
  }
  c->done = true;
  return ZC_OK;
}

int zc_sha256_destroy(zc_sha256* c) {
  if (!c) return ZC_ERR_ARG;
  free(c);
  return ZC_OK;
}

int zc_sha256_impl(const zc_sha256* c) {
  if (!c) return -1;
  return c->blocks == blocks_shani ? 1 : 0;
}

}  // extern "C"
