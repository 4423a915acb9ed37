// Test infrastructure: checks zc_lzo_core.h (the LZO1X-1 parse, staging and
// bundle assembly the GPU bundle compressor runs) against liblzo2 2.10's own
// lzo1x_1_compress on the same inputs, compiled for the host.  Every block is
// parsed independently (ti = 0 for a payload's first block, else the real
// inherited count, which must be >= 4) and staged, then each payload is
// assembled as zc_lzo.hip does.  Prints "ok N" or the first mismatch.  Built
// and run by tests/test_lzo.py (g++ against /opt/conda/lib/liblzo2.so.2).
#include <lzo/lzo1x.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "zc_lzo_core.h"

using namespace zclzo;

struct HostDict {  // lzo1x_1's dictionary, reset per block
  std::vector<uint32_t> d = std::vector<uint32_t>(kDictSize, 0);
  uint32_t exchange(uint32_t i, uint32_t pos) {
    uint32_t o = d[i];
    d[i] = pos;
    return o;
  }
};

// the GPU pipeline's steps, in order: every block parsed on its own
// (zc_lzo_parse_kernel), then the bundle assembled (zc_lzo_chain_kernel), the
// copies done (zc_lzo_copy_kernel) and the final or applied
static std::vector<uint8_t> core_compress(const uint8_t* in, size_t n) {
  const uint32_t nb = block_count(n);
  std::vector<BlkOut> bo(nb);
  std::vector<uint8_t> stage((size_t)nb * kStageCap);
  size_t pos = 0;
  for (uint32_t k = 0; k < nb; k++) {
    const uint32_t ll = (uint32_t)std::min<size_t>(n - pos, kBlock);
    HostDict dict;
    bo[k] = parse_block(in + pos, ll, k == 0 ? 0 : 4, dict, stage.data() + (size_t)k * kStageCap);
    pos += ll;
  }
  std::vector<uint8_t> out(frame_capacity(n));
  auto copy = [&](bool from_stage, uint64_t src, uint64_t dst, uint64_t len) {
    const uint8_t* s = from_stage ? stage.data() + src * kStageCap : in + src;
    memcpy(out.data() + dst, s, len);
  };
  uint64_t or_at;
  uint32_t or_val;
  uint64_t size = chain_bundle(n, bo.data(), out.data(), copy, &or_at, &or_val);
  if (or_val) out[or_at] |= (uint8_t)or_val;
  out.resize(size);
  return out;
}

static std::vector<uint8_t> lzo_compress(const uint8_t* in, size_t n) {
  std::vector<uint8_t> out(n + n / 16 + 64 + 3);
  std::vector<uint8_t> wrk(LZO1X_1_MEM_COMPRESS);
  lzo_uint olen = out.size();
  if (lzo1x_1_compress(in, n, out.data(), &olen, wrk.data()) != LZO_E_OK) exit(3);
  out.resize(olen);
  std::vector<uint8_t> framed(kFrame + olen);
  put_frame(framed.data(), (uint32_t)n, (uint32_t)olen);
  memcpy(framed.data() + kFrame, out.data(), olen);
  return framed;
}

static std::vector<uint8_t> make_input(uint64_t seed, size_t n, int kind) {
  std::mt19937_64 g(seed);
  std::vector<uint8_t> v(n);
  switch (kind) {
    case 0:  // random
      for (auto& b : v) b = (uint8_t)g();
      break;
    case 1:  // zeros
      break;
    case 2: {  // text-like: words from a small vocabulary
      static const char* words[] = {"the ", "backup ", "chunk ", "index ", "bundle ", "of ", "and ",
                                    "zbackup ", "rolling ", "hash ", "\n", "data ", "stream "};
      size_t i = 0;
      while (i < n) {
        const char* w = words[g() % 13];
        for (const char* c = w; *c && i < n; c++) v[i++] = (uint8_t)*c;
      }
      break;
    }
    case 3: {  // random with repeated pieces at random distances
      for (auto& b : v) b = (uint8_t)g();
      for (size_t i = 0; i + 64 < n; i += 1 + g() % 300) {
        size_t len = 4 + g() % 200, back = 1 + g() % 60000;
        if (i >= back && i + len < n) memmove(&v[i], &v[i - back], len);
      }
      break;
    }
    case 4: {  // low-entropy bytes (small alphabet)
      for (auto& b : v) b = (uint8_t)('a' + g() % 3);
      break;
    }
    case 5: {  // long runs of a few values with random bytes between
      size_t i = 0;
      while (i < n) {
        size_t run = g() % 2000;
        uint8_t c = (uint8_t)g();
        for (size_t k = 0; k < run && i < n; k++) v[i++] = (g() % 8) ? c : (uint8_t)g();
      }
      break;
    }
  }
  return v;
}

int main(int argc, char** argv) {
  if (lzo_init() != LZO_E_OK) return 3;
  int cases = argc > 1 ? atoi(argv[1]) : 400;
  const size_t sizes[] = {0, 1, 3, 4, 17, 20, 21, 22, 27, 29, 31, 32, 33, 40, 41, 100, 1000, 49151, 49152, 49153,
                          49172, 49173, 49174, 49175, 49180, 49183, 49184, 98304, 98324, 98325, 98335, 100000,
                          262144, 2097152};
  int n_ok = 0;
  for (int c = 0; c < cases; c++) {
    size_t n = c < (int)(sizeof(sizes) / sizeof(sizes[0])) * 6 ? sizes[c / 6] : (size_t)(std::mt19937_64(c)() % 3000000);
    int kind = c % 6;
    auto in = make_input(1000 + c, n, kind);
    auto a = lzo_compress(in.data(), n);
    auto b = core_compress(in.data(), n);
    if (a != b) {
      size_t i = 0;
      while (i < a.size() && i < b.size() && a[i] == b[i]) i++;
      printf("MISMATCH case %d kind %d n %zu: lzo %zu bytes, core %zu bytes, first diff at %zu\n", c, kind, n,
             a.size(), b.size(), i);
      return 1;
    }
    n_ok++;
  }
  // every length up to 160 and every short last block (49152 + 21 .. 63), all kinds
  for (int kind = 0; kind < 6; kind++)
    for (size_t n = 0; n <= 160 + 43; n++) {
      const size_t len = n <= 160 ? n : 49152 + 21 + (n - 161);
      auto in = make_input(90000 + 1000 * kind + n, len, kind);
      if (lzo_compress(in.data(), len) != core_compress(in.data(), len)) {
        printf("MISMATCH kind %d n %zu\n", kind, len);
        return 1;
      }
      n_ok++;
    }
  printf("ok %d\n", n_ok);
  return 0;
}
