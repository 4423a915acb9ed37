// zc_gen.cpp -- TEST INFRASTRUCTURE ONLY: seeded synthetic byte streams for
// the golden fixtures and parity tests (spec grammar in zc_oracle.h).
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "zc_oracle.h"

extern "C" int zco_gen(const char* spec, uint8_t** out, uint64_t* n) {
  std::vector<uint8_t> buf;
  std::string s(spec ? spec : "");
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    std::string seg = s.substr(i, j - i);
    i = j + 1;
    if (seg.empty()) continue;
    size_t colon = seg.find(':');
    if (colon == std::string::npos) return -1;
    char type = seg[0];
    std::string arg = seg.substr(1, colon - 1);
    uint64_t len = strtoull(seg.c_str() + colon + 1, 0, 0);
    size_t base = buf.size();
    buf.resize(base + len);
    if (type == 'R') {
      zco_fill_splitmix64(buf.data() + base, len, strtoull(arg.c_str(), 0, 0));
    } else if (type == 'Z') {
      // already zero
    } else if (type == 'B') {
      memset(buf.data() + base, (int)strtoul(arg.c_str(), 0, 0), len);
    } else if (type == 'C') {
      uint64_t src = strtoull(arg.c_str(), 0, 0);
      if (src >= base) return -2;
      for (uint64_t k = 0; k < len; ++k) buf[base + k] = buf[src + k];
    } else {
      return -3;
    }
  }
  uint8_t* p = (uint8_t*)malloc(buf.size() ? buf.size() : 1);
  if (!p) return -4;
  if (!buf.empty()) memcpy(p, buf.data(), buf.size());
  *out = p;
  *n = buf.size();
  return 0;
}
