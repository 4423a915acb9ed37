// zc_oracle_cli.cpp -- TEST INFRASTRUCTURE ONLY.  Prints the record list of a
// synthetic stream: used by tests/golden/make_golden.py (built against the
// reference's own rolling_hash.cc as oracle/_ref/zco_ref_cli) and for manual
// checks.  Usage: zco_cli <spec> <W> [feed_max] [--time]
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "zc_oracle.h"

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <spec> <W> [feed_max] [--time]\n", argv[0]);
    return 2;
  }
  uint8_t* data;
  uint64_t n;
  if (zco_gen(argv[1], &data, &n)) {
    fprintf(stderr, "bad spec\n");
    return 2;
  }
  uint32_t W = (uint32_t)strtoul(argv[2], 0, 0);
  uint64_t feed = argc > 3 ? strtoull(argv[3], 0, 0) : 0;
  int timing = argc > 4 && !strcmp(argv[4], "--time");
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  zco_record* r;
  size_t nr;
  if (zco_chunk(data, n, W, 0, 0, feed, &r, &nr)) return 1;
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (timing) {
    double s = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    fprintf(stderr, "%" PRIu64 " bytes in %.3f s = %.1f MiB/s, %zu records\n", n, s,
            n / s / 1048576.0, nr);
  }
  printf("# n=%" PRIu64 " W=%u records=%zu\n", n, W, nr);
  static const char kinds[] = "NDB";
  for (size_t i = 0; i < nr; ++i) {
    printf("%c %" PRIu64 " %u %016" PRIx64 " ", kinds[r[i].kind], r[i].offset, r[i].size, r[i].rolling);
    for (int k = 0; k < 16; ++k) printf("%02x", r[i].sha1[k]);
    printf("\n");
  }
  zco_free(r);
  free(data);
  return 0;
}
