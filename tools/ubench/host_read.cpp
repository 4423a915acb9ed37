// Host-side read rate of the buffers the engine copies results into:
// hipHostMalloc (default, coherent, non-coherent flags) against pageable
// memory, each filled by a device-to-host copy first, then read by one CPU
// thread (the records' SHA-1 fill reads 20 bytes per chunk this way).  Tooling only.
// Build: hipcc -O2 -std=c++17 host_read.cpp -o host_read
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                   \
    }                                                             \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t n = 2621440;  // 131,072 x 20 bytes
  uint8_t* d;
  CK(hipMalloc(&d, n));
  CK(hipMemset(d, 7, n));
  struct Kind {
    const char* name;
    unsigned flags;  // ~0u: pageable
  } kinds[] = {{"pageable", ~0u},
               {"hipHostMallocDefault", hipHostMallocDefault},
               {"hipHostMallocCoherent", hipHostMallocCoherent},
               {"hipHostMallocNonCoherent", hipHostMallocNonCoherent}};
  std::vector<uint8_t> recs(131072 * 40);
  for (auto& k : kinds) {
    uint8_t* h = nullptr;
    if (k.flags == ~0u)
      h = (uint8_t*)malloc(n);
    else
      CK(hipHostMalloc((void**)&h, n, k.flags));
    double best_copy = 1e9, best_read = 1e9, best_fill = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      double t0 = now_ms();
      CK(hipMemcpy(h, d, n, hipMemcpyDeviceToHost));
      double t1 = now_ms();
      uint64_t s = 0;
      for (size_t i = 0; i < n; i += 8) {
        uint64_t v;
        memcpy(&v, h + i, 8);
        s += v;
      }
      double t2 = now_ms();
      // the records' fill: 16 of every 20 bytes into a 40-byte record
      for (size_t q = 0; q < 131072; ++q) memcpy(&recs[q * 40 + 24], h + q * 20, 16);
      double t3 = now_ms();
      if (s == 42) printf(" ");
      best_copy = std::min(best_copy, t1 - t0);
      best_read = std::min(best_read, t2 - t1);
      best_fill = std::min(best_fill, t3 - t2);
    }
    printf("%-26s D2H %.3f ms  CPU read %.3f ms (%.2f GB/s)  record fill %.3f ms\n", k.name, best_copy, best_read,
           n / best_read / 1e6, best_fill);
    if (k.flags == ~0u)
      free(h);
    else
      CK(hipHostFree(h));
  }
  return 0;
}
