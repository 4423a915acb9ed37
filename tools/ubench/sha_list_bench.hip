// The grid SHA-1 over a list of chunks (zc_sha1_list_kernel, the classes-first
// schedule) against the plain grid kernel, on 8 GiB: the list in chunk order,
// in 64-chunk runs of shuffled order (as the class leads append it), and with
// the tail branch unused.  Tooling only.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include sha_list_bench.hip -o sha_list_bench
#include "../../zbackup_amd/csrc/zc_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

using namespace zc;
#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);          \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
  const uint32_t W = 65536;
  const uint32_t k = (uint32_t)(n / W);
  uint8_t* d;
  CK(hipMalloc(&d, n));
  CK(launch_fill_splitmix64(d, n, 2024, 0));
  uint8_t *o1, *o2;
  uint32_t *l_ord, *l_shuf;
  unsigned long long* cnt;
  CK(hipMalloc(&o1, (size_t)k * 20));
  CK(hipMalloc(&o2, (size_t)k * 20));
  CK(hipMalloc(&l_ord, (size_t)k * 4));
  CK(hipMalloc(&l_shuf, (size_t)k * 4));
  CK(hipMalloc(&cnt, 8));
  std::vector<uint32_t> ord(k), shuf(k);
  std::iota(ord.begin(), ord.end(), 0u);
  std::vector<uint32_t> runs(k / 64);
  std::iota(runs.begin(), runs.end(), 0u);
  std::shuffle(runs.begin(), runs.end(), std::mt19937(7));
  for (uint32_t r = 0; r < k / 64; ++r)
    for (uint32_t j = 0; j < 64; ++j) shuf[r * 64 + j] = runs[r] * 64 + j;
  CK(hipMemcpy(l_ord, ord.data(), (size_t)k * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(l_shuf, shuf.data(), (size_t)k * 4, hipMemcpyHostToDevice));
  const unsigned long long kk = k;
  CK(hipMemcpy(cnt, &kk, 8, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct Arm {
    const char* name;
    int kind;
    std::vector<float> t;
  } arms[] = {{"grid16 kernel", 0, {}}, {"list, chunk order", 1, {}}, {"list, shuffled 64-runs", 2, {}}};
  for (int round = 0; round < 7; ++round)
    for (auto& v : arms) {
      CK(hipEventRecord(a, 0));
      if (v.kind == 0)
        CK(launch_sha1_grid(d, n, W, k, o1, 0));
      else
        CK(launch_sha1_list(d, n, W, v.kind == 1 ? l_ord : l_shuf, cnt, 0, k, 0, 0, o2, 0));
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (round) v.t.push_back(ms);
    }
  for (auto& v : arms) {
    std::sort(v.t.begin(), v.t.end());
    printf("%-28s median %7.3f ms  min %7.3f ms\n", v.name, v.t[v.t.size() / 2], v.t[0]);
  }
  std::vector<uint8_t> h1((size_t)k * 20), h2((size_t)k * 20);
  CK(hipMemcpy(h1.data(), o1, h1.size(), hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2.data(), o2, h2.size(), hipMemcpyDeviceToHost));
  printf("list digests %s the grid kernel's\n", memcmp(h1.data(), h2.data(), h1.size()) ? "DIFFER from" : "equal");
  return 0;
}
