// zc_sha1_grid_kernel alone: 8 GiB as W-byte grid chunks, for several W
// (threads = chunks, so W sets the parallelism).  Tooling only.
// Build: hipcc -O3 --offload-arch=gfx950 -I../../zbackup_amd/csrc sha_bench.hip
#include "../../zbackup_amd/csrc/zc_kernels.hip"

#include <cstdio>
#include <vector>
#include <algorithm>

using namespace zc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
  uint8_t* d; CK(hipMalloc(&d, n));
  CK(launch_fill_splitmix64(d, n, 2024, 0));
  uint8_t* out; CK(hipMalloc(&out, (n / 1024 + 1) * 20));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (uint32_t W : {65536u, 32768u, 16384u, 4096u}) {
    const uint32_t nr = (uint32_t)((n + W - 1) / W);
    std::vector<float> t;
    for (int r = 0; r < 6; ++r) {
      CK(hipEventRecord(a));
      CK(launch_sha1_grid(d, n, W, nr, out, 0));
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (r) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("W %6u chunks %8u  median %7.3f ms  min %7.3f ms  %7.1f GB/s\n", W, nr, t[t.size() / 2], t[0],
           n / (t[0] * 1e6));
  }
  return 0;
}
