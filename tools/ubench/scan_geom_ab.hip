// A/B of scan geometries, interleaved in one process: the product zc_scan_kernel
// built with different workgroups per CU / round sizes / anchor-list sizes (scan_variant.hip,
// one object per variant, tools/ubench/make_geom_ab.sh), 8 GiB of seeded
// random bytes.  Span digests compared (identical in every variant); the
// anchor count is printed (a variant whose list is small overflows wave-tiles,
// which then store no anchors: timing only).  Tooling only.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef hipError_t (*ScanFn)(const uint8_t*, uint64_t, uint64_t, uint64_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*,
                             uint32_t, unsigned long long*);
#define DECL(N) extern "C" hipError_t N(const uint8_t*, uint64_t, uint64_t, uint64_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t, unsigned long long*);
DECL(scan_v_prod) DECL(scan_v_prio1) DECL(scan_v_prio2) DECL(scan_v_prio3)
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void fill(uint8_t* d, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    ((uint64_t*)d)[i] = z ^ (z >> 31);
  }
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
  const int rounds = argc > 2 ? atoi(argv[2]) : 25;
  // sized for the smallest geometry built (2 KiB lane spans: 128 KiB
  // wave-tiles, 128 pool entries each); each variant launches its own tiles
  const uint64_t ntiles = n / (2ull << 20), nwt = n / (128ull << 10), nblk = n / 1024;
  const uint32_t wcap = 2u * ((1u << 18) / 4096) + 64u;
  uint8_t* d; CK(hipMalloc(&d, n));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, d, n);
  struct V { const char* name; ScanFn f; uint64_t* blk; std::vector<float> t; unsigned long long pool; };
  std::vector<V> vs = {{"product (2 x 4 waves, list 144)", scan_v_prod, nullptr, {}, 0},
                       {"hand-off at priority 1", scan_v_prio1, nullptr, {}, 0},
                       {"hand-off at priority 2", scan_v_prio2, nullptr, {}, 0},
                       {"hand-off at priority 3", scan_v_prio3, nullptr, {}, 0}};
  uint32_t *dbase, *dcnt, *prel, *pg; unsigned long long* cnt;
  CK(hipMalloc(&dbase, nwt * 4)); CK(hipMalloc(&dcnt, nwt * 4));
  CK(hipMalloc(&prel, nwt * wcap * 4)); CK(hipMalloc(&pg, nwt * wcap * 4)); CK(hipMalloc(&cnt, 64));
  for (auto& v : vs) CK(hipMalloc(&v.blk, nblk * 8));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      CK(hipMemset(cnt, 0, 64));
      CK(hipEventRecord(a));
      CK(v.f(d, n, ntiles, v.blk, dbase, dcnt, prel, pg, wcap, cnt));
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (r) v.t.push_back(ms);
      CK(hipMemcpy(&v.pool, cnt, 8, hipMemcpyDeviceToHost));  // CNT_POOL is counter 0
    }
  std::vector<uint64_t> h0(nblk), h1(nblk);
  CK(hipMemcpy(h0.data(), vs[0].blk, nblk * 8, hipMemcpyDeviceToHost));
  bool same = true;
  for (auto& v : vs) {
    CK(hipMemcpy(h1.data(), v.blk, nblk * 8, hipMemcpyDeviceToHost));
    if (!strstr(v.name, "(probe)")) same = same && h0 == h1;  // a timing probe hashes the wrong bytes
    std::sort(v.t.begin(), v.t.end());
    printf("%-34s median %7.3f ms  min %7.3f ms  %7.1f GB/s (min)  pool %llu\n", v.name, v.t[v.t.size() / 2], v.t[0],
           n / (v.t[0] * 1e6), v.pool);
  }
  printf(same ? "span digests identical\n" : "SPAN DIGESTS DIFFER\n");
  return same ? 0 : 2;
}
