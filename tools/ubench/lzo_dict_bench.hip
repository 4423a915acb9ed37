// Dictionary placements for the lzo1x_1 block parse.
// Tooling only: times zc_lzo_parse on compressible text with its 2^14-entry
// dictionary (a) as shipped: u32 entries tagged with the call's generation in
// HBM, one per block, every block in flight; (b) u16 entries in LDS (32 KiB per
// block: one parsing lane per 64-thread workgroup, 5 workgroups per CU);
// (c) u16 entries in HBM, one per block, cleared by the wave at the start;
// (d) u32 tagged entries in HBM, one per LANE of a capped persistent grid (the
// lanes walk the blocks, a new tag per block), so the live dictionaries fit
// the MALL (4096 lanes: 256 MiB) or an XCD's L2 share (512 lanes: 32 MiB).
// Every variant's per-block result and staged encoding is compared with (a)'s
// (parse_block is the same code; only the Dict differs), then the variants are
// timed in interleaved rounds (medians).
//
//   hipcc -O3 --offload-arch=gfx950 -o lzo_dict_bench lzo_dict_bench.hip
//   ./lzo_dict_bench <payload file> [GiB]   (the file is tiled to GiB)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define ZC_HD __host__ __device__
#include "../../zbackup_amd/csrc/zc_lzo_core.h"

using zclzo::BlkOut;
using zclzo::kDictSize;
using zclzo::kStageCap;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("HIP %s at line %d\n", hipGetErrorString(e_), __LINE__);           \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

struct BlkDesc {
  uint64_t start;
  uint32_t ll;
  uint32_t first;
};

struct TagDict {
  uint32_t* d;
  uint32_t tag;
  __device__ uint32_t exchange(uint32_t i, uint32_t pos) {
    const uint32_t o = d[i];
    d[i] = tag | pos;
    return (o & 0xffff0000u) == tag ? (o & 0xffffu) : 0u;
  }
};
struct Dict16 {  // LDS or HBM, cleared before the block
  uint16_t* d;
  __device__ uint32_t exchange(uint32_t i, uint32_t pos) {
    const uint32_t o = d[i];
    d[i] = (uint16_t)pos;
    return o;
  }
};

// (a) shipped
__global__ __launch_bounds__(64) void k_tag32(const uint8_t* __restrict__ pay, const BlkDesc* __restrict__ blks,
                                              uint32_t nblk, uint32_t* __restrict__ dict, uint32_t tag,
                                              uint8_t* __restrict__ stage, BlkOut* __restrict__ out) {
  const uint32_t b = blockIdx.x * 64 + threadIdx.x;
  if (b >= nblk) return;
  const BlkDesc d = blks[b];
  TagDict td{dict + (size_t)b * kDictSize, tag << 16};
  out[b] = zclzo::parse_block(pay + d.start, d.ll, d.first ? 0u : 4u, td, stage + (size_t)b * kStageCap);
}

// (b) LDS: one parsing lane per workgroup; the wave clears the 32 KiB first
__global__ __launch_bounds__(64) void k_lds16(const uint8_t* __restrict__ pay, const BlkDesc* __restrict__ blks,
                                              uint32_t nblk, uint8_t* __restrict__ stage,
                                              BlkOut* __restrict__ out) {
  extern __shared__ uint4 lds[];
  const uint32_t b = blockIdx.x;
  for (uint32_t i = threadIdx.x; i < kDictSize * 2 / 16; i += 64) lds[i] = uint4{0, 0, 0, 0};
  __syncthreads();
  if (threadIdx.x != 0 || b >= nblk) return;
  const BlkDesc d = blks[b];
  Dict16 dd{reinterpret_cast<uint16_t*>(lds)};
  out[b] = zclzo::parse_block(pay + d.start, d.ll, d.first ? 0u : 4u, dd, stage + (size_t)b * kStageCap);
}

// (c) u16 in HBM, one per block; the wave clears its 64 dictionaries (2 MiB,
// contiguous) with coalesced 16-byte stores first
__global__ __launch_bounds__(64) void k_hbm16(const uint8_t* __restrict__ pay, const BlkDesc* __restrict__ blks,
                                              uint32_t nblk, uint16_t* __restrict__ dict,
                                              uint8_t* __restrict__ stage, BlkOut* __restrict__ out) {
  uint4* base = reinterpret_cast<uint4*>(dict + (size_t)blockIdx.x * 64 * kDictSize);
  for (uint32_t i = threadIdx.x; i < 64 * kDictSize * 2 / 16; i += 64) base[i] = uint4{0, 0, 0, 0};
  __syncthreads();
  const uint32_t b = blockIdx.x * 64 + threadIdx.x;
  if (b >= nblk) return;
  const BlkDesc d = blks[b];
  Dict16 dd{dict + (size_t)b * kDictSize};
  out[b] = zclzo::parse_block(pay + d.start, d.ll, d.first ? 0u : 4u, dd, stage + (size_t)b * kStageCap);
}

// (d) capped persistent grid: lane t parses blocks t, t + L, t + 2L, ... with
// its own tagged dictionary (tag = iteration + 1)
__global__ __launch_bounds__(64) void k_capped(const uint8_t* __restrict__ pay, const BlkDesc* __restrict__ blks,
                                               uint32_t nblk, uint32_t lanes, uint32_t* __restrict__ dict,
                                               uint8_t* __restrict__ stage, BlkOut* __restrict__ out) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  if (t >= lanes) return;
  uint32_t it = 0;
  for (uint32_t b = t; b < nblk; b += lanes, ++it) {
    const BlkDesc d = blks[b];
    TagDict td{dict + (size_t)t * kDictSize, (it + 1) << 16};
    out[b] = zclzo::parse_block(pay + d.start, d.ll, d.first ? 0u : 4u, td, stage + (size_t)b * kStageCap);
  }
}

int main(int argc, char** argv) {
  if (argc < 2) {
    printf("usage: %s payload_file [GiB]\n", argv[0]);
    return 2;
  }
  const double gib = argc > 2 ? atof(argv[2]) : 4.0;
  FILE* f = fopen(argv[1], "rb");
  if (!f) {
    printf("cannot open %s\n", argv[1]);
    return 2;
  }
  std::vector<uint8_t> base;
  {
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) base.insert(base.end(), buf, buf + k);
    fclose(f);
  }
  const uint64_t B = 0x200000;  // bundle.max_payload_size
  const uint64_t n = (uint64_t)(gib * (1ull << 30)) / B * B;
  uint8_t* pay;
  CK(hipMalloc(&pay, n));
  for (uint64_t o = 0; o < n; o += base.size())
    CK(hipMemcpy(pay + o, base.data(), std::min<uint64_t>(base.size(), n - o), hipMemcpyHostToDevice));
  // blocks of every 2 MiB bundle (lzo1x_1_compress's 49152-byte split)
  std::vector<BlkDesc> hb;
  for (uint64_t p = 0; p < n; p += B)
    for (uint64_t s = 0; s < B; s += zclzo::kBlock) hb.push_back({p + s, (uint32_t)std::min<uint64_t>(zclzo::kBlock, B - s), s == 0});
  const uint32_t nblk = (uint32_t)hb.size();
  BlkDesc* blks;
  CK(hipMalloc(&blks, nblk * sizeof(BlkDesc)));
  CK(hipMemcpy(blks, hb.data(), nblk * sizeof(BlkDesc), hipMemcpyHostToDevice));
  uint8_t* stage;
  CK(hipMalloc(&stage, (size_t)nblk * kStageCap));
  BlkOut *out0, *out1;
  CK(hipMalloc(&out0, nblk * sizeof(BlkOut)));
  CK(hipMalloc(&out1, nblk * sizeof(BlkOut)));
  const uint32_t caps[] = {4096, 2048, 1024, 512};
  size_t dict_bytes = std::max<size_t>((size_t)nblk * kDictSize * 4, (size_t)(nblk + 63) / 64 * 64 * kDictSize * 2);
  void* dict;
  CK(hipMalloc(&dict, dict_bytes));
  CK(hipMemset(dict, 0, dict_bytes));
  uint32_t tag = 0;
  const uint32_t g64 = (nblk + 63) / 64;

  struct V {
    std::string name;
    int kind;
    uint32_t cap;
    std::vector<float> t;
  };
  std::vector<V> vs = {{"a: u32 tagged HBM, all blocks", 0, 0, {}},
                       {"b: u16 LDS, 5 blocks per CU", 1, 0, {}},
                       {"c: u16 HBM cleared, all blocks", 2, 0, {}}};
  for (uint32_t c : caps) vs.push_back({"d: u32 tagged HBM, " + std::to_string(c) + " lanes", 3, c, {}});

  auto launch = [&](const V& v, BlkOut* out) {
    switch (v.kind) {
      case 0:
        ++tag;
        hipLaunchKernelGGL(k_tag32, dim3(g64), dim3(64), 0, 0, pay, blks, nblk, (uint32_t*)dict, tag, stage, out);
        break;
      case 1:
        hipLaunchKernelGGL(k_lds16, dim3(nblk), dim3(64), kDictSize * 2, 0, pay, blks, nblk, stage, out);
        break;
      case 2:
        hipLaunchKernelGGL(k_hbm16, dim3(g64), dim3(64), 0, 0, pay, blks, nblk, (uint16_t*)dict, stage, out);
        break;
      case 3:  // (prep cleared the lanes' dictionaries: the tags restart per call)
        hipLaunchKernelGGL(k_capped, dim3((v.cap + 63) / 64), dim3(64), 0, 0, pay, blks, nblk, v.cap,
                           (uint32_t*)dict, stage, out);
        break;
    }
    CK(hipGetLastError());
  };
  // before the start event: the other variants overwrite the shared buffer,
  // so the shipped variant's tags restart from a cleared buffer after them
  bool dirty = true;
  auto prep = [&](const V& v) {
    if (v.kind == 0) {
      if (dirty || tag >= 0xFFFE) {
        CK(hipMemset(dict, 0, dict_bytes));
        tag = 0;
        dirty = false;
      }
    } else {
      if (v.kind == 3) CK(hipMemset(dict, 0, (size_t)v.cap * kDictSize * 4));
      dirty = true;
    }
  };

  // parity: every variant's block results and staged bytes equal (a)'s
  std::vector<BlkOut> h0(nblk), h1(nblk);
  std::vector<uint8_t> s0((size_t)nblk * kStageCap), s1;
  prep(vs[0]);
  launch(vs[0], out0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h0.data(), out0, nblk * sizeof(BlkOut), hipMemcpyDeviceToHost));
  CK(hipMemcpy(s0.data(), stage, s0.size(), hipMemcpyDeviceToHost));
  uint64_t toks = 0, staged = 0;
  for (auto& o : h0) toks += o.ntok, staged += o.staged;
  printf("payload %.2f GiB, %u blocks, %.1f matches per block, %.3f staged bytes per input byte\n",
         n / 1073741824.0, nblk, (double)toks / nblk, (double)staged / n);
  bool all_ok = true;
  for (size_t i = 1; i < vs.size(); ++i) {
    CK(hipMemset(stage, 0xEE, (size_t)nblk * kStageCap));
    prep(vs[i]);
    launch(vs[i], out1);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h1.data(), out1, nblk * sizeof(BlkOut), hipMemcpyDeviceToHost));
    s1.resize(s0.size());
    CK(hipMemcpy(s1.data(), stage, s1.size(), hipMemcpyDeviceToHost));
    bool ok = true;
    for (uint32_t b = 0; b < nblk && ok; ++b) {
      ok = memcmp(&h0[b], &h1[b], sizeof(BlkOut)) == 0 &&
           memcmp(&s0[(size_t)b * kStageCap], &s1[(size_t)b * kStageCap], h0[b].staged) == 0;
      if (!ok) printf("  %s: block %u differs\n", vs[i].name.c_str(), b);
    }
    printf("parity %-34s %s\n", vs[i].name.c_str(), ok ? "identical" : "DIFFERS");
    all_ok &= ok;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int rounds = argc > 3 ? atoi(argv[3]) : 5;
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      prep(v);
      CK(hipEventRecord(e0));
      launch(v, out1);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms);
      printf("  round %d %-34s %9.2f ms\n", r, v.name.c_str(), ms);
      fflush(stdout);
    }
  for (auto& v : vs) {
    std::sort(v.t.begin(), v.t.end());
    printf("%-34s median %9.2f ms  min %9.2f ms  %7.2f GiB/s\n", v.name.c_str(), v.t[v.t.size() / 2], v.t[0],
           n / 1073741824.0 / (v.t[v.t.size() / 2] * 1e-3));
  }
  return all_ok ? 0 : 1;
}
