// zc_lzo.hip -- bundle writer offload: Bundle::Creator::addChunk's payload
// assembly (bundle.cc:30-36) and the lzo1x_1 compression of
// Bundle::Creator::write (bundle.cc:120-151 -> LZO1X_1_Encoder::doProcessNoSize,
// compression.cc:586-606, i.e. liblzo2 2.10's lzo1x_1_compress) with zbackup's
// framing, on the GPU, byte-identical to the library's output.
//
// Work split (zc_lzo_core.h explains why the blocks are independent):
//   zc_lzo_parse_kernel  one lane per 48 KiB block: the greedy parse over a
//                        2^14-entry dictionary of its own (u32 entries tagged
//                        with the call's generation in HBM, so no per-block
//                        memset), staging the block's encoding from its first
//                        match on;
//   zc_lzo_chain_kernel  one lane per bundle: walks its blocks in order, writes
//                        the frame, first-literal-run headers, final run and
//                        end marker, and lists the byte copies;
//   zc_lzo_copy_kernel   one wave per copy (literal runs from the payload,
//                        staged encodings), 16-byte stores aligned on the
//                        destination;
//   zc_lzo_or_kernel     a final run of 1-3 literals or-ed into the last match.
// The same copy kernel gathers chunk extents into bundle payloads.
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <algorithm>
#include <vector>

#define ZC_HD __host__ __device__
#include "zc_device.h"
#include "zc_lzo_core.h"

namespace zc {

using zclzo::BlkOut;
using zclzo::kDictSize;
using zclzo::kStageCap;

namespace {

struct BlkDesc {
  uint64_t start;  // offset in the payload buffer
  uint32_t ll;
  uint32_t first;  // a payload's first block (inherits no literals)
};
struct BundleDesc {
  uint64_t pay_off, pay_size, out_off;
  uint32_t blk0;
  uint64_t copy0;
};
struct Copy {
  const uint8_t* src;
  uint8_t* dst;
  uint64_t n;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct TagDict {
  uint32_t* d;
  uint32_t tag;  // generation << 16
  __device__ uint32_t exchange(uint32_t i, uint32_t pos) {
    const uint32_t o = d[i];
    d[i] = tag | pos;
    return (o & 0xffff0000u) == tag ? (o & 0xffffu) : 0u;
  }
};

__global__ __launch_bounds__(64) void zc_lzo_parse_kernel(const uint8_t* __restrict__ payload,
                                                          const BlkDesc* __restrict__ blks, uint32_t nblk,
                                                          uint32_t* __restrict__ dict, uint32_t tag,
                                                          uint8_t* __restrict__ stage, BlkOut* __restrict__ out) {
  const uint32_t b = blockIdx.x * 64 + threadIdx.x;
  if (b >= nblk) return;
  const BlkDesc d = blks[b];
  TagDict td{dict + (size_t)b * kDictSize, tag << 16};
  out[b] = zclzo::parse_block(payload + d.start, d.ll, d.first ? 0u : 4u, td, stage + (size_t)b * kStageCap);
}

__global__ __launch_bounds__(64) void zc_lzo_chain_kernel(const uint8_t* __restrict__ payload,
                                                          const BundleDesc* __restrict__ bund, uint32_t nb,
                                                          const BlkOut* __restrict__ bo,
                                                          const uint8_t* __restrict__ stage, uint8_t* __restrict__ out,
                                                          Copy* __restrict__ copies, uint64_t* __restrict__ out_size,
                                                          uint64_t* __restrict__ or_at, uint32_t* __restrict__ or_val) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= nb) return;
  const BundleDesc d = bund[i];
  uint8_t* o = out + d.out_off;
  Copy* c = copies + d.copy0;
  uint64_t nc = 0;
  // pieces of at most 64 KiB, one wave's work each
  auto copy = [&](bool from_stage, uint64_t src, uint64_t dst, uint64_t n) {
    const uint8_t* s = from_stage ? stage + (size_t)(d.blk0 + src) * kStageCap : payload + d.pay_off + src;
    for (uint64_t k = 0; k < n; k += zclzo::kPiece)
      c[nc++] = Copy{s + k, o + dst + k, n - k < zclzo::kPiece ? n - k : zclzo::kPiece};
  };
  uint64_t oa;
  uint32_t ov;
  out_size[i] = zclzo::chain_bundle(d.pay_size, bo + d.blk0, o, copy, &oa, &ov);
  const uint64_t cap = zclzo::copies_cap(zclzo::block_count(d.pay_size), d.pay_size);
  for (uint64_t k = nc; k < cap; k++) c[k].n = 0;
  or_at[i] = d.out_off + oa;
  or_val[i] = ov;
}

// one wave per copy: a head of bytes up to the destination's 16-byte
// alignment, 16-byte aligned stores (the source read unaligned), a byte tail
__global__ __launch_bounds__(256) void zc_lzo_copy_kernel(const Copy* __restrict__ copies, uint32_t n) {
  const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  if (w >= n) return;
  const Copy c = copies[w];
  if (!c.n) return;
  uint64_t len = c.n;
  const uint8_t* src = c.src;
  uint8_t* dst = c.dst;
  uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15);
  if (head > len) head = (uint32_t)len;
  if (lane < head) dst[lane] = src[lane];
  src += head;
  dst += head;
  len -= head;
  const uint64_t nv = len >> 4;
  uint64_t v = lane;
  // four 16-byte loads in flight per lane before their stores
  for (; v + 3 * 64 < nv; v += 4 * 64) {
    u32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_memcpy(&x[u], src + (v + u * 64) * 16, 16);
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(x[u], reinterpret_cast<u32x4*>(dst + (v + u * 64) * 16));
  }
  for (; v < nv; v += 64) {
    u32x4 x;
    __builtin_memcpy(&x, src + v * 16, 16);
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(dst + v * 16));
  }
  const uint32_t t = (uint32_t)(len & 15);
  if (lane < t) dst[nv * 16 + lane] = src[nv * 16 + lane];
}

__global__ void zc_lzo_or_kernel(uint8_t* out, const uint64_t* or_at, const uint32_t* or_val, uint32_t nb) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb && or_val[i]) out[or_at[i]] |= (uint8_t)or_val[i];
}

// Adler-32 (zlib's, as Adler32 wraps it: adler32.hh:13-33) of one range per
// 256-thread block, from the initial value 1: a = 1 + sum b_i, b = n + sum
// (n - i) b_i (mod 65521) = n + n * S1 - sum i b_i.  Thread t takes the
// 16-byte slots t, t + 256, ... of the 16-byte grid over the range (bytes
// outside it masked), accumulating S1 and sum (i mod 65521) b_i exactly in 64
// bits; the block sums them and reduces once.
constexpr uint32_t kAdlerMod = 65521;
__global__ __launch_bounds__(256) void zc_adler32_kernel(const uint8_t* __restrict__ base,
                                                         const uint64_t* __restrict__ off,
                                                         const uint64_t* __restrict__ len, uint32_t* __restrict__ out) {
  __shared__ uint64_t red[2][256];
  const uint64_t n = len[blockIdx.x];
  const uint64_t a0 = (uint64_t)(uintptr_t)(base + off[blockIdx.x]);  // absolute address
  const uint64_t g0 = a0 & ~15ull;                   // its 16-byte slot: never crosses a page
  const uint64_t nslot = (a0 + n + 15 - g0) >> 4;     // slots touching the range
  uint64_t s1 = 0, si = 0;
  for (uint64_t k = threadIdx.x; k < nslot && n; k += 256) {
    const uint64_t q = g0 + 16 * k;                   // the slot's address
    u32x4 v = *reinterpret_cast<const u32x4*>((uintptr_t)q);
    const uint32_t w[4] = {v[0], v[1], v[2], v[3]};
    // position of the slot's byte 0 in the range (may be "negative" for the
    // head slot: those bytes are masked); congruent mod 65521 is enough
    const int64_t p0 = (int64_t)q - (int64_t)a0;
    const bool full = p0 >= 0 && (uint64_t)p0 + 16 <= n;
    uint32_t bs = 0, bk = 0;  // sum of bytes, sum of j * byte (j = byte index in the slot)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t x = w[d];
      if (!full) {
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t p = p0 + 4 * d + j;
          if (p >= 0 && (uint64_t)p < n) m |= 0xFFu << (8 * j);
        }
        x &= m;
      }
      bs = __builtin_amdgcn_udot4(x, 0x01010101u, bs, false);
      bk = __builtin_amdgcn_udot4(x, (uint32_t)((4 * d) | (4 * d + 1) << 8 | (4 * d + 2) << 16 | (4 * d + 3) << 24),
                                  bk, false);
    }
    const uint64_t pm = (uint64_t)((p0 % (int64_t)kAdlerMod + kAdlerMod) % kAdlerMod);
    s1 += bs;
    si += pm * bs + bk;
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = si;
  __syncthreads();
  for (uint32_t h = 128; h; h >>= 1) {
    if (threadIdx.x < h) {
      red[0][threadIdx.x] += red[0][threadIdx.x + h];
      red[1][threadIdx.x] += red[1][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const uint64_t S1 = red[0][0] % kAdlerMod, SI = red[1][0] % kAdlerMod, nm = n % kAdlerMod;
    const uint32_t a = (uint32_t)((1 + S1) % kAdlerMod);
    const uint32_t b = (uint32_t)((nm + nm * S1 % kAdlerMod + kAdlerMod - SI) % kAdlerMod);
    out[blockIdx.x] = b << 16 | a;
  }
}

template <class T>
struct Buf {
  T* p = nullptr;
  size_t cap = 0;
  // grow to n elements; *fresh (if given) reports a new allocation
  hipError_t ensure(size_t n, bool* fresh = nullptr) {
    if (fresh) *fresh = false;
    if (n <= cap && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    cap = n;
    if (fresh) *fresh = true;
    return hipSuccess;
  }
  ~Buf() {
    if (p) (void)hipFree(p);
  }
};

#define LCK(x)                            \
  do {                                    \
    hipError_t e_ = (x);                  \
    if (e_ != hipSuccess) return e_;      \
  } while (0)

// at most this many blocks per device batch (12 GiB of payload; the
// dictionaries take 64 KiB and the staging 51 KiB per block); the environment
// variable ZC_LZO_BATCH_BLOCKS lowers it (tests: a call split into batches)
constexpr uint32_t kMaxBatchBlocks = 1u << 18;
uint32_t max_batch_blocks() {
  const char* e = getenv("ZC_LZO_BATCH_BLOCKS");
  const unsigned long v = e ? strtoul(e, nullptr, 10) : 0;
  return v >= 1 && v < kMaxBatchBlocks ? (uint32_t)v : kMaxBatchBlocks;
}

}  // namespace

struct LzoScratch {
  Buf<uint32_t> dict;
  Buf<uint64_t> ad_off, ad_len;
  Buf<uint32_t> ad_out;
  Buf<uint8_t> stage;
  Buf<BlkOut> bo;
  Buf<BlkDesc> blks;
  Buf<BundleDesc> bund;
  Buf<Copy> copies;
  Buf<uint64_t> out_size, or_at;
  Buf<uint32_t> or_val;
  uint32_t gen = 0;  // tag of the dictionaries' live entries
  hipEvent_t e0 = nullptr, e1 = nullptr;
  LzoTimes times{};
};

LzoScratch* lzo_scratch_new() { return new LzoScratch(); }
void lzo_scratch_free(LzoScratch* s) {
  if (!s) return;
  if (s->e0) (void)hipEventDestroy(s->e0);
  if (s->e1) (void)hipEventDestroy(s->e1);
  delete s;
}
const LzoTimes* lzo_times(const LzoScratch* s) { return &s->times; }

hipError_t lzo_copy_list(LzoScratch* s, const std::vector<Copy>& list, hipStream_t st) {
  if (list.empty()) return hipSuccess;
  LCK(s->copies.ensure(list.size()));
  LCK(hipMemcpyAsync(s->copies.p, list.data(), list.size() * sizeof(Copy), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(zc_lzo_copy_kernel, dim3((uint32_t)((list.size() + 3) / 4)), dim3(256), 0, st, s->copies.p,
                     (uint32_t)list.size());
  LCK(hipGetLastError());
  return hipStreamSynchronize(st);  // the list's host memory is reused
}

hipError_t lzo_gather(LzoScratch* s, const uint8_t* d_src, const uint64_t* off, const uint64_t* size, size_t n,
                      uint8_t* d_dst, hipStream_t st) {
  // pieces of at most 64 KiB, so one long extent is not one wave's work
  constexpr uint64_t kPiece = zclzo::kPiece;
  std::vector<Copy> list;
  uint64_t pos = 0;
  for (size_t i = 0; i < n; i++) {
    for (uint64_t k = 0; k < size[i]; k += kPiece)
      list.push_back(Copy{d_src + off[i] + k, d_dst + pos + k, std::min(kPiece, size[i] - k)});
    pos += size[i];
  }
  return lzo_copy_list(s, list, st);
}

hipError_t lzo_adler32(LzoScratch* s, const uint8_t* d_base, const uint64_t* off, const uint64_t* len, size_t n,
                       uint32_t* out, hipStream_t st) {
  if (!n) return hipSuccess;
  LCK(s->ad_off.ensure(n));
  LCK(s->ad_len.ensure(n));
  LCK(s->ad_out.ensure(n));
  LCK(hipMemcpyAsync(s->ad_off.p, off, n * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  LCK(hipMemcpyAsync(s->ad_len.p, len, n * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(zc_adler32_kernel, dim3((uint32_t)n), dim3(256), 0, st, d_base, s->ad_off.p, s->ad_len.p,
                     s->ad_out.p);
  LCK(hipGetLastError());
  LCK(hipMemcpyAsync(out, s->ad_out.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

static hipError_t lzo_batch(LzoScratch* s, const uint8_t* d_payload, const uint64_t* pay_off,
                            const uint64_t* pay_size, size_t b0, size_t b1, uint8_t* d_out, const uint64_t* out_off,
                            uint64_t* out_size, hipStream_t st) {
  std::vector<BlkDesc> blks;
  std::vector<BundleDesc> bund;
  uint64_t ncopy = 0;
  for (size_t i = b0; i < b1; i++) {
    const uint32_t nblk = zclzo::block_count(pay_size[i]);
    bund.push_back(BundleDesc{pay_off[i], pay_size[i], out_off[i], (uint32_t)blks.size(), ncopy});
    uint64_t pos = 0;
    for (uint32_t k = 0; k < nblk; k++) {
      const uint32_t ll = (uint32_t)std::min<uint64_t>(pay_size[i] - pos, zclzo::kBlock);
      blks.push_back(BlkDesc{pay_off[i] + pos, ll, k == 0 ? 1u : 0u});
      pos += ll;
    }
    ncopy += zclzo::copies_cap(nblk, pay_size[i]);
  }
  const uint32_t nblk = (uint32_t)blks.size(), nb = (uint32_t)bund.size();
  // dictionaries: entries of an earlier generation read as empty; zeroed
  // when (re)allocated and when the 16-bit generation wraps
  // (the clear is queued on the call's stream, ahead of the parse: the
  // context's streams are non-blocking, so a null-stream memset would not be)
  bool fresh = false;
  LCK(s->dict.ensure((size_t)nblk * kDictSize, &fresh));
  if (fresh || s->gen == 0xffff) {
    LCK(hipMemsetAsync(s->dict.p, 0, s->dict.cap * sizeof(uint32_t), st));
    s->gen = 0;
  }
  const uint32_t tag = ++s->gen;
  LCK(s->stage.ensure((size_t)nblk * kStageCap));
  LCK(s->bo.ensure(nblk));
  LCK(s->blks.ensure(nblk));
  LCK(s->bund.ensure(nb));
  LCK(s->copies.ensure(ncopy));
  LCK(s->out_size.ensure(nb));
  LCK(s->or_at.ensure(nb));
  LCK(s->or_val.ensure(nb));
  if (!s->e0) LCK(hipEventCreate(&s->e0));
  if (!s->e1) LCK(hipEventCreate(&s->e1));
  if (nblk) LCK(hipMemcpyAsync(s->blks.p, blks.data(), nblk * sizeof(BlkDesc), hipMemcpyHostToDevice, st));
  LCK(hipMemcpyAsync(s->bund.p, bund.data(), nb * sizeof(BundleDesc), hipMemcpyHostToDevice, st));
  LCK(hipEventRecord(s->e0, st));
  if (nblk)
    hipLaunchKernelGGL(zc_lzo_parse_kernel, dim3((nblk + 63) / 64), dim3(64), 0, st, d_payload, s->blks.p, nblk,
                       s->dict.p, tag, s->stage.p, s->bo.p);
  LCK(hipEventRecord(s->e1, st));
  hipLaunchKernelGGL(zc_lzo_chain_kernel, dim3((nb + 63) / 64), dim3(64), 0, st, d_payload, s->bund.p, nb, s->bo.p,
                     s->stage.p, d_out, s->copies.p, s->out_size.p, s->or_at.p, s->or_val.p);
  if (ncopy)
    hipLaunchKernelGGL(zc_lzo_copy_kernel, dim3((uint32_t)((ncopy + 3) / 4)), dim3(256), 0, st, s->copies.p,
                       (uint32_t)ncopy);
  hipLaunchKernelGGL(zc_lzo_or_kernel, dim3((nb + 255) / 256), dim3(256), 0, st, d_out, s->or_at.p, s->or_val.p, nb);
  LCK(hipGetLastError());
  LCK(hipMemcpyAsync(out_size + b0, s->out_size.p, nb * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  LCK(hipStreamSynchronize(st));
  float ms = 0;
  LCK(hipEventElapsedTime(&ms, s->e0, s->e1));
  s->times.parse_ms += ms;
  s->times.blocks += nblk;
  return hipSuccess;
}

hipError_t lzo_compress(LzoScratch* s, const uint8_t* d_payload, const uint64_t* pay_off, const uint64_t* pay_size,
                        size_t n, uint8_t* d_out, const uint64_t* out_off, uint64_t* out_size, hipStream_t st) {
  s->times = LzoTimes{};
  const uint32_t cap = max_batch_blocks();
  size_t b0 = 0;
  while (b0 < n) {
    size_t b1 = b0;
    uint64_t blk = 0;
    while (b1 < n) {
      const uint32_t k = zclzo::block_count(pay_size[b1]);
      if (b1 > b0 && blk + k > cap) break;
      blk += k;
      b1++;
    }
    LCK(lzo_batch(s, d_payload, pay_off, pay_size, b0, b1, d_out, out_off, out_size, st));
    b0 = b1;
  }
  return hipSuccess;
}

}  // namespace zc
