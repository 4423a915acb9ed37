// BENCH TOOLING: the drop-in feed path end to end, in one process --
// ZBackup::backupFromFileHandle's read loop (zutils.cc:100-127) over
// integration/gpu_backup_creator.hh: the input copied into getInputBuffer()
// (standing for fread, T copy threads), handleMoreData (the window's H2D
// copies, scan and resolution during the call), the adapter draining the
// records as they are cut (zc_take_records; a NEW chunk's bytes read with
// zc_read_stream into Writer::add, which appends them to a 2 MiB bundle
// payload; every record through Message::serialize), finish, getBackupData,
// then the iterative shrink passes (zutils.cc:137-166) on the same index.
// The backup's whole-stream SHA-256 (BackupInfo.sha256, zutils.cc:94,119,134)
// is kept too: sha256 = 1 adds every piece inline after the read, as the
// reference loop does (a serial chain: the loop can run no faster than it);
// 2 hashes piece i on a helper thread while handleMoreData(i) runs, joined
// before the next getInputBuffer (the piece's bytes are overwritten then);
// 0 leaves it out.
//
//   feed_bench W bytes seed sha1(0|1) copy_threads [sha256(0|1|2) [window_bytes]]
// prints one JSON object: seconds of the whole loop and of its parts
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "gpu_backup_creator.hh"

namespace {
using Clock = std::chrono::steady_clock;
double since(Clock::time_point t) { return std::chrono::duration<double>(Clock::now() - t).count(); }

// the engine's synthetic stream: byte k = byte k mod 8 of splitmix64 word k / 8
void fill(uint8_t* p, uint64_t n, uint64_t seed, unsigned threads) {
  std::vector<std::thread> th;
  const uint64_t nw = n / 8;
  for (unsigned t = 0; t < threads; ++t)
    th.emplace_back([=] {
      for (uint64_t i = nw * t / threads; i < nw * (t + 1) / threads; ++i) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        memcpy(p + 8 * i, &z, 8);
      }
    });
  for (auto& x : th) x.join();
  for (uint64_t k = nw * 8; k < n; ++k) p[k] = 0;
}

void copy_mt(void* dst, const void* src, size_t n, unsigned threads) {
  if (threads <= 1 || n < (4u << 20)) {
    memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < threads; ++t) {
    const size_t a = n * t / threads, b = n * (t + 1) / threads;
    th.emplace_back([=] { memcpy((char*)dst + a, (const char*)src + a, b - a); });
  }
  for (auto& x : th) x.join();
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 6 || argc > 8) {
    fprintf(stderr, "usage: %s W bytes seed sha1 copy_threads [sha256 [window_bytes]]\n", argv[0]);
    return 2;
  }
  const int sha256_mode = argc >= 7 ? atoi(argv[6]) : 0;
  const uint64_t window = argc == 8 ? strtoull(argv[7], 0, 0) : 0;  // 0: the library's default
  const uint32_t W = (uint32_t)strtoul(argv[1], 0, 10);
  const uint64_t n = strtoull(argv[2], 0, 0), seed = strtoull(argv[3], 0, 0);
  const bool sha1 = atoi(argv[4]) != 0;
  const unsigned threads = (unsigned)atoi(argv[5]);
  std::vector<uint8_t> input(n);
  fill(input.data(), n, seed, 16);
  StorableConfig st;
  st.chunk_.max_size_ = W;
  Config config;
  config.storable = &st;
  ChunkIndex chunkIndex;
  ChunkStorage::Writer writer;
  try {
    GpuChunkIndex gpuIndex(config, chunkIndex, 0, (sha1 ? ZC_FLAG_SHA1 : 0) | ZC_FLAG_TIMING);
    if (window && zc_set_window(gpuIndex.context(), window) != ZC_OK) throw std::runtime_error("zc_set_window");
    double copy_s = 0, sha256_s = 0, getbuf_s = 0, hmd_s = 0, window_setup_s = 0;
    size_t pieces = 0;
    zc_sha256* sha256 = nullptr;
    if (sha256_mode && zc_sha256_create(&sha256) != ZC_OK) throw std::runtime_error("zc_sha256_create");
    std::thread hasher;
    const auto t0 = Clock::now();
    GpuBackupCreator backupCreator(gpuIndex, writer);
    uint64_t pos = 0;
    for (;;) {
      if (hasher.joinable()) {  // the previous piece's bytes are hashed before they are overwritten
        const auto tj = Clock::now();
        hasher.join();
        sha256_s += since(tj);
      }
      const auto tg = Clock::now();
      size_t toRead = backupCreator.getInputBufferSize();
      void* inputBuffer = backupCreator.getInputBuffer();
      // the first call makes the context's feed window (pinned host mirror +
      // HBM: a per-context setup cost, reported apart); later ones slide it
      (pieces ? getbuf_s : window_setup_s) += since(tg);
      const size_t rd = (size_t)std::min<uint64_t>(toRead, n - pos);
      if (!rd) break;
      const auto tc = Clock::now();
      copy_mt(inputBuffer, input.data() + pos, rd, threads);
      copy_s += since(tc);
      pos += rd;
      ++pieces;
      if (sha256_mode == 1) {  // zutils.cc:119
        const auto th = Clock::now();
        zc_sha256_add(sha256, inputBuffer, rd);
        sha256_s += since(th);
      } else if (sha256_mode == 2) {
        hasher = std::thread([=] { zc_sha256_add(sha256, inputBuffer, rd); });
      }
      const auto thm = Clock::now();
      backupCreator.handleMoreData((unsigned)rd);
      hmd_s += since(thm);
    }
    const auto tf = Clock::now();
    backupCreator.finish();
    const double finish_s = since(tf);
    zc_stats stats;  // the backup stream's (the shrink passes are streams of their own)
    zc_get_stats(gpuIndex.context(), &stats);
    std::string sha256_hex;
    if (sha256) {
      uint8_t dg[32];
      zc_sha256_finish(sha256, dg);
      zc_sha256_destroy(sha256);
      char hx[3];
      for (uint8_t b : dg) {
        snprintf(hx, sizeof hx, "%02x", b);
        sha256_hex += hx;
      }
    }
    std::string serialized;
    backupCreator.getBackupData(serialized);
    const double loop_s = since(t0);
    const auto ts = Clock::now();
    unsigned iterations = 0;
    for (;;) {  // zutils.cc:137-166
      GpuBackupCreator shrink(gpuIndex, writer);
      const char* ptr = serialized.data();
      size_t left = serialized.size();
      while (left) {
        size_t bufferSize = shrink.getInputBufferSize();
        size_t toCopy = bufferSize > left ? left : bufferSize;
        memcpy(shrink.getInputBuffer(), ptr, toCopy);
        shrink.handleMoreData((unsigned)toCopy);
        ptr += toCopy;
        left -= toCopy;
      }
      shrink.finish();
      std::string newGen;
      shrink.getBackupData(newGen);
      if (newGen.size() < serialized.size()) {
        serialized.swap(newGen);
        ++iterations;
      } else {
        break;
      }
    }
    const double shrink_s = since(ts);
    printf("{\"bytes\": %llu, \"W\": %u, \"sha1\": %d, \"copy_threads\": %u, \"pieces\": %zu, \"loop_s\": %.6f, "
           "\"copy_s\": %.6f, \"writer_add_s\": %.6f, \"engine_and_adapter_s\": %.6f, \"shrink_s\": %.6f, "
           "\"shrink_iterations\": %u, \"writer_chunks\": %zu, \"writer_bytes\": %zu, \"bundles\": %zu, "
           "\"backup_data_bytes\": %zu, \"window_bytes\": %llu, \"sha256_mode\": %d, \"sha256_s\": %.6f, "
           "\"sha256\": \"%s\", \"window_setup_s\": %.6f, \"getbuf_s\": %.6f, \"handle_more_data_s\": %.6f, \"finish_s\": %.6f, "
           "\"segments\": %llu, \"engine_total_ms\": %.3f, \"engine_meta_ms\": %.3f, \"engine_walk_ms\": %.3f, "
           "\"engine_finalize_ms\": %.3f, \"engine_scan_ms\": %.3f}\n",
           (unsigned long long)n, W, sha1 ? 1 : 0, threads, pieces, loop_s, copy_s, writer.seconds,
           loop_s - copy_s - writer.seconds - sha256_s - window_setup_s, shrink_s, iterations, writer.chunks, writer.bytes, writer.bundles + 1,
           serialized.size(), (unsigned long long)stats.window_bytes, sha256_mode, sha256_s, sha256_hex.c_str(),
           window_setup_s, getbuf_s, hmd_s, finish_s, (unsigned long long)stats.segments, stats.total_ms, stats.meta_ms,
           stats.walk_ms, stats.finalize_ms, stats.scan_ms);
  } catch (const std::exception& e) {
    fprintf(stderr, "feed_bench: %s\n", e.what());
    return 1;
  }
  return 0;
}
