// BENCH TOOLING (tools/feedbench): a ChunkStorage::Writer whose add() does what
// the reference's does with the bytes -- Bundle::Creator::addChunk appends them
// to the current bundle's payload, a new bundle once payload + size exceeds
// bundle.max_payload_size (chunk_storage.cc:31-46, bundle.cc:30-36,
// zbackup.proto:88) -- and times itself.  Finished payloads are dropped (the
// compressor threads are not part of the feed loop).
#pragma once
#include <chrono>
#include <string>
#include "chunk_id.hh"
#include "nocopy.hh"
namespace ChunkStorage {
class Writer : NoCopy {
 public:
  std::string payload;
  size_t maxPayload = 0x200000, chunks = 0, bundles = 0, bytes = 0;
  double seconds = 0;
  bool add(ChunkId const& id, void const* data, size_t size) {
    auto t0 = std::chrono::steady_clock::now();
    (void)id;
    if (payload.size() + size > maxPayload) {
      payload.clear();
      ++bundles;
    }
    payload.append((const char*)data, size);
    ++chunks;
    bytes += size;
    seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return true;
  }
};
}  // namespace ChunkStorage
