// TEST INFRASTRUCTURE (see nocopy.hh): a Writer that records what it is given
// (Writer::add, chunk_storage.hh:50)
#pragma once
#include <string>
#include <vector>
#include "chunk_id.hh"
#include "nocopy.hh"
namespace ChunkStorage {
class Writer : NoCopy {
 public:
  std::vector<std::string> ids;     // blobs, in call order
  std::vector<std::string> chunks;  // the bytes
  bool add(ChunkId const& id, void const* data, size_t size) {
    ids.push_back(id.toBlob());
    chunks.push_back(std::string((const char*)data, size));
    return true;
  }
};
}  // namespace ChunkStorage
