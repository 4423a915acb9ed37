// TEST INFRASTRUCTURE (see nocopy.hh): Config's storable chunk.max_size and
// the GET_STORABLE macro (config.hh:18-19)
#pragma once
#include <stdint.h>
#define GET_STORABLE(storage, property) storable->storage().property()
struct ChunkConfig {
  uint32_t max_size_;
  uint32_t max_size() const { return max_size_; }
};
struct StorableConfig {
  ChunkConfig chunk_;
  const ChunkConfig& chunk() const { return chunk_; }
};
class Config {
 public:
  StorableConfig* storable;
};
