// TEST INFRASTRUCTURE (see nocopy.hh): IndexProcessor (chunk_index.hh:47-55)
// and a ChunkIndex whose loadIndex replays the ids it was given
#pragma once
#include <utility>
#include <vector>
#include "chunk_id.hh"
#include "nocopy.hh"
#include "zbackup.pb.h"
namespace Bundle {
struct Id {
  char blob[24];
};
}  // namespace Bundle
class IndexProcessor {
 public:
  virtual ~IndexProcessor() {}
  virtual void startIndex(string const&) = 0;
  virtual void startBundle(Bundle::Id const&) = 0;
  virtual void processChunk(ChunkId const&, uint32_t) = 0;
  virtual void finishBundle(Bundle::Id const&, BundleInfo const&) = 0;
  virtual void finishIndex(string const&) = 0;
};
class ChunkIndex : NoCopy {
 public:
  std::vector<std::pair<ChunkId, uint32_t> > ids;
  void loadIndex(IndexProcessor& ip) {
    ip.startIndex("index");
    for (size_t i = 0; i < ids.size(); ++i) ip.processChunk(ids[i].first, ids[i].second);
    ip.finishIndex("index");
  }
};
