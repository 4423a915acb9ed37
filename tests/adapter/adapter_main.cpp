// TEST INFRASTRUCTURE: ZBackup::backupFromFileHandle's loops (zutils.cc:89-182)
// driving integration/gpu_backup_creator.hh -- the read loop into
// getInputBuffer / handleMoreData, finish, then the iterative shrink passes on
// the same index -- over the stand-in types of tests/adapter/mock.
//
//   adapter_main W input seeds.bin|- out_prefix [meta_dir]
//     seeds.bin: zc_seed records (the repository's index before the backup)
//     meta_dir: the repository's chunk-metadata directory (GpuChunkMetaSidecar):
//       read when the index is seeded, a file for this backup written at its end
//     writes out_prefix.data (the final backup data), out_prefix.meta
//     ("iterations adds hist_seeded by_value"), out_prefix.adds (24-byte ids of
//     Writer::add calls)
#include <stdio.h>
#include <stdlib.h>

#include <string>

#include "gpu_backup_creator.hh"

int main(int argc, char** argv) {
  if (argc != 5 && argc != 6) {
    fprintf(stderr, "usage: %s W input seeds.bin|- out_prefix [meta_dir]\n", argv[0]);
    return 2;
  }
  const std::string metaDir = argc == 6 ? argv[5] : "";
  StorableConfig st;
  st.chunk_.max_size_ = (uint32_t)strtoul(argv[1], 0, 10);
  Config config;
  config.storable = &st;
  ChunkIndex chunkIndex;
  if (std::string(argv[3]) != "-") {
    FILE* sf = fopen(argv[3], "rb");
    if (!sf) return 3;
    zc_seed s;
    while (fread(&s, sizeof s, 1, sf) == 1) {
      ChunkId id;
      memcpy(id.cryptoHash, s.sha1, 16);
      id.rollingHash = s.rolling;
      chunkIndex.ids.push_back(std::make_pair(id, s.size));
    }
    fclose(sf);
  }
  ChunkStorage::Writer chunkStorageWriter;
  try {
    GpuChunkIndex gpuIndex(config, chunkIndex, 0, ZC_FLAG_SHA1, metaDir);
    zc_stats seeded;
    zcCheck(zc_get_stats(gpuIndex.context(), &seeded), gpuIndex.context(), "zc_get_stats");
    FILE* in = fopen(argv[2], "rb");
    if (!in) return 3;
    GpuBackupCreator backupCreator(gpuIndex, chunkStorageWriter);
    for (;;) {
      size_t toRead = backupCreator.getInputBufferSize();
      void* inputBuffer = backupCreator.getInputBuffer();
      size_t rd = fread(inputBuffer, 1, toRead, in);
      if (!rd) break;
      backupCreator.handleMoreData(rd);
    }
    fclose(in);
    backupCreator.finish();
    std::string serialized;
    backupCreator.getBackupData(serialized);
    unsigned iterations = 0;
    for (;;) {
      GpuBackupCreator shrink(gpuIndex, chunkStorageWriter);
      const char* ptr = serialized.data();
      size_t left = serialized.size();
      while (left) {
        size_t bufferSize = shrink.getInputBufferSize();
        size_t toCopy = bufferSize > left ? left : bufferSize;
        memcpy(shrink.getInputBuffer(), ptr, toCopy);
        shrink.handleMoreData(toCopy);
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
    // Writer::commit (zutils.cc:175) would move the bundles and the index file
    // into place here; the chunk metadata of this backup follows it
    if (!metaDir.empty()) gpuIndex.saveChunkMeta(metaDir);
    const std::string p(argv[4]);
    FILE* f = fopen((p + ".data").c_str(), "wb");
    fwrite(serialized.data(), 1, serialized.size(), f);
    fclose(f);
    f = fopen((p + ".adds").c_str(), "wb");
    for (size_t i = 0; i < chunkStorageWriter.ids.size(); ++i) fwrite(chunkStorageWriter.ids[i].data(), 1, 24, f);
    fclose(f);
    f = fopen((p + ".meta").c_str(), "w");
    fprintf(f, "%u %zu %llu %llu\n", iterations, chunkStorageWriter.ids.size(),
            (unsigned long long)seeded.hist_seeded, (unsigned long long)seeded.by_value);
    fclose(f);
  } catch (const std::exception& e) {
    fprintf(stderr, "adapter_main: %s\n", e.what());
    return 1;
  }
  return 0;
}
