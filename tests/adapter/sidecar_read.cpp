// TEST INFRASTRUCTURE: GpuChunkMetaSidecar::readDir of integration/
// gpu_backup_creator.hh on the CPU (no context, no GPU): prints the number of
// entries read from a chunk-metadata directory and, per entry, its rolling
// hash and anchor, so tests/test_adapter.py can check the file format, the
// checksum and the skipping of damaged or foreign files.
//
//   sidecar_read dir
#include <stdio.h>

#include "gpu_backup_creator.hh"

int main(int argc, char** argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s dir\n", argv[0]);
    return 2;
  }
  std::vector<zc_chunk_meta> meta;
  GpuChunkMetaSidecar::readDir(argv[1], meta);
  printf("%zu\n", meta.size());
  for (size_t i = 0; i < meta.size(); ++i)
    printf("%016llx %u\n", (unsigned long long)meta[i].rolling, meta[i].anchor);
  return 0;
}
