// TEST INFRASTRUCTURE (see nocopy.hh): ChunkId and its blob (chunk_id.cc:19-27)
#pragma once
#include <stdint.h>
#include <string.h>
#include <string>
using std::string;
struct ChunkId {
  typedef char CryptoHashPart[16];
  CryptoHashPart cryptoHash;
  uint64_t rollingHash;
  string toBlob() const {
    char b[24];
    memcpy(b, cryptoHash, 16);
    for (int i = 0; i < 8; ++i) b[16 + i] = (char)(rollingHash >> (8 * i));
    return string(b, 24);
  }
};
