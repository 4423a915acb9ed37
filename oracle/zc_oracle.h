/* zc_oracle.h -- TEST INFRASTRUCTURE ONLY.  C ABI of the CPU restatement in
 * zc_oracle.cpp; loaded by tests/ (ctypes), __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg.  Never linked by the product library. */
#ifndef ZC_ORACLE_H
#define ZC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ZCO_CHUNK_NEW = 0, ZCO_CHUNK_DUP = 1, ZCO_BYTES = 2 };

/* One instruction of the backup stream (zbackup.proto:149-159), with the
 * stream offset/size it covers.  kind NEW = chunk_to_emit of a chunk cut and
 * saved here; DUP = chunk_to_emit of a window matched in the index; BYTES =
 * bytes_to_emit (fragments under 128 bytes, backup_creator.cc:114-121). */
typedef struct {
  uint64_t offset;
  uint32_t size;
  uint32_t kind;
  uint64_t rolling;   /* ChunkId rolling-hash part; 0 for BYTES */
  uint8_t sha1[16];   /* ChunkId crypto part (SHA-1 prefix); 0 for BYTES */
} zco_record;

/* A chunk already in the repository index (ChunkIndex::loadIndex input). */
typedef struct {
  uint8_t sha1[16];
  uint64_t rolling;
  uint32_t size;
  uint32_t pad;
} zco_seed;

uint64_t zco_digest(const uint8_t* p, uint64_t n);
int zco_chunk(const uint8_t* data, uint64_t n, uint32_t W, const zco_seed* seeds,
              size_t nseeds, uint64_t feed_max, zco_record** out, size_t* nout);
/* the same with options: ZCO_OPT_PREFILTER adds an exact key prefilter in
 * front of the hash_map (identical records, faster misses) */
enum { ZCO_OPT_PREFILTER = 1 };
int zco_chunk_ex(const uint8_t* data, uint64_t n, uint32_t W, const zco_seed* seeds,
                 size_t nseeds, uint64_t feed_max, uint32_t opts, zco_record** out, size_t* nout);
void zco_free(void* p);
void zco_sha1(const uint8_t* p, uint64_t n, uint8_t* out20);
void zco_fill_splitmix64(uint8_t* out, uint64_t n, uint64_t seed);
/* Synthetic stream from a spec: comma-separated segments
 *   R<seed>:<len>  splitmix64 bytes      Z:<len>      zeros
 *   B<byte>:<len>  constant byte          C<off>:<len> copy of earlier bytes
 *                                                      (overlap allowed)  */
int zco_gen(const char* spec, uint8_t** out, uint64_t* n);

#ifdef __cplusplus
}
#endif
#endif
