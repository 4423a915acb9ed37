/* zchunk.h -- C ABI of the MI355X rolling-hash chunking engine (libzchunk.so).
 *
 * Drop-in for the inner loop of zbackup's BackupCreator: a byte stream goes
 * in, the backup instruction records come out, bit-exact with
 * /root/reference/backup_creator.cc for the same bytes, chunk.max_size and
 * index contents.  Plain C types only; every call returns an int status
 * (ZC_OK == 0, negative on error; zc_last_error() has the message).  One
 * context per stream per GPU.  Every entry point that takes a context holds a
 * per-context lock for the whole call, so calls on one context from several
 * threads are serialized; give each concurrent thread (a bundle compressor
 * beside the feeding thread, say) a context of its own for concurrency.
 *
 * Reference interfaces each entry point replaces:
 *   zc_create              BackupCreator::BackupCreator(Config const &, ChunkIndex &,
 *                          ChunkStorage::Writer &)        backup_creator.hh:83 / .cc:18-38
 *                          (chunk.max_size = W: zbackup.proto:79, config.cc:266-282)
 *   zc_seed_index          ChunkIndex::loadIndex -> registerNewChunkId, the static
 *                          probe set of an existing repository   chunk_index.cc:26-79,163-182
 *   zc_seed_index_meta     the same, with the content-anchor metadata a sidecar kept for
 *                          the ids (so the anchor probe finds them, not the per-byte
 *                          screen): loadIndex + the sidecar read beside it
 *                                                                chunk_index.cc:26-79,163-182,
 *                                                                zbackup_base.cc:87-100
 *   zc_export_chunk_meta   that metadata for the chunks this context's streams added, for the
 *                          sidecar written at ChunkStorage::Writer::commit
 *                                                                chunk_storage.cc:61-90,
 *                                                                chunk_index.cc:185-202
 *   zc_set_window          the ring of W + page bytes the creator reads through
 *                          (backup_creator.cc:28-37): the stream's bytes held in HBM
 *   zc_get_input_buffer    BackupCreator::getInputBuffer()       backup_creator.hh:78 / .cc:40-43
 *   zc_get_input_buffer_size  BackupCreator::getInputBufferSize() backup_creator.hh:79 / .cc:45-54
 *   zc_handle_more_data    BackupCreator::handleMoreData(unsigned) backup_creator.hh:81 / .cc:56-108
 *   zc_finish              BackupCreator::finish()               backup_creator.hh:85 / .cc:147-172
 *   zc_get_records         BackupCreator::getBackupData(string &) as structured records
 *                          (one per BackupInstruction, zbackup.proto:149-159)
 *                                                                backup_creator.hh:89 / .cc:275-280
 *   zc_take_records        the same, drained as they are cut (outputInstruction,
 *                          backup_creator.cc:267-273, runs during handleMoreData)
 *   zc_chunk_device        the same stream already resident in HBM (feed + finish in one call)
 *   zc_chunk_host          the same stream in host memory, copy overlapped with the scan
 *                          (the read loop of zutils.cc:100-124 + finish in one call)
 *   zc_last_error          the DEF_EX exceptions / CHECK aborts of the reference
 *                          (backup_creator.cc:112,165-166, chunk_index.hh:88-89)
 */
#ifndef ZCHUNK_H
#define ZCHUNK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZCHUNK_ABI_VERSION 5

enum zc_status {
  ZC_OK = 0,
  ZC_ERR_ARG = -1,      /* bad argument (null pointer, W == 0, misaligned device buffer) */
  ZC_ERR_HIP = -2,      /* HIP runtime error (message in zc_last_error) */
  ZC_ERR_NOMEM = -3,    /* device or host allocation failed */
  ZC_ERR_STATE = -4     /* call out of order (e.g. feeding after zc_finish) */
};

/* context flags */
enum {
  ZC_FLAG_SHA1 = 1u,     /* compute the SHA-1 half of every chunk id (ChunkId::cryptoHash)
                            and register the stream's new chunks in the context's index,
                            so a later stream on the same context can match them */
  ZC_FLAG_TIMING = 2u,   /* record per-stage device timings (zc_get_stats) */
  ZC_FLAG_NO_STAGED_SCREEN = 4u  /* diagnostics: run the exact-hash screen on its lane-per-KiB
                                    kernel only (same records, slower; tests cover both) */
};

/* record kinds: chunk_to_emit of a chunk cut and saved by this stream (NEW),
 * chunk_to_emit of a window matched in the index (DUP), bytes_to_emit (BYTES,
 * fragments under 128 bytes; the bytes are the caller's [offset, offset+size)) */
enum { ZC_CHUNK_NEW = 0, ZC_CHUNK_DUP = 1, ZC_BYTES = 2 };

typedef struct {
  uint64_t offset;   /* stream offset of the first byte the instruction covers */
  uint32_t size;     /* bytes covered */
  uint32_t kind;     /* ZC_CHUNK_NEW / ZC_CHUNK_DUP / ZC_BYTES */
  uint64_t rolling;  /* ChunkId::rollingHash (RollingHash digest); 0 for BYTES */
  uint8_t sha1[16];  /* ChunkId::cryptoHash (SHA-1 prefix) if ZC_FLAG_SHA1, else 0 */
} zc_record;

/* one entry of an existing index: a ChunkId and the chunk size */
typedef struct {
  uint8_t sha1[16];
  uint64_t rolling;
  uint32_t size;
  uint32_t reserved;
} zc_seed;

/* ABI 5: the content-anchor metadata of one W-byte chunk of an index.  The
 * engine finds windows equal to indexed chunks by their first content anchor
 * (DESIGN.md §2); chunks whose bytes it never held (a repository's earlier
 * backups, known to ChunkIndex only by id) are otherwise screened for by key at
 * every byte.  The metadata is a pure function of the chunk's bytes, so it never
 * goes stale: a caller keeps it beside the repository's index, keyed by the
 * ChunkId, and seeds it with the ids (zc_seed_index_meta).  Matches are still
 * confirmed by rolling key + SHA-1 prefix, as ChunkIndex::findChunk confirms
 * them (chunk_index.cc:119-143), whatever the metadata says. */
#define ZC_META_NO_ANCHOR 0xFFFFFFFFu
typedef struct {
  uint8_t sha1[16];      /* ChunkId::cryptoHash */
  uint64_t rolling;      /* ChunkId::rollingHash */
  uint32_t size;         /* chunk size (W for every entry the engine exports) */
  uint32_t anchor_def;   /* zc_anchor_def() of the engine that computed the entry */
  uint32_t anchor;       /* offset of the chunk's first content anchor, ZC_META_NO_ANCHOR: none */
  uint32_t gear;         /* the anchor's key */
  uint64_t fingerprint;  /* the anchor's 64-bit fingerprint */
} zc_chunk_meta;

typedef struct {
  double scan_ms;        /* zc_scan kernel (HIP events on the context stream) */
  double resolve_ms;     /* everything after the scan: total_ms - scan_ms with ZC_FLAG_TIMING */
  double total_ms;       /* whole call, wall clock */
  uint64_t bytes;        /* stream length */
  uint64_t anchors;      /* content anchors found by the scan */
  uint64_t candidates;   /* anchor-probe candidates */
  uint64_t epochs;       /* resolution epochs (1 + grid-shifting matches) */
  uint64_t fscan_runs;   /* screen-hit runs from the exact-hash screen */
  double meta_ms;        /* epoch index + probe batch (first epoch: device time from the scan's end;
                            later ones: wall clock; summed) */
  double probe_ms;       /* anchor table + probe + candidate verification */
  double fscan_ms;       /* exact-hash screen */
  double walk_ms;        /* boundary walk + record assembly on the host */
  double finalize_ms;    /* digests of cut pieces, SHA-1 ids */
  double fbatch_ms;      /* (part of walk_ms) batched key/byte/SHA-1 checks of screen hits */
  uint64_t window_bytes; /* feed window (zc_set_window; 0: unbounded) */
  uint64_t hbm_bytes;    /* device memory the context holds now */
  uint64_t segments;     /* window segments resolved during the feed */
  uint64_t hist_entries; /* historic index entries (chunks whose bytes have left HBM) */
  /* parts of finalize_ms (ZC_FLAG_SHA1): */
  double sha_wait_ms;    /* blocked on the grid chunks' SHA-1 and its copy to the host */
  double sha_fill_ms;    /* after it: SHA-1 prefixes into the records, the new chunks' index entries completed */
  double hist_ms;        /* before it: the stream's new chunks joining the context's index (keys, anchors) */
  uint64_t respeculations; /* streams redone because a speculative key + SHA-1 class join proved wrong */
  /* ABI 4: */
  uint64_t chk_rebuilds;   /* the one-level static screen's check table rebuilt larger for an epoch's own keys */
  /* ABI 5: */
  uint64_t hist_seeded;    /* historic index entries seeded with anchor metadata (zc_seed_index_meta) */
  uint64_t by_value;       /* index entries known by value only (the exact screen's key set) */
} zc_stats;

typedef struct zc_ctx zc_ctx;

int zc_create(zc_ctx** out, uint32_t chunk_max_size, int device, uint32_t flags);
int zc_destroy(zc_ctx* ctx);
int zc_seed_index(zc_ctx* ctx, const zc_seed* seeds, size_t n);
/* ABI 5.  Seed the ids of an existing index (as zc_seed_index) together with the
 * metadata kept for them: an id whose entry in meta[0, nm) matches its full
 * ChunkId and size W and carries this engine's anchor definition joins the
 * historic index (found by the anchor probe); the other ids are seeded by value
 * (the exact screen); meta entries for ids not in seeds are ignored (an id
 * that is not in the index never matches).  Call before the context's first
 * stream adds chunks to its index (or after zc_forget_stream_chunks):
 * ZC_ERR_STATE otherwise. */
int zc_seed_index_meta(zc_ctx* ctx, const zc_seed* seeds, size_t n, const zc_chunk_meta* meta, size_t nm);
/* ABI 5.  The metadata of the W-byte chunks this context's streams added to its
 * index (ZC_FLAG_SHA1: Writer::add -> ChunkIndex::addChunk; in the order they
 * were added; not the seeded ones): *n_out = their count; ZC_ERR_ARG (with
 * *n_out the count) when cap is smaller. */
int zc_export_chunk_meta(const zc_ctx* ctx, zc_chunk_meta* out, size_t cap, size_t* n_out);
/* the anchor definition of this build for chunk.max_size W (it names the gear,
 * the anchor rate for W, the minimum anchor offset and the fingerprint);
 * metadata of another definition is ignored when seeding */
uint32_t zc_anchor_def(uint32_t chunk_max_size);

/* Host feed (zero-copy contract of BackupCreator: fill getInputBuffer() with up
 * to getInputBufferSize() bytes, then report how many were written).
 *
 * The feed streams through a bounded window (default 1 GiB, at least
 * 8 W + 16 MiB; zc_set_window before the stream's first byte, 0 = keep the whole
 * stream in HBM and resolve it at zc_finish): the bytes are copied to HBM as
 * they arrive, each half window is chunked during zc_handle_more_data, and the
 * window then slides, so device and pinned host memory stay at the window's
 * size for a stream of any length.  Chunks whose bytes leave the window stay
 * in the index by {rolling key, SHA-1 prefix, first content anchor} (the
 * historic index), as the reference's index keeps ids, not bytes.
 * Records are complete as soon as they are cut; zc_take_records drains them.
 * The payload bytes of records taken (NEW chunks for Writer::add, BYTES for
 * bytes_to_emit) stay readable with zc_read_stream until the next
 * zc_get_input_buffer / zc_get_input_buffer_size / zc_feed / zc_finish call. */
/* (the window's buffers are made on a helper thread from this call on, joined
 * by the first zc_get_input_buffer: call it early -- before the index load --
 * to overlap the ~0.3 s it takes to pin 1 GiB of host memory) */
int zc_set_window(zc_ctx* ctx, uint64_t bytes);
uint64_t zc_get_window(const zc_ctx* ctx);
void* zc_get_input_buffer(zc_ctx* ctx);
size_t zc_get_input_buffer_size(zc_ctx* ctx);
int zc_handle_more_data(zc_ctx* ctx, size_t added);
/* copying convenience form: n bytes through getInputBuffer / handleMoreData in
 * pieces.  A call of more than getInputBufferSize() bytes may resolve several
 * window halves and slide the window between them, so take the records after
 * every call of at most that size when their payload bytes are needed
 * (bytes_to_emit, Writer::add), as the zero-copy loop does. */
int zc_feed(zc_ctx* ctx, const void* host, size_t n);
int zc_finish(zc_ctx* ctx);

/* device-resident stream: d_data is a device pointer on the context's GPU,
 * 16-byte aligned; the call runs the whole pipeline and fills the records.
 * The context's stream is ordered after work already queued on the legacy
 * default stream (so a buffer just written there is read complete). */
int zc_chunk_device(zc_ctx* ctx, const void* d_data, uint64_t n);

/* stream in host memory (pinned for full speed): copied to HBM in 64 MiB
 * segments on a side stream, each segment scanned as soon as it has landed,
 * then the same pipeline as zc_chunk_device; the end-to-end form of
 * backup_creator.cc's loop, with the feed's copies overlapped with the work */
int zc_chunk_host(zc_ctx* ctx, const void* host, uint64_t n);

size_t zc_record_count(const zc_ctx* ctx);  /* complete records held (cut, ids filled in, not yet taken) */
int zc_get_records(const zc_ctx* ctx, zc_record* out, size_t cap, size_t* n_out);
/* move up to cap complete records out of the context, in stream order */
int zc_take_records(zc_ctx* ctx, zc_record* out, size_t cap, size_t* n_out);
int zc_get_stats(const zc_ctx* ctx, zc_stats* out);
int zc_reset(zc_ctx* ctx); /* begin a new stream (the seeded index is kept) */
/* drop the index entries this context's streams added (ZC_FLAG_SHA1: Writer::add ->
 * ChunkIndex::addChunk, chunk_storage.cc:31-46), keeping the seeded ones.  Only for streams
 * whose backups are DISCARDED (never committed), or for benchmarking a first backup on warm
 * buffers: a committed backup's chunks are in its index file, which ChunkIndex::loadIndex
 * reads on the next open (chunk_storage.cc:61-80, chunk_index.cc:26-79), so they must stay
 * in the index (keep them, or re-seed them from the written index). */
int zc_forget_stream_chunks(zc_ctx* ctx);
/* copy bytes [offset, offset+n) of the last processed stream to host memory
 * (the payload of BYTES records, for serializing bytes_to_emit, and of NEW
 * chunks, for Writer::add); for a fed stream, the bytes still in its window */
int zc_read_stream(const zc_ctx* ctx, uint64_t offset, size_t n, void* host_out);
/* the same bytes without a copy, for a fed stream: a pointer into the feed
 * window's pinned host mirror, valid until the next zc_get_input_buffer /
 * zc_get_input_buffer_size / zc_feed / zc_finish / zc_reset call; NULL when
 * the range is not in host memory (a device-resident stream: zc_read_stream) */
const void* zc_stream_data(const zc_ctx* ctx, uint64_t offset, size_t n);
/* the records' BackupInstruction stream, as BackupCreator::outputInstruction writes it
 * (Message::serialize, message.cc:16-23: varint32 length + field 1 chunk_to_emit =
 * ChunkId::toBlob (chunk_id.cc:19-27) | field 2 bytes_to_emit, the record's bytes read from
 * the last stream as zc_read_stream does): n records into out (cap bytes); *n_out = the bytes
 * written, or needed (ZC_ERR_ARG) when cap is too small */
int zc_serialize_records(const zc_ctx* ctx, const zc_record* recs, size_t n, void* out, size_t cap,
                         size_t* n_out);
const char* zc_last_error(const zc_ctx* ctx);

/* synthetic seeded stream on the device (tests / benchmarks): byte k is byte
 * k mod 8 of splitmix64 word k / 8, little-endian */
int zc_fill_splitmix64(void* d_data, uint64_t n, uint64_t seed, int device);

/* Whole-stream SHA-256 of the input, host side (replaces the Sha256 the feed loop
 * keeps beside BackupCreator: sha256.hh:14-35, fed at zutils.cc:119, finished into
 * BackupInfo.sha256 at zutils.cc:134, checked on restore at zutils.cc:225-232).
 * One serial chain, so it runs on the host CPU (SHA extensions when present). */
typedef struct zc_sha256 zc_sha256;
int zc_sha256_create(zc_sha256** out);                           /* Sha256::Sha256  sha256.cc:8-11 */
int zc_sha256_add(zc_sha256* h, const void* data, size_t n);     /* Sha256::add     sha256.cc:13-16 */
int zc_sha256_finish(zc_sha256* h, uint8_t out[32]);             /* Sha256::finish  sha256.cc:18-21; once */
int zc_sha256_destroy(zc_sha256* h);
int zc_sha256_impl(const zc_sha256* h); /* 1: x86 SHA extensions, 0: scalar */

/* ---- Bundle writer offload ----
 * ChunkStorage::Writer::add's bundling rule (chunk_storage.cc:31-46): the chunks that
 * index.addChunk accepted, in order; chunk i joins the current bundle unless the bundle's
 * payload + sizes[i] > max_payload (config bundle.max_payload_size, default 0x200000,
 * zbackup.proto:88), which first finishes the bundle.  bundle_of[i] receives chunk i's
 * bundle, *n_bundles their count.  Host bookkeeping only (no device work). */
int zc_bundle_plan(const uint64_t* sizes, size_t n, uint64_t max_payload, uint32_t* bundle_of,
                   size_t* n_bundles);
/* Bundle::Creator::addChunk's payload (bundle.cc:30-36) on the device: chunk i's bytes
 * d_src[src_off[i] ..+ sizes[i]) appended to d_payload back to back (HBM to HBM). */
int zc_bundle_gather(zc_ctx* ctx, const void* d_src, const uint64_t* src_off, const uint64_t* sizes,
                     size_t n, void* d_payload);
/* The lzo1x_1 compression Bundle::Creator::write runs on each bundle's payload
 * (bundle.cc:120-151 -> LZO1X_1_Encoder::doProcessNoSize, compression.cc:586-606 -> liblzo2
 * lzo1x_1_compress) with zbackup's framing (NoStreamAndUnknownSizeEncoder::doProcess,
 * compression.cc:435-466: LE32 size, "EFGH", LE32 compressed size, "MNOP", the LZO stream):
 * payload i = d_payload[pay_off[i] ..+ pay_size[i]) (pay_size[i] < 2^32), its framed bytes go
 * to d_out + out_off[i], which must leave zc_lzo_capacity(pay_size[i]) bytes; out_size[i]
 * (host) receives their count.  The bytes equal what the reference writes for the payload. */
uint64_t zc_lzo_capacity(uint64_t payload_size); /* LZO1X_1_Encoder::suggestOutputSize + 16 */
int zc_lzo_compress(zc_ctx* ctx, const void* d_payload, const uint64_t* pay_off, const uint64_t* pay_size,
                    size_t n, void* d_out, const uint64_t* out_off, uint64_t* out_size);
/* the same for payloads in host memory (copied to HBM, compressed, copied back to
 * out + out_off[i]): the form Bundle::Creator::write can call per finished bundle (or per
 * batch of them) without device buffers of its own */
int zc_lzo_compress_host(zc_ctx* ctx, const void* payload, const uint64_t* pay_off, const uint64_t* pay_size,
                         size_t n, void* out, const uint64_t* out_off, uint64_t* out_size);
/* Adler-32 (zlib's adler32 from its initial value 1, as Adler32 wraps it: adler32.hh:13-33) of
 * each device range d_base[off[i] ..+ len[i]) -> out[i] (host).  EncryptedFile::OutputStream
 * keeps one running Adler-32 over everything a bundle file holds and writes it after the
 * BundleInfo and after the payload (encrypted_file.cc:248-300,336-340, bundle.cc:116,153):
 * the payload's share comes from here, joined to the running value with zlib's
 * adler32_combine(running, out[i], len[i]). */
int zc_adler32(zc_ctx* ctx, const void* d_base, const uint64_t* off, const uint64_t* len, size_t n,
               uint32_t* out);
/* device time of the last zc_lzo_compress's parse kernel (ms) and its 48 KiB blocks */
int zc_lzo_last_stats(const zc_ctx* ctx, double* parse_ms, uint64_t* blocks);

int zc_abi_version(void);
/* digest of the sources this library was built from (zbackup_amd/_build.py
 * source_digest(): sha256 of every source and header, first 16 hex digits).
 * Loaders compare it with the checked-out tree and refuse a stale binary. */
const char* zc_build_id(void);

#ifdef __cplusplus
}
#endif
#endif
