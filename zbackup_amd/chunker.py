"""Python host mirror of zbackup's BackupCreator on the MI355X engine.

Names, argument meaning and error behaviour follow the reference:
  BackupCreator(config, chunkIndex, writer)      backup_creator.hh:83
    getInputBuffer / getInputBufferSize          backup_creator.cc:40-54
    handleMoreData(added)                        backup_creator.cc:56-108
    finish()                                     backup_creator.cc:147-172
    getBackupData(string &)  -- callable once    backup_creator.cc:275-280
  ChunkId::toBlob  (16-byte SHA-1 prefix + LE rolling hash)   chunk_id.cc:19-27
  Message::serialize (varint32 length + BackupInstruction)    message.cc:16-23

All work runs in libzchunk.so on the GPU; there is no CPU fallback.
"""
import ctypes
import struct

import numpy as np

from . import _lib

RECORD_DTYPE = np.dtype([("offset", "<u8"), ("size", "<u4"), ("kind", "<u4"),
                         ("rolling", "<u8"), ("sha1", "u1", (16,))])
KIND_CHAR = "NDB"
SEED_DTYPE = np.dtype([("sha1", np.uint8, 16), ("rolling", np.uint64), ("size", np.uint32), ("reserved", np.uint32)])
# zc_chunk_meta (ABI 5): a chunk's content-anchor metadata, keyed by its ChunkId
META_DTYPE = np.dtype([("sha1", np.uint8, 16), ("rolling", "<u8"), ("size", "<u4"), ("anchor_def", "<u4"),
                       ("anchor", "<u4"), ("gear", "<u4"), ("fingerprint", "<u8")])


def _check(L, ctx, rc, what):
    if rc != _lib.ZC_OK:
        msg = L.zc_last_error(ctx) if ctx else b""
        raise _lib.ZcError(f"{what} failed ({rc}): {(msg or b'').decode(errors='replace')}")


def chunk_id_blob(sha1_16, rolling):
    """ChunkId::toBlob (chunk_id.cc:19-27)."""
    return bytes(sha1_16) + struct.pack("<Q", rolling)


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def serialize_instruction(chunk_blob=None, raw=None):
    """Message::serialize of one BackupInstruction (zbackup.proto:149-159)."""
    body = b""
    if chunk_blob is not None:
        body += b"\x0a" + _varint(len(chunk_blob)) + chunk_blob
    if raw is not None:
        body += b"\x12" + _varint(len(raw)) + raw
    return _varint(len(body)) + body


def _seed_array(sha1, rolling, size):
    """(sha1 (n, 16) uint8, rolling (n,) uint64, size scalar or (n,)) -> SEED_DTYPE array (zc_seed)."""
    rolling = np.ascontiguousarray(rolling, dtype=np.uint64).reshape(-1)
    n = rolling.size
    rec = np.zeros(n, dtype=SEED_DTYPE)
    assert rec.dtype.itemsize == ctypes.sizeof(_lib.ZcSeed)
    if n:
        rec["sha1"] = np.asarray(sha1, dtype=np.uint8).reshape(n, 16)
        rec["rolling"] = rolling
        rec["size"] = size
    return rec


def anchor_def(chunk_max_size):
    """zc_anchor_def: the anchor definition this build's metadata carries for W."""
    return int(_lib.load().zc_anchor_def(int(chunk_max_size)))


class BackupCreator:
    """One stream through the engine.  `seeds` are (sha1_16, rolling, size)
    entries of an existing index (ChunkIndex::loadIndex).  `window`: bytes of
    the feed held in HBM (None: the library's default, 1 GiB; 0: the whole
    stream, resolved at finish()); see zc_set_window."""

    def __init__(self, chunk_max_size=65536, seeds=(), device=0, sha1=True, timing=False, staged_screen=True,
                 window=None):
        self._L = _lib.load()
        self.chunk_max_size = int(chunk_max_size)
        flags = (_lib.ZC_FLAG_SHA1 if sha1 else 0) | (_lib.ZC_FLAG_TIMING if timing else 0)
        if not staged_screen:  # diagnostics: the lane-per-KiB exact screen only
            flags |= _lib.ZC_FLAG_NO_STAGED_SCREEN
        ctx = ctypes.c_void_p()
        rc = self._L.zc_create(ctypes.byref(ctx), self.chunk_max_size, device, flags)
        if rc != _lib.ZC_OK:
            raise _lib.ZcError(f"zc_create failed ({rc})")
        self._ctx = ctx
        self._new_stream()
        if window is not None:
            _check(self._L, self._ctx, self._L.zc_set_window(self._ctx, int(window)), "zc_set_window")
        self.seed_index(seeds)

    def seed_index(self, seeds):
        """Add (sha1_16, rolling, size) ids to the context's index (zc_seed_index:
        what ChunkIndex::loadIndex registers, chunk_index.cc:26-79,163-182)."""
        seeds = list(seeds)
        if seeds:
            arr = (_lib.ZcSeed * len(seeds))()
            for i, (sha, rolling, size) in enumerate(seeds):
                arr[i].sha1[:] = list(sha[:16])
                arr[i].rolling = rolling
                arr[i].size = size
            _check(self._L, self._ctx, self._L.zc_seed_index(self._ctx, arr, len(seeds)), "zc_seed_index")

    def seed_index_arrays(self, sha1, rolling, size):
        """seed_index for ids given as arrays: sha1 (n, 16) uint8, rolling (n,)
        uint64, size a scalar or (n,) -- one copy into the ZcSeed array (an
        index file's worth of ids without a Python loop)."""
        rec = _seed_array(sha1, rolling, size)
        if rec.size == 0:
            return
        arr = (_lib.ZcSeed * rec.size).from_buffer(rec)
        _check(self._L, self._ctx, self._L.zc_seed_index(self._ctx, arr, rec.size), "zc_seed_index")

    def seed_index_meta(self, sha1, rolling, size, meta):
        """zc_seed_index_meta: the ids of an existing index (arrays as in
        seed_index_arrays) with the anchor metadata kept for them (a META_DTYPE
        array, e.g. from export_chunk_meta of the backups that wrote them).  Ids
        whose metadata matches join the anchor-probed historic index, the rest
        are seeded by value; metadata of ids not given is ignored."""
        rec = _seed_array(sha1, rolling, size)
        meta = np.ascontiguousarray(meta, dtype=META_DTYPE)
        assert META_DTYPE.itemsize == ctypes.sizeof(_lib.ZcChunkMeta)
        _check(self._L, self._ctx,
               self._L.zc_seed_index_meta(self._ctx, rec.ctypes.data if rec.size else None, rec.size,
                                          meta.ctypes.data if meta.size else None, meta.size),
               "zc_seed_index_meta")

    def export_chunk_meta(self):
        """zc_export_chunk_meta: the anchor metadata of the W-byte chunks this
        context's streams added to its index (ZC_FLAG_SHA1), as a META_DTYPE
        array in the order they were added."""
        need = ctypes.c_size_t()
        self._L.zc_export_chunk_meta(self._ctx, None, 0, ctypes.byref(need))
        out = np.zeros(need.value, dtype=META_DTYPE)
        if need.value:
            _check(self._L, self._ctx,
                   self._L.zc_export_chunk_meta(self._ctx, out.ctypes.data, out.size, ctypes.byref(need)),
                   "zc_export_chunk_meta")
        return out

    def _new_stream(self):
        # A fed stream's records are taken from the context as they are cut and
        # serialized right away, while their bytes are still in the feed window
        # (bytes_to_emit reads them): BackupCreator::outputInstruction also runs
        # inside handleMoreData (backup_creator.cc:267-273).  A long stream through
        # a bounded window would otherwise have evicted them by getBackupData.
        self._data = bytearray()  # BackupInstruction stream of the records taken
        self._taken = []          # record arrays taken from the context, stream order
        self._given = 0           # arrays of _taken that take_records() has returned
        self._data_taken = False

    def _drain(self):
        """Take the complete records from the context and serialize them now."""
        n = self._L.zc_record_count(self._ctx)
        if not n:
            return
        out = np.zeros(n, dtype=RECORD_DTYPE)
        got = ctypes.c_size_t()
        _check(self._L, self._ctx,
               self._L.zc_take_records(self._ctx, out.ctypes.data_as(ctypes.POINTER(_lib.ZcRecord)), n,
                                       ctypes.byref(got)), "zc_take_records")
        out = out[: got.value]
        self._data += self._serialize(out)
        self._taken.append(out)

    def _serialize(self, recs):
        recs = np.ascontiguousarray(recs)
        need = ctypes.c_size_t()
        self._L.zc_serialize_records(self._ctx, recs.ctypes.data, len(recs), None, 0, ctypes.byref(need))
        out = np.zeros(max(need.value, 1), dtype=np.uint8)
        rc = self._L.zc_serialize_records(self._ctx, recs.ctypes.data, len(recs), out.ctypes.data, out.size,
                                          ctypes.byref(need))
        _check(self._L, self._ctx, rc, "zc_serialize_records")
        return out[:need.value].tobytes()

    # -- feed contract -------------------------------------------------------
    def get_input_buffer(self):
        """Writable view of getInputBufferSize() bytes (pinned host staging)."""
        p = self._L.zc_get_input_buffer(self._ctx)
        if not p:
            raise _lib.ZcError("no input buffer after finish()")
        n = self._L.zc_get_input_buffer_size(self._ctx)
        return (ctypes.c_uint8 * n).from_address(p)

    def get_input_buffer_size(self):
        return self._L.zc_get_input_buffer_size(self._ctx)

    def handle_more_data(self, added):
        _check(self._L, self._ctx, self._L.zc_handle_more_data(self._ctx, added), "handleMoreData")
        self._drain()

    def feed(self, data):
        """The read loop of zutils.cc:100-124 over `data`: each piece copied into
        getInputBuffer() (at most getInputBufferSize() bytes), handleMoreData,
        and the records cut by then taken and serialized while their payload
        bytes are still in the feed window (a long stream slides the window on
        the next getInputBuffer call)."""
        data = np.ascontiguousarray(np.frombuffer(memoryview(data), dtype=np.uint8))
        pos = 0
        while pos < data.size:
            p = self._L.zc_get_input_buffer(self._ctx)
            room = self._L.zc_get_input_buffer_size(self._ctx)
            if not p or not room:
                msg = self._L.zc_last_error(self._ctx) or b""
                raise _lib.ZcError(f"getInputBuffer failed: {msg.decode(errors='replace')}")
            take = min(room, data.size - pos)
            ctypes.memmove(p, data.ctypes.data + pos, take)
            self.handle_more_data(take)
            pos += take

    def finish(self):
        _check(self._L, self._ctx, self._L.zc_finish(self._ctx), "finish")
        self._drain()

    # -- device-resident stream ----------------------------------------------
    def chunk_device(self, ptr, n):
        """Process `n` bytes already in HBM at device pointer `ptr` (e.g. a torch
        uint8 tensor's data_ptr()); feed + finish in one call."""
        self._new_stream()
        _check(self._L, self._ctx, self._L.zc_chunk_device(self._ctx, ctypes.c_void_p(ptr), n),
               "zc_chunk_device")

    def chunk_host(self, ptr, n):
        """Process `n` bytes in host memory at address `ptr` (pinned for full
        speed): HBM copies in 64 MiB segments overlapped with the scan, then
        the same pipeline as chunk_device (zutils.cc:100-124 read loop + finish)."""
        self._new_stream()
        _check(self._L, self._ctx, self._L.zc_chunk_host(self._ctx, ctypes.c_void_p(ptr), n), "zc_chunk_host")

    # -- results -------------------------------------------------------------
    def _held(self):
        n = self._L.zc_record_count(self._ctx)
        out = np.zeros(n, dtype=RECORD_DTYPE)
        got = ctypes.c_size_t()
        _check(self._L, self._ctx,
               self._L.zc_get_records(self._ctx, out.ctypes.data_as(ctypes.POINTER(_lib.ZcRecord)), n,
                                      ctypes.byref(got)), "zc_get_records")
        return out[: got.value]

    def records(self):
        """Every record of the stream so far, in stream order (those already
        taken from the context and those it still holds)."""
        held = self._held()
        if not self._taken:
            return held
        return np.concatenate(self._taken + [held])

    def take_records(self):
        """Complete records cut since the last take_records() (the
        instructions outputInstruction writes during handleMoreData)."""
        self._drain()
        new = self._taken[self._given:]
        self._given = len(self._taken)
        return np.concatenate(new) if new else np.zeros(0, dtype=RECORD_DTYPE)

    @property
    def window(self):
        return int(self._L.zc_get_window(self._ctx))

    def record_tuples(self):
        """(kind_char, offset, size, rolling, sha1_hex) -- the oracle's format."""
        return [(KIND_CHAR[r["kind"]], int(r["offset"]), int(r["size"]), int(r["rolling"]),
                 bytes(r["sha1"]).hex()) for r in self.records()]

    def read_stream(self, offset, n):
        buf = np.empty(n, dtype=np.uint8)
        _check(self._L, self._ctx, self._L.zc_read_stream(self._ctx, offset, n, buf.ctypes.data),
               "zc_read_stream")
        return buf.tobytes()

    def stream_data(self, offset, n):
        """zc_stream_data: the bytes from the feed window's host mirror without a
        library-side copy (None when they are not in host memory)."""
        p = self._L.zc_stream_data(self._ctx, offset, n)
        return ctypes.string_at(p, n) if p else None

    def get_backup_data(self):
        """Serialized BackupInstruction stream; like the reference, only once."""
        if self._data_taken:
            raise _lib.ZcError("getBackupData() called twice")
        self._data_taken = True
        self._drain()
        return bytes(self._data)

    def stats(self):
        st = _lib.ZcStats()
        _check(self._L, self._ctx, self._L.zc_get_stats(self._ctx, ctypes.byref(st)), "zc_get_stats")
        return {name: getattr(st, name) for name, _ in _lib.ZcStats._fields_}

    def scan_ms(self):
        """zc_stats.scan_ms of the last stream, without building the stats dict
        (bench.py reads it inside its timed loop)."""
        st = getattr(self, "_st_buf", None)
        if st is None:
            st = self._st_buf = _lib.ZcStats()
        _check(self._L, self._ctx, self._L.zc_get_stats(self._ctx, ctypes.byref(st)), "zc_get_stats")
        return st.scan_ms

    def reset(self):
        _check(self._L, self._ctx, self._L.zc_reset(self._ctx), "zc_reset")
        self._new_stream()

    def forget_stream_chunks(self):
        """Drop the index entries this context's streams added (Writer::add ->
        ChunkIndex::addChunk), keeping the seeded index: the next stream sees the
        index a fresh ZBackup instance loads (chunk_index.cc:26-79)."""
        _check(self._L, self._ctx, self._L.zc_forget_stream_chunks(self._ctx), "zc_forget_stream_chunks")

    def close(self):
        if self._ctx:
            self._L.zc_destroy(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fill_splitmix64(ptr, n, seed, device=0):
    """Seeded synthetic stream written straight into HBM (same bytes as the oracle's)."""
    L = _lib.load()
    rc = L.zc_fill_splitmix64(ctypes.c_void_p(ptr), n, seed, device)
    if rc != _lib.ZC_OK:
        raise _lib.ZcError(f"zc_fill_splitmix64 failed ({rc})")


class Sha256:
    """Whole-stream SHA-256 kept beside BackupCreator by the feed loop
    (sha256.hh:14-35; fed at zutils.cc:119, finished into BackupInfo.sha256 at
    zutils.cc:134).  Host-side, in libzchunk.so (zc_sha256_*)."""

    Size = 32

    def __init__(self):
        self._L = _lib.load()
        h = ctypes.c_void_p()
        _check(self._L, None, self._L.zc_sha256_create(ctypes.byref(h)), "zc_sha256_create")
        self._h = h

    def add(self, data, size=None):
        """Sha256::add(data, size): bytes-like data, or a host address with its size."""
        if size is None:
            buf = memoryview(data).cast("B")
            arr = (ctypes.c_char * len(buf)).from_buffer_copy(buf) if buf.readonly else \
                (ctypes.c_char * len(buf)).from_buffer(buf)
            ptr, size = ctypes.addressof(arr), len(buf)
        else:
            ptr = data
        _check(self._L, None, self._L.zc_sha256_add(self._h, ptr, size), "zc_sha256_add")

    def finish(self):
        """Sha256::finish() -> the 32-byte digest; callable once, like SHA256_Final."""
        out = ctypes.create_string_buffer(32)
        _check(self._L, None, self._L.zc_sha256_finish(self._h, out), "zc_sha256_finish")
        return out.raw

    @property
    def uses_sha_extensions(self):
        return self._L.zc_sha256_impl(self._h) == 1

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.zc_sha256_destroy(h)
            self._h = None
