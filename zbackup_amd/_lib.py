"""ctypes binding of libzchunk.so (include/zchunk.h).

The library is built in-tree (zbackup_amd/libzchunk.so).  Loading fails loudly
if it is missing: there is no CPU fallback for the product path.
"""
import ctypes
import os

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libzchunk.so")

ZC_OK, ZC_ERR_ARG, ZC_ERR_HIP, ZC_ERR_NOMEM, ZC_ERR_STATE = 0, -1, -2, -3, -4
ZC_FLAG_SHA1, ZC_FLAG_TIMING, ZC_FLAG_NO_STAGED_SCREEN = 1, 2, 4
ZC_CHUNK_NEW, ZC_CHUNK_DUP, ZC_BYTES = 0, 1, 2

# every symbol include/zchunk.h declares
EXPORTS = ["zc_create", "zc_destroy", "zc_seed_index", "zc_get_input_buffer",
           "zc_get_input_buffer_size", "zc_handle_more_data", "zc_feed", "zc_finish",
           "zc_chunk_device", "zc_record_count", "zc_get_records", "zc_get_stats", "zc_reset",
           "zc_last_error", "zc_fill_splitmix64", "zc_abi_version", "zc_read_stream", "zc_chunk_host",
           "zc_forget_stream_chunks", "zc_set_window", "zc_get_window", "zc_take_records", "zc_sha256_create", "zc_sha256_add", "zc_sha256_finish", "zc_sha256_destroy", "zc_sha256_impl",
           "zc_bundle_plan", "zc_bundle_gather", "zc_lzo_capacity", "zc_lzo_compress", "zc_lzo_compress_host", "zc_lzo_last_stats", "zc_adler32", "zc_serialize_records", "zc_stream_data", "zc_build_id",
           "zc_seed_index_meta", "zc_export_chunk_meta", "zc_anchor_def"]
ZC_META_NO_ANCHOR = 0xFFFFFFFF


class ZcRecord(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("size", ctypes.c_uint32), ("kind", ctypes.c_uint32),
                ("rolling", ctypes.c_uint64), ("sha1", ctypes.c_uint8 * 16)]


class ZcSeed(ctypes.Structure):
    _fields_ = [("sha1", ctypes.c_uint8 * 16), ("rolling", ctypes.c_uint64),
                ("size", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class ZcChunkMeta(ctypes.Structure):
    _fields_ = [("sha1", ctypes.c_uint8 * 16), ("rolling", ctypes.c_uint64), ("size", ctypes.c_uint32),
                ("anchor_def", ctypes.c_uint32), ("anchor", ctypes.c_uint32), ("gear", ctypes.c_uint32),
                ("fingerprint", ctypes.c_uint64)]


class ZcStats(ctypes.Structure):
    _fields_ = [("scan_ms", ctypes.c_double), ("resolve_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("bytes", ctypes.c_uint64),
                ("anchors", ctypes.c_uint64), ("candidates", ctypes.c_uint64),
                ("epochs", ctypes.c_uint64), ("fscan_runs", ctypes.c_uint64),
                ("meta_ms", ctypes.c_double), ("probe_ms", ctypes.c_double),
                ("fscan_ms", ctypes.c_double), ("walk_ms", ctypes.c_double),
                ("finalize_ms", ctypes.c_double), ("fbatch_ms", ctypes.c_double),
                ("window_bytes", ctypes.c_uint64), ("hbm_bytes", ctypes.c_uint64),
                ("segments", ctypes.c_uint64), ("hist_entries", ctypes.c_uint64),
                ("sha_wait_ms", ctypes.c_double), ("sha_fill_ms", ctypes.c_double), ("hist_ms", ctypes.c_double),
                ("respeculations", ctypes.c_uint64), ("chk_rebuilds", ctypes.c_uint64),
                ("hist_seeded", ctypes.c_uint64), ("by_value", ctypes.c_uint64)]


class ZcError(RuntimeError):
    pass


_lib = None


def load(path=LIB_PATH):
    """Load libzchunk.so; raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ZcError(f"{path} not built (run zbackup_amd/_build.py or __graft_entry__.build())")
    from . import _build
    if os.path.abspath(path) == LIB_PATH:
        # the in-tree library must be the one the checked-out sources build
        have, want = _build.lib_build_id(path), _build.source_digest()
        if have != want:
            raise ZcError(f"{path} has build id {have}, the sources give {want}: stale binary "
                          "(run zbackup_amd/_build.py)")
    L = ctypes.CDLL(path)
    vp, u32, u64, sz, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int
    sig = {
        "zc_create": (i32, [ctypes.POINTER(vp), u32, i32, u32]),
        "zc_destroy": (i32, [vp]),
        "zc_seed_index": (i32, [vp, ctypes.POINTER(ZcSeed), sz]),
        "zc_get_input_buffer": (vp, [vp]),
        "zc_get_input_buffer_size": (sz, [vp]),
        "zc_handle_more_data": (i32, [vp, sz]),
        "zc_feed": (i32, [vp, vp, sz]),
        "zc_finish": (i32, [vp]),
        "zc_chunk_device": (i32, [vp, vp, u64]),
        "zc_record_count": (sz, [vp]),
        "zc_get_records": (i32, [vp, ctypes.POINTER(ZcRecord), sz, ctypes.POINTER(sz)]),
        "zc_get_stats": (i32, [vp, ctypes.POINTER(ZcStats)]),
        "zc_reset": (i32, [vp]),
        "zc_last_error": (ctypes.c_char_p, [vp]),
        "zc_fill_splitmix64": (i32, [vp, u64, u64, i32]),
        "zc_abi_version": (i32, []),
        "zc_read_stream": (i32, [vp, u64, sz, vp]),
        "zc_chunk_host": (i32, [vp, vp, u64]),
        "zc_forget_stream_chunks": (i32, [vp]),
        "zc_set_window": (i32, [vp, u64]),
        "zc_get_window": (u64, [vp]),
        "zc_take_records": (i32, [vp, ctypes.POINTER(ZcRecord), sz, ctypes.POINTER(sz)]),
        "zc_sha256_create": (i32, [ctypes.POINTER(vp)]),
        "zc_sha256_add": (i32, [vp, vp, sz]),
        "zc_sha256_finish": (i32, [vp, ctypes.c_char_p]),
        "zc_sha256_destroy": (i32, [vp]),
        "zc_sha256_impl": (i32, [vp]),
        # bundle writer offload (host arrays as pointers: numpy .ctypes.data)
        "zc_bundle_plan": (i32, [vp, sz, u64, vp, ctypes.POINTER(sz)]),
        "zc_bundle_gather": (i32, [vp, vp, vp, vp, sz, vp]),
        "zc_lzo_capacity": (u64, [u64]),
        "zc_lzo_compress": (i32, [vp, vp, vp, vp, sz, vp, vp, vp]),
        "zc_lzo_compress_host": (i32, [vp, vp, vp, vp, sz, vp, vp, vp]),
        "zc_adler32": (i32, [vp, vp, vp, vp, sz, vp]),
        "zc_serialize_records": (i32, [vp, vp, sz, vp, sz, ctypes.POINTER(sz)]),
        "zc_lzo_last_stats": (i32, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64)]),
        "zc_stream_data": (vp, [vp, u64, sz]),
        "zc_build_id": (ctypes.c_char_p, []),
        "zc_seed_index_meta": (i32, [vp, vp, sz, vp, sz]),
        "zc_export_chunk_meta": (i32, [vp, vp, sz, ctypes.POINTER(sz)]),
        "zc_anchor_def": (u32, [u32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def build_id():
    """The build id of the loaded library (the digest of its sources)."""
    return load().zc_build_id().decode()
