"""Bundle writer offload: the host mirror of the reference's bundle path.

  ChunkStorage::Writer::add -> bundling rule          chunk_storage.cc:31-46
  Bundle::Creator::addChunk -> payload assembly       bundle.cc:30-36
  Bundle::Creator::write    -> lzo1x_1 compression    bundle.cc:120-151,
                               framing                compression.cc:435-466, 586-606

`plan_bundles` is host bookkeeping; `BundleCompressor.gather` and `.compress`
run on the GPU through libzchunk.so (zc_bundle_gather / zc_lzo_compress);
there is no CPU fallback.  Device buffers are passed as raw pointers (e.g. a
torch uint8 tensor's data_ptr()).
"""
import ctypes

import numpy as np

from . import _lib
from .chunker import _check

MAX_PAYLOAD_SIZE = 0x200000  # bundle.max_payload_size default, zbackup.proto:88


def _u64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


def plan_bundles(sizes, max_payload=MAX_PAYLOAD_SIZE):
    """Writer::add's rule over the sizes of the chunks index.addChunk accepted,
    in order: returns (bundle index of each chunk, number of bundles)."""
    L = _lib.load()
    sizes = _u64(sizes)
    out = np.zeros(len(sizes), dtype=np.uint32)
    nb = ctypes.c_size_t()
    rc = L.zc_bundle_plan(sizes.ctypes.data, len(sizes), int(max_payload), out.ctypes.data, ctypes.byref(nb))
    _check(L, None, rc, "zc_bundle_plan")
    return out, nb.value


def lzo_capacity(payload_size):
    """Output bytes to reserve for one framed payload (suggestOutputSize + 16)."""
    return int(_lib.load().zc_lzo_capacity(int(payload_size)))


class BundleCompressor:
    """GPU payload assembly + lzo1x_1 compression on a context of its own
    (or on a BackupCreator's, `ctx=bc._ctx`)."""

    def __init__(self, device=0, ctx=None):
        self._L = _lib.load()
        self._own = ctx is None
        if ctx is None:
            ctx = ctypes.c_void_p()
            rc = self._L.zc_create(ctypes.byref(ctx), 65536, device, 0)
            if rc != _lib.ZC_OK:
                raise _lib.ZcError(f"zc_create failed ({rc})")
        self._ctx = ctx

    def gather(self, d_src, src_off, sizes, d_payload):
        """Bundle::Creator::addChunk for every chunk: d_payload <- the extents
        d_src[src_off[i] ..+ sizes[i]) back to back."""
        src_off, sizes = _u64(src_off), _u64(sizes)
        rc = self._L.zc_bundle_gather(self._ctx, d_src, src_off.ctypes.data, sizes.ctypes.data, len(sizes), d_payload)
        _check(self._L, self._ctx, rc, "zc_bundle_gather")

    def compress(self, d_payload, pay_off, pay_size, d_out, out_off):
        """Framed lzo1x_1 of payload i to d_out + out_off[i]; returns the framed sizes."""
        pay_off, pay_size, out_off = _u64(pay_off), _u64(pay_size), _u64(out_off)
        out_size = np.zeros(len(pay_size), dtype=np.uint64)
        rc = self._L.zc_lzo_compress(self._ctx, d_payload, pay_off.ctypes.data, pay_size.ctypes.data, len(pay_size),
                                     d_out, out_off.ctypes.data, out_size.ctypes.data)
        _check(self._L, self._ctx, rc, "zc_lzo_compress")
        return out_size

    def compress_host(self, payloads):
        """Host bytes in, framed bytes out (zc_lzo_compress_host), one call for all."""
        payloads = [bytes(p) for p in payloads]
        sizes = np.array([len(p) for p in payloads], dtype=np.uint64)
        pay_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64) if len(sizes) else sizes
        caps = np.array([lzo_capacity(int(s)) for s in sizes], dtype=np.uint64)
        out_off = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.uint64) if len(caps) else caps
        src = np.frombuffer(b"".join(payloads) or b"\0", dtype=np.uint8)
        out = np.zeros(int(caps.sum()) or 1, dtype=np.uint8)
        out_size = np.zeros(len(sizes), dtype=np.uint64)
        rc = self._L.zc_lzo_compress_host(self._ctx, src.ctypes.data, pay_off.ctypes.data, sizes.ctypes.data,
                                          len(sizes), out.ctypes.data, out_off.ctypes.data, out_size.ctypes.data)
        _check(self._L, self._ctx, rc, "zc_lzo_compress_host")
        return [out[int(o):int(o) + int(s)].tobytes() for o, s in zip(out_off, out_size)]

    def adler32(self, d_base, off, length):
        """zlib adler32 (from 1) of each device range d_base[off[i] ..+ length[i])."""
        off, length = _u64(off), _u64(length)
        out = np.zeros(len(off), dtype=np.uint32)
        rc = self._L.zc_adler32(self._ctx, d_base, off.ctypes.data, length.ctypes.data, len(off), out.ctypes.data)
        _check(self._L, self._ctx, rc, "zc_adler32")
        return out

    def last_stats(self):
        """(parse kernel ms, 48 KiB blocks) of the last compress()."""
        ms, blocks = ctypes.c_double(), ctypes.c_uint64()
        self._L.zc_lzo_last_stats(self._ctx, ctypes.byref(ms), ctypes.byref(blocks))
        return ms.value, blocks.value

    def close(self):
        if self._own and self._ctx:
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
