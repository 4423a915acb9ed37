"""Bundle-writer oracle (TEST INFRASTRUCTURE ONLY: imported by tests/, smoke()
and bench.py's cpu_baseline leg as the checker, never by the product).

* lzo1x_1 compression: the real third-party library zbackup calls,
  liblzo2 2.10 (`lzo1x_1_compress`, compression.cc:586-606), loaded from the
  image (/opt/conda/lib/liblzo2.so.2; not part of the reference tree), with
  zbackup's framing restated from NoStreamAndUnknownSizeEncoder::doProcess
  (compression.cc:435-466).  Parity pinned by the library itself.
* The bundling rule of ChunkStorage::Writer::add (chunk_storage.cc:31-46)
  together with ChunkIndex::addChunk's "only ids not yet in the index"
  (chunk_index.cc:163-202), restated.
"""
import ctypes
import os
import struct

LZO_PATHS = ("/opt/conda/lib/liblzo2.so.2", "liblzo2.so.2")
LZO1X_1_MEM_COMPRESS = 16384 * 4  # lzo1x.h: 16384 * lzo_sizeof_dict_t (room for pointer-sized entries)

_lzo = None


def lzo_lib():
    """liblzo2, or None when the image lacks it."""
    global _lzo
    if _lzo is None:
        for p in LZO_PATHS:
            if os.path.isabs(p) and not os.path.exists(p):
                continue
            try:
                L = ctypes.CDLL(p)
            except OSError:
                continue
            L.__lzo_init_v2.restype = ctypes.c_int
            # lzo_init() = __lzo_init_v2(LZO_VERSION, sizeof(short), sizeof(int), sizeof(long),
            #   sizeof(lzo_uint32_t), sizeof(lzo_uint), lzo_sizeof_dict_t, sizeof(char*),
            #   sizeof(lzo_voidp), sizeof(lzo_callback_t))  (lzoconf.h)
            rc = L.__lzo_init_v2(ctypes.c_uint(0x20a0), 2, 4, 8, 4, 8, 8, 8, 8, 48)
            if rc != 0:
                raise RuntimeError(f"lzo_init failed ({rc})")
            _lzo = L
            break
    return _lzo


def lzo1x_1(data):
    """lzo1x_1_compress(data) -> the raw LZO stream."""
    L = lzo_lib()
    n = len(data)
    out = ctypes.create_string_buffer(n + n // 16 + 64 + 3)
    olen = ctypes.c_size_t(len(out))
    wrk = ctypes.create_string_buffer(LZO1X_1_MEM_COMPRESS * 2)
    src = ctypes.create_string_buffer(bytes(data), n) if n else ctypes.create_string_buffer(1)
    rc = L.lzo1x_1_compress(src, ctypes.c_size_t(n), out, ctypes.byref(olen), wrk)
    if rc != 0:
        raise RuntimeError(f"lzo1x_1_compress failed ({rc})")
    return out.raw[:olen.value]


def lzo1x_decompress(stream, n):
    """lzo1x_decompress_safe: the raw stream back to its n bytes."""
    L = lzo_lib()
    out = ctypes.create_string_buffer(max(n, 1))
    olen = ctypes.c_size_t(n)
    src = ctypes.create_string_buffer(bytes(stream), len(stream))
    rc = L.lzo1x_decompress_safe(src, ctypes.c_size_t(len(stream)), out, ctypes.byref(olen), None)
    if rc != 0 or olen.value != n:
        raise RuntimeError(f"lzo1x_decompress_safe failed ({rc}, {olen.value} of {n} bytes)")
    return out.raw[:n]


def frame(payload):
    """The bytes LZO1X_1_Encoder writes for one bundle payload: the template
    "ABCDEFGHIJKLMNOP" with LE32 size at 0 and LE32 compressed size at 8
    (compression.cc:443-460), then the LZO stream."""
    z = lzo1x_1(payload)
    head = bytearray(b"ABCDEFGHIJKLMNOP")
    head[0:4] = struct.pack("<I", len(payload))
    head[8:12] = struct.pack("<I", len(z))
    return bytes(head) + z


def unframe(framed):
    """NoStreamAndUnknownSizeDecoder's view: the payload back."""
    n, = struct.unpack_from("<I", framed, 0)
    cz, = struct.unpack_from("<I", framed, 8)
    return lzo1x_decompress(framed[16:16 + cz], n)


def writer_bundles(chunks, max_payload=0x200000, index=None):
    """ChunkStorage::Writer::add over (id, size) chunks in stream order: a chunk
    whose id the index already holds is not stored; a stored chunk finishes the
    current bundle first when payload + size > max_payload.  Returns the list of
    bundles, each a list of chunk positions (into `chunks`)."""
    index = set() if index is None else index
    bundles = []
    cur = None
    payload = 0
    for i, (cid, size) in enumerate(chunks):
        if cid in index:  # ChunkIndex::addChunk returns false
            continue
        index.add(cid)
        if cur is None:  # getCurrentBundle() creates one before the size test
            cur, payload = [], 0
        if payload + size > max_payload:
            bundles.append(cur)
            cur, payload = [], 0
        cur.append(i)
        payload += size
    if cur is not None:
        bundles.append(cur)
    return bundles
