"""TEST INFRASTRUCTURE ONLY -- ctypes view of the CPU restatement (zc_oracle.cpp).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker.  The product (zbackup_amd) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

KIND_NEW, KIND_DUP, KIND_BYTES = 0, 1, 2
KIND_CHAR = "NDB"


class Record(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("size", ctypes.c_uint32),
                ("kind", ctypes.c_uint32), ("rolling", ctypes.c_uint64),
                ("sha1", ctypes.c_uint8 * 16)]


class Seed(ctypes.Structure):
    _fields_ = [("sha1", ctypes.c_uint8 * 16), ("rolling", ctypes.c_uint64),
                ("size", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


def build(ref=False):
    """Compile the oracle (and, with ref=True, the reference-built checkers)."""
    targets = ["all"] + (["ref"] if ref else [])
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


_LIBS = {}


def lib(ref=False):
    name = os.path.join(HERE, "_ref", "liboracle_ref.so") if ref else os.path.join(HERE, "liboracle.so")
    if name in _LIBS:
        return _LIBS[name]
    if not os.path.exists(name):
        build(ref=ref)
    L = ctypes.CDLL(name)
    L.zco_digest.restype = ctypes.c_uint64
    L.zco_digest.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    L.zco_chunk.restype = ctypes.c_int
    L.zco_chunk.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                            ctypes.c_size_t, ctypes.c_uint64, ctypes.POINTER(ctypes.POINTER(Record)),
                            ctypes.POINTER(ctypes.c_size_t)]
    L.zco_chunk_ex.restype = ctypes.c_int
    L.zco_chunk_ex.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                               ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32,
                               ctypes.POINTER(ctypes.POINTER(Record)), ctypes.POINTER(ctypes.c_size_t)]
    L.zco_free.argtypes = [ctypes.c_void_p]
    L.zco_sha1.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    L.zco_fill_splitmix64.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
    L.zco_gen.restype = ctypes.c_int
    L.zco_gen.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                          ctypes.POINTER(ctypes.c_uint64)]
    _LIBS[name] = L
    return L


def gen(spec, ref=False):
    """Synthetic stream from a spec string (grammar in zc_oracle.h) as uint8 numpy array."""
    L = lib(ref)
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_uint64()
    rc = L.zco_gen(spec.encode(), ctypes.byref(p), ctypes.byref(n))
    if rc:
        raise ValueError(f"bad spec {spec!r} ({rc})")
    arr = np.ctypeslib.as_array(p, shape=(max(n.value, 1),))[: n.value].copy()
    L.zco_free(p)
    return arr


def splitmix64(n, seed):
    out = np.empty(n, dtype=np.uint8)
    lib().zco_fill_splitmix64(out.ctypes.data, n, seed)
    return out


def digest(data):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    return int(lib().zco_digest(data.ctypes.data, data.size))


def sha1(data):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = (ctypes.c_uint8 * 20)()
    lib().zco_sha1(data.ctypes.data, data.size, out)
    return bytes(out)


def chunk(data, W, seeds=(), feed_max=0, ref=False):
    """Run the restated BackupCreator over `data`; returns a list of record tuples
    (kind_char, offset, size, rolling, sha1_16_hex)."""
    L = lib(ref)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    seed_arr = (Seed * max(len(seeds), 1))()
    for i, (sha16, rolling, size) in enumerate(seeds):
        seed_arr[i].sha1[:] = list(sha16)
        seed_arr[i].rolling = rolling
        seed_arr[i].size = size
    out = ctypes.POINTER(Record)()
    nout = ctypes.c_size_t()
    rc = L.zco_chunk(data.ctypes.data, data.size, W, seed_arr, len(seeds), feed_max,
                     ctypes.byref(out), ctypes.byref(nout))
    if rc:
        raise RuntimeError(f"zco_chunk failed: {rc}")
    recs = []
    for i in range(nout.value):
        r = out[i]
        recs.append((KIND_CHAR[r.kind], r.offset, r.size, r.rolling, bytes(r.sha1).hex()))
    L.zco_free(out)
    return recs


RECORD_DTYPE = np.dtype([("offset", "<u8"), ("size", "<u4"), ("kind", "<u4"),
                         ("rolling", "<u8"), ("sha1", "u1", (16,))])
OPT_PREFILTER = 1


SEED_DTYPE = np.dtype([("sha1", np.uint8, 16), ("rolling", "<u8"), ("size", "<u4"), ("pad", "<u4")])


def seed_array(seeds):
    """Seeds as a SEED_DTYPE array (laid out like Seed): a list of (sha1_16,
    rolling, size) tuples, or such an array already (passed through)."""
    if isinstance(seeds, np.ndarray):
        return np.ascontiguousarray(seeds, dtype=SEED_DTYPE)
    seeds = list(seeds)
    out = np.zeros(len(seeds), dtype=SEED_DTYPE)
    if seeds:
        out["sha1"] = np.frombuffer(b"".join(bytes(sha16)[:16] for sha16, _, _ in seeds),
                                    dtype=np.uint8).reshape(-1, 16)
        out["rolling"] = np.array([rolling for _, rolling, _ in seeds], dtype=np.uint64)
        out["size"] = np.array([size for _, _, size in seeds], dtype=np.uint32)
    return out


def chunk_array(data, W, seeds=(), prefilter=True):
    """The same run as chunk(), returned as a numpy structured array laid out
    like zc_record (for full-size comparisons).  prefilter=True puts an exact
    key bitmap in front of the hash_map: identical records, faster misses.
    seeds: (sha1_16, rolling, size) tuples or a SEED_DTYPE array."""
    L = lib()
    data = np.ascontiguousarray(data, dtype=np.uint8)
    sa = seed_array(seeds)
    assert SEED_DTYPE.itemsize == ctypes.sizeof(Seed)
    seed_arr = (Seed * max(len(sa), 1)).from_buffer(sa) if len(sa) else (Seed * 1)()
    out = ctypes.POINTER(Record)()
    nout = ctypes.c_size_t()
    rc = L.zco_chunk_ex(data.ctypes.data, data.size, W, seed_arr, len(sa), 0,
                        OPT_PREFILTER if prefilter else 0, ctypes.byref(out), ctypes.byref(nout))
    if rc:
        raise RuntimeError(f"zco_chunk_ex failed: {rc}")
    n = nout.value
    res = np.empty(n, dtype=RECORD_DTYPE)
    if n:
        ctypes.memmove(res.ctypes.data, out, n * RECORD_DTYPE.itemsize)
    L.zco_free(out)
    return res


def format_records(recs):
    return [f"{k} {o} {s} {h:016x} {sha}" for (k, o, s, h, sha) in recs]
