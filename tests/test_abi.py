"""CPU tests of the drop-in boundary: the C-ABI library builds, loads and exports
every symbol include/zchunk.h declares (no compute calls without a GPU), and
the host-side serializer matches the reference's wire format."""
import os
import re
import struct
import subprocess

import pytest

from zbackup_amd import _build, _lib
from zbackup_amd.chunker import chunk_id_blob, serialize_instruction

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "zchunk.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zc_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    _build.build()
    return _lib.load()


def test_header_declares_the_binding(lib):
    assert declared_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (zc_[a-z0-9_]+)", out))
    missing = set(declared_functions()) - exported
    assert not missing, missing


def test_abi_version_and_argument_errors(lib):
    import ctypes
    assert lib.zc_abi_version() == 5
    ctx = ctypes.c_void_p()
    assert lib.zc_create(None, 65536, 0, 0) == _lib.ZC_ERR_ARG
    assert lib.zc_create(ctypes.byref(ctx), 0, 0, 0) == _lib.ZC_ERR_ARG  # chunk.max_size 0
    assert lib.zc_destroy(None) == _lib.ZC_ERR_ARG
    assert lib.zc_record_count(None) == 0
    assert lib.zc_last_error(None) == b"null context"


def test_record_layout_matches_header():
    import ctypes
    assert ctypes.sizeof(_lib.ZcRecord) == 40
    assert ctypes.sizeof(_lib.ZcSeed) == 32
    assert ctypes.sizeof(_lib.ZcChunkMeta) == 48
    from zbackup_amd.chunker import META_DTYPE, RECORD_DTYPE, SEED_DTYPE
    assert RECORD_DTYPE.itemsize == 40
    assert SEED_DTYPE.itemsize == 32
    assert META_DTYPE.itemsize == 48
    for name, _ in _lib.ZcChunkMeta._fields_:
        assert META_DTYPE.fields[name][1] == getattr(_lib.ZcChunkMeta, name).offset, name


def test_chunk_meta_calls_without_a_gpu(lib):
    """The ABI-5 index-metadata entry points: argument errors and the anchor
    definition need no device (no context is made)."""
    import ctypes
    n = ctypes.c_size_t()
    assert lib.zc_export_chunk_meta(None, None, 0, ctypes.byref(n)) == _lib.ZC_ERR_ARG
    assert lib.zc_seed_index_meta(None, None, 0, None, 0) == _lib.ZC_ERR_ARG
    d64, d4k = lib.zc_anchor_def(65536), lib.zc_anchor_def(4096)
    assert d64 >> 16 == 0x5A41 and d64 & 0xFF == 12  # anchors at 1 in 4096 positions for W = 64 KiB
    assert d4k != d64 and d4k & 0xFF == 8            # 1 in 256 for W = 4 KiB (~16 per chunk)
    assert lib.zc_anchor_def(0) == 0


def test_chunk_id_blob_and_framing():
    # ChunkId::toBlob = sha1[0:16] || little-endian rolling (chunk_id.cc:19-27);
    # Message::serialize = varint32(len) + BackupInstruction (message.cc:16-23)
    sha = bytes(range(16))
    blob = chunk_id_blob(sha, 0x172AEAFF81000001)
    assert blob == sha + struct.pack("<Q", 0x172AEAFF81000001)
    msg = serialize_instruction(chunk_blob=blob)
    assert msg == bytes([26, 0x0A, 24]) + blob  # 27 bytes per chunk record
    raw = b"x" * 200
    msg = serialize_instruction(raw=raw)
    assert msg[:4] == bytes([203, 1, 0x12, 200 | 0x80]) and msg[4] == 1 and msg[5:] == raw


def test_clean_tree_compiles(tmp_path):
    """The checked-out sources compile and link (into a temp dir, so a stale
    in-tree binary cannot hide a tree that does not build)."""
    out = str(tmp_path / "libzchunk.so")
    _build.build(force=True, out=out)
    assert _build.lib_build_id(out) == _build.source_digest()


def test_in_tree_library_is_built_from_these_sources(lib):
    """bench.py, smoke() and the GPU tests load the in-tree library; it must
    carry the digest of the checked-out sources."""
    assert _build.lib_build_id() == _build.source_digest()
    assert _lib.build_id() == _build.source_digest()
