"""The zbackup-side binding (integration/gpu_backup_creator.hh) compiles
against include/zchunk.h: the zutils.cc loops of tests/adapter/adapter_main.cpp
over the adapter, built with -Wall -Werror and linked to libzchunk.so (CPU
only: nothing runs on a GPU here)."""
import os

import pytest

from tests.adapter import build as adapter_build


def test_adapter_compiles_and_links(tmp_path):
    from zbackup_amd import _build
    _build.build()
    out = adapter_build.build(str(tmp_path / "adapter_main"))
    assert os.path.getsize(out) > 0


def _sidecar_bytes(entries):
    """A chunk-metadata file as GpuChunkMetaSidecar::write lays it out: "ZCMETA01",
    LE32 48, LE32 0, LE64 count, the 48-byte zc_chunk_meta records, SHA-256."""
    import hashlib
    import struct
    body = b"ZCMETA01" + struct.pack("<IIQ", 48, 0, len(entries))
    for sha, rolling, size, adef, anchor, gear, fp in entries:
        body += bytes(sha) + struct.pack("<QIIIIQ", rolling, size, adef, anchor, gear, fp)
    return body + hashlib.sha256(body).digest()


def test_chunk_meta_sidecar_files_read_back(tmp_path):
    """The adapter's chunk-metadata files (integration/gpu_backup_creator.hh,
    GpuChunkMetaSidecar): valid files are read whole, a damaged one (a flipped
    byte: the SHA-256 no longer matches), a truncated one and files with other
    names are skipped -- metadata only speeds matching up, so a bad file may
    cost speed, never change a backup (CPU only: no context is made)."""
    import subprocess
    from tests.adapter import build as adapter_build
    from zbackup_amd import _build
    _build.build()
    exe = adapter_build.build_sidecar_reader(str(tmp_path / "sidecar_read"))
    d = tmp_path / "zchunk"
    d.mkdir()
    a = [(bytes([i] * 16), 0x1000 + i, 65536, 0x5A41020C, 100 + i, 0x7FF00000 | i, 0xABCD0000 + i) for i in range(5)]
    b = [(bytes([0x80 + i] * 16), 0x2000 + i, 65536, 0x5A41020C, 200 + i, 0x7FF10000 | i, 0xDCBA0000 + i)
         for i in range(3)]
    good_a, good_b = _sidecar_bytes(a), _sidecar_bytes(b)
    (d / ("a" * 64)).write_bytes(good_a)
    (d / ("b" * 64)).write_bytes(good_b)
    bad = bytearray(_sidecar_bytes(a))
    bad[40] ^= 1
    (d / ("c" * 64)).write_bytes(bytes(bad))
    (d / ("d" * 64)).write_bytes(good_a[:-7])
    (d / "notes.txt").write_bytes(good_a)
    (d / ("e" * 64 + ".tmp")).write_bytes(good_a)
    out = subprocess.run([exe, str(d)], capture_output=True, text=True, check=True).stdout.split("\n")
    assert int(out[0]) == 8
    got = sorted(tuple(x.split()) for x in out[1:] if x)
    want = sorted((f"{r:016x}", str(anc)) for (_, r, _, _, anc, _, _) in a + b)
    assert got == want
