"""GPU run of the zbackup-side binding: ZBackup::backupFromFileHandle's read
loop and iterative shrink passes (zutils.cc:89-182) driving
integration/gpu_backup_creator.hh (tests/adapter/adapter_main, built in-tree
by __graft_entry__.build()) against a repository index, compared with the
same loops over the oracle: the final backup data, the shrink iterations and
every Writer::add, in order.  The shrink passes run on the same index, so
they match the chunks the passes before them wrote (chunk_storage.cc:31-46)."""
import os
import subprocess
import struct

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "adapter", "adapter_main")


def _expected(data, W, seeds):
    from zbackup_amd.chunker import chunk_id_blob, serialize_instruction
    index = list(seeds)
    adds = []

    def one_pass(buf):
        out = bytearray()
        for (k, off, size, h, sha) in oracle.chunk(buf, W, seeds=index):
            if k == "B":
                out += serialize_instruction(raw=buf[off:off + size].tobytes())
                continue
            blob = chunk_id_blob(bytes.fromhex(sha), h)
            if k == "N":  # saveChunkToSave -> Writer::add -> ChunkIndex::addChunk
                adds.append(blob)
                index.append((bytes.fromhex(sha), h, size))
            out += serialize_instruction(chunk_blob=blob)
        return bytes(out)

    serialized = one_pass(data)
    it = 0
    while True:
        new = one_pass(np.frombuffer(serialized, dtype=np.uint8))
        if len(new) < len(serialized):
            serialized, it = new, it + 1
        else:
            break
    return serialized, it, adds, index


@pytest.mark.parametrize("W,spec,seed_spec", [
    (65536, "R1:20000000,C100:3000000,Z:500000,R2:5000000,C7000000:2000000", "R1:4000000"),
    (4096, "R3:3000000,C5:700000,B9:20000,R4:100000", ""),
])
def test_adapter_backup_vs_oracle_loops(tmp_path, W, spec, seed_spec):
    if not os.path.exists(BIN):
        pytest.fail("tests/adapter/adapter_main not built (run __graft_entry__.build())")
    data = oracle.gen(spec)
    seeds = []
    if seed_spec:
        seeds = [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in oracle.chunk(oracle.gen(seed_spec), W)
                 if k == "N"]
    inp = tmp_path / "in.bin"
    data.tofile(inp)
    sf = "-"
    if seeds:
        sf = str(tmp_path / "seeds.bin")
        with open(sf, "wb") as f:
            for sha, h, s in seeds:
                f.write(sha + struct.pack("<QII", h, s, 0))
    out = str(tmp_path / "out")
    r = subprocess.run([BIN, str(W), str(inp), sf, out], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    want_data, want_it, want_adds, _ = _expected(data, W, seeds)
    with open(out + ".meta") as f:
        it, nadds = map(int, f.read().split()[:2])
    with open(out + ".data", "rb") as f:
        got = f.read()
    with open(out + ".adds", "rb") as f:
        adds = f.read()
    assert it == want_it and it >= 1
    assert got == want_data
    assert nadds == len(want_adds) and adds == b"".join(want_adds)


def _run_adapter(tmp_path, tag, W, data, seeds, meta_dir):
    inp = tmp_path / f"{tag}.bin"
    data.tofile(inp)
    sf = "-"
    if seeds:
        sf = str(tmp_path / f"{tag}.seeds")
        with open(sf, "wb") as f:
            for sha, h, s in seeds:
                f.write(sha + struct.pack("<QII", h, s, 0))
    out = str(tmp_path / tag)
    r = subprocess.run([BIN, str(W), str(inp), sf, out, str(meta_dir)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    with open(out + ".meta") as f:
        it, nadds, hist_seeded, by_value = map(int, f.read().split())
    with open(out + ".data", "rb") as f:
        got = f.read()
    with open(out + ".adds", "rb") as f:
        adds = f.read()
    return got, it, adds, nadds, hist_seeded, by_value


@pytest.mark.parametrize("W", [65536, 4096])
def test_adapter_chunk_meta_sidecar_across_backups(tmp_path, W):
    # backup 1 into an empty repository writes its chunk-metadata file; backup 2
    # (a new process: the index = backup 1's Writer::add ids) reads it, so its
    # W-byte ids are seeded with their anchors; both backups' data, shrink
    # iterations and Writer::adds equal the oracle loops'.  A damaged file is
    # ignored (its ids are screened by key): the same backup either way.
    if not os.path.exists(BIN):
        pytest.fail("tests/adapter/adapter_main not built (run __graft_entry__.build())")
    meta_dir = tmp_path / "zchunk"
    a = oracle.gen("R41:9000000,C100:700000,Z:300000,R42:1000000")
    got, it, adds, nadds, hs, bv = _run_adapter(tmp_path, "b1", W, a, [], meta_dir)
    want_data, want_it, want_adds, seeds = _expected(a, W, [])
    assert (got, it, adds) == (want_data, want_it, b"".join(want_adds)) and hs == 0
    files = sorted(os.listdir(meta_dir))
    assert len(files) == 1 and len(files[0]) == 64
    # the repository's index after backup 1: every Writer::add (backup and shrink passes)
    b = np.concatenate([a[:3_000_000], a[3_000_013:8_000_000], oracle.gen("R43:777"), a[8_000_000:]])
    want_data, want_it, want_adds, _ = _expected(b, W, seeds)
    got, it, adds, nadds, hs, bv = _run_adapter(tmp_path, "b2", W, b, seeds, meta_dir)
    assert hs > 0.9 * sum(1 for s in seeds if s[2] == W)  # found by anchors, not screened by key
    assert (got, it, adds) == (want_data, want_it, b"".join(want_adds))
    assert len(os.listdir(meta_dir)) == 2
    # damage backup 1's file: it is skipped, the ids go by value, the backup is the same
    p = meta_dir / files[0]
    raw = bytearray(p.read_bytes())
    raw[100] ^= 0xFF
    p.write_bytes(bytes(raw))
    got, it, adds, nadds, hs, bv = _run_adapter(tmp_path, "b3", W, b, seeds, tmp_path / "zchunk")
    assert hs == 0 or hs < 0.5 * len(seeds)
    assert (got, it, adds) == (want_data, want_it, b"".join(want_adds))
