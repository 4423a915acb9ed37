"""Full-size parity: the three single-GPU BASELINE.json configs (C2 8 GiB random,
C3 two copies of 4 GiB, C5 8 GiB zeros) chunked with SHA-1 chunk ids and in the
benched mode (rolling-hash ids), and EVERY record (offset, size, kind, 64-bit
rolling hash, SHA-1 prefix) compared with a full oracle run over the same
8 GiB (backup_creator.cc:56-172,242-265, chunk_id.cc:19-27); then an
incremental backup at that size: the C2 stream edited (a grid shift every
MiB) against the index of its first backup, on the same context and on a
fresh one seeded with the exported anchor metadata.  The oracle runs on a host thread while the GPU chunks
(ctypes releases the GIL); it uses its exact key prefilter (identical
records, faster misses: oracle/zc_oracle.cpp ProbeSet)."""
import threading

import numpy as np
import pytest

from oracle import oracle

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

W64 = 65536
N = 8 << 30


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from zbackup_amd import _build
    _build.build()
    oracle.build()
    return torch


@pytest.fixture(scope="module")
def big(torch_cuda):
    t = torch_cuda.empty(N, dtype=torch_cuda.uint8, device="cuda")
    yield t
    del t
    torch_cuda.cuda.empty_cache()


def _same(got, want, sha1=True, what=""):
    assert len(got) == len(want), (what, len(got), len(want))
    for f in ("offset", "size", "kind", "rolling"):
        bad = np.nonzero(got[f] != want[f])[0]
        assert bad.size == 0, f"{what}: {f} differs at {bad.size} records, first {bad[:4]}"
    if sha1:
        bad = np.nonzero((got["sha1"] != want["sha1"]).any(axis=1))[0]
        assert bad.size == 0, f"{what}: sha1 differs at {bad.size} records, first {bad[:4]}"
    else:  # rolling-hash ids: no SHA-1 prefix on chunk records
        assert not got["sha1"][got["kind"] != 2].any(), what


def _check_all_records(torch, t):
    """GPU vs the oracle over the whole buffer, every field of every record: with
    SHA-1 ids, and in the headline mode (rolling-hash ids, sha1=False: its
    windows are confirmed by bytes, not by key + SHA-1 joins)."""
    from zbackup_amd import BackupCreator
    host = t.cpu().numpy()
    box = {}

    def run_oracle():
        box["want"] = oracle.chunk_array(host, W64)

    th = threading.Thread(target=run_oracle)
    th.start()
    with BackupCreator(W64, sha1=True) as bc:
        bc.chunk_device(t.data_ptr(), t.numel())
        got = bc.records()
        # equal-key grid pairs (C3, C5) are joined speculatively by key and
        # confirmed by their digests: no stream is redone
        assert bc.stats()["respeculations"] == 0
    with BackupCreator(W64, sha1=False) as bc:
        bc.chunk_device(t.data_ptr(), t.numel())
        got_roll = bc.records()
    th.join()
    want = box["want"]
    _same(got, want, True, "sha1 ids")
    _same(got_roll, want, False, "rolling-hash ids")
    return got


@pytest.mark.timeout(900)
def test_c2_every_record_vs_oracle(torch_cuda, big):
    from zbackup_amd import fill_splitmix64
    fill_splitmix64(big.data_ptr(), N, 2024)
    got = _check_all_records(torch_cuda, big)
    assert len(got) == N // W64 and (got["kind"] == 0).all()


@pytest.mark.timeout(900)
def test_c3_every_record_vs_oracle(torch_cuda, big):
    from zbackup_amd import fill_splitmix64
    half = N // 2
    fill_splitmix64(big.data_ptr(), half, 2024)
    big[half:].copy_(big[:half])
    got = _check_all_records(torch_cuda, big)
    m = half // W64
    assert len(got) == 2 * m and (got["kind"][m:] == 1).all()


@pytest.mark.timeout(900)
def test_c5_every_record_vs_oracle(torch_cuda, big):
    big.zero_()
    got = _check_all_records(torch_cuda, big)
    assert got["kind"][0] == 0 and (got["kind"][1:] == 1).all()
    assert (got["rolling"] == 0x172AEAFF81000001).all()


def _edit_on_device(torch, src, n, seed):
    """src's bytes with 1-100 random bytes inserted every MiB, cut at n bytes
    (as bench.fill_edited does for the edited-duplicate config)."""
    rng = np.random.default_rng(seed)
    dst = torch.empty(n, dtype=torch.uint8, device=src.device)
    noise = torch.from_numpy(rng.integers(0, 256, 1 << 20, dtype=np.uint8)).to(src.device)
    pos = srcpos = 0
    piece = 1 << 20
    while pos < n:
        ln = min(piece, n - pos, src.numel() - srcpos)
        dst[pos:pos + ln].copy_(src[srcpos:srcpos + ln])
        pos += ln
        srcpos += ln
        k = min(int(rng.integers(1, 101)), n - pos)
        if k > 0:
            o = int(rng.integers(0, noise.numel() - 128))
            dst[pos:pos + k].copy_(noise[o:o + k])
            pos += k
    return dst


@pytest.mark.timeout(900)
def test_incremental_edited_every_record_vs_oracle(torch_cuda, big):
    # stream 1 = C2; stream 2 = stream 1 with an insertion every MiB (8,192 grid
    # shifts).  Stream 2 is backed up (a) on the context that backed up stream 1
    # (its chunks in the historic index) and (b) on a fresh context seeded with
    # stream 1's ids and exported anchor metadata -- both against the oracle
    # seeded with stream 1's ids (ChunkIndex::loadIndex of its index file)
    from zbackup_amd import BackupCreator, fill_splitmix64
    fill_splitmix64(big.data_ptr(), N, 2024)
    s2 = _edit_on_device(torch_cuda, big, N, 5)
    h2 = s2.cpu().numpy()
    with BackupCreator(W64, sha1=True) as a:
        a.chunk_device(big.data_ptr(), N)
        r1 = a.records()
        meta = a.export_chunk_meta()
        ids = r1[r1["kind"] == 0]
        seeds = [(bytes(r["sha1"]), int(r["rolling"]), int(r["size"])) for r in ids]
        box = {}
        th = threading.Thread(target=lambda: box.update(want=oracle.chunk_array(h2, W64, seeds=seeds)))
        th.start()
        a.chunk_device(s2.data_ptr(), N)
        got_a = a.records()
    with BackupCreator(W64, sha1=True) as b:
        b.seed_index_meta(ids["sha1"], ids["rolling"], ids["size"], meta)
        assert b.stats()["hist_seeded"] == len(meta)  # random bytes: every chunk has an anchor
        b.chunk_device(s2.data_ptr(), N)
        got_b = b.records()
    th.join()
    want = box["want"]
    assert int((want["kind"] == 1).sum()) > 100_000  # most windows are found again across the shifts
    _same(got_a, want, True, "same context")
    _same(got_b, want, True, "seeded context")
    del s2
