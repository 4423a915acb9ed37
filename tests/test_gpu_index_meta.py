"""GPU parity of a non-empty repository seeded with content-anchor metadata
(ABI 5: zc_export_chunk_meta / zc_seed_index_meta).

zbackup opens a repository by reading every id of its index files
(ChunkIndex::loadIndex, chunk_index.cc:26-79, driven by zbackup_base.cc:87-100).
Ids alone reach the engine's by-value screen (an exact key test at every
byte); ids seeded with the metadata an earlier context exported join the
historic index and are found by their first content anchor.  Either way a
window matches only when its rolling key and SHA-1 prefix equal an indexed
id's (ChunkIndex::findChunk, chunk_index.cc:119-143), so the records must equal
the oracle's run seeded with the same ids -- whatever metadata came with them:
missing, of another anchor definition, or for ids that are not in the index.
"""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

W64 = 65536


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from zbackup_amd import _build
    _build.build()
    oracle.build()
    return torch


def _edited(base, seed, every=1 << 20):
    """base with 1-100 random bytes inserted every `every` bytes (a grid shift each)."""
    rng = np.random.default_rng(seed)
    out, pos = [], 0
    while pos < base.size:
        out.append(base[pos:pos + every])
        out.append(rng.integers(0, 256, int(rng.integers(1, 101)), dtype=np.uint8))
        pos += every
    return np.concatenate(out)


def _ids(recs):
    """index ids (sha1_16, rolling, size) of a record array's NEW chunks."""
    sel = recs[recs["kind"] == 0]
    return sel


def _seed_tuples(sel):
    return [(bytes(r["sha1"]), int(r["rolling"]), int(r["size"])) for r in sel]


def _first_backup(torch, data, W):
    """A context's first backup of `data` (SHA-1 ids): its records and the
    metadata of the W-byte chunks it added to the index."""
    from zbackup_amd import BackupCreator
    t = torch.from_numpy(np.ascontiguousarray(data)).to("cuda")
    with BackupCreator(W, sha1=True) as bc:
        bc.chunk_device(t.data_ptr(), data.size)
        recs = bc.records()
        meta = bc.export_chunk_meta()
        st = bc.stats()
    assert len(meta) == st["hist_entries"]
    return recs, meta


def _run(torch, data, W, ids, meta, path="device", sha1=True, window=1):
    from zbackup_amd import BackupCreator
    with BackupCreator(W, sha1=sha1, window=window if path == "window" else None) as bc:
        bc.seed_index_meta(ids["sha1"], ids["rolling"], ids["size"], meta)
        st0 = bc.stats()
        if path == "device":
            t = torch.from_numpy(np.ascontiguousarray(data)).to("cuda")
            bc.chunk_device(t.data_ptr(), data.size)
        else:
            bc.feed(data)
            bc.finish()
        return bc.record_tuples(), st0, bc.stats()


def _strip_sha(recs):
    return [(k, o, s, h, "0" * 32 if k != "B" else sha) for (k, o, s, h, sha) in recs]


A_SPEC = "R5:24000000,C100:3000000,Z:1000000,R6:2000000,C9000000:700001,B9:300000,R7:99999"


@pytest.mark.parametrize("W", [4096, W64])
@pytest.mark.parametrize("path", ["device", "window"])
def test_seeded_meta_same_stream_vs_oracle(torch_cuda, W, path):
    a = oracle.gen(A_SPEC)
    recs, meta = _first_backup(torch_cuda, a, W)
    ids = _ids(recs)
    anchored = int((meta["anchor"] != 0xFFFFFFFF).sum())
    assert anchored > 0.9 * len(meta)  # random bytes: nearly every chunk has an anchor
    want = oracle.chunk(a, W, seeds=_seed_tuples(ids))
    got, st0, st = _run(torch_cuda, a, W, ids, meta, path)
    assert st0["hist_seeded"] == anchored
    # the W-byte ids without metadata (anchorless: zero and one-byte runs) go by value
    assert st0["by_value"] == int((ids["size"] == W).sum()) - anchored
    assert got == want
    # the repeat of an indexed stream: every W-byte window on the grid is a duplicate
    assert sum(1 for r in got if r[0] == "D") >= len(meta) - 2


@pytest.mark.parametrize("W", [4096, W64])
def test_seeded_meta_edited_copy_vs_oracle(torch_cuda, W):
    a = oracle.gen(A_SPEC)
    b = _edited(a, 77, every=(1 << 20) if W == W64 else 150_001)
    recs, meta = _first_backup(torch_cuda, a, W)
    ids = _ids(recs)
    want = oracle.chunk(b, W, seeds=_seed_tuples(ids))
    assert sum(1 for r in want if r[0] == "D") > 0.5 * len(meta)  # shifted windows match
    for path in ("device", "window"):
        got, _, _ = _run(torch_cuda, b, W, ids, meta, path)
        assert got == want, path


@pytest.mark.parametrize("W", [4096, W64])
def test_seeded_meta_some_ids_without_metadata(torch_cuda, W):
    # a repository partly written by stock zbackup: a third of the ids have no
    # metadata, a sixth carry another anchor definition (ignored): both go by value
    a = oracle.gen(A_SPEC)
    b = _edited(a, 78, every=(1 << 20) if W == W64 else 150_001)
    recs, meta = _first_backup(torch_cuda, a, W)
    ids = _ids(recs)
    keep = np.ones(len(meta), bool)
    keep[::3] = False
    meta2 = meta[keep].copy()
    meta2["anchor_def"][::2] ^= 0x100
    want = oracle.chunk(b, W, seeds=_seed_tuples(ids))
    got, st0, _ = _run(torch_cuda, b, W, ids, meta2, "device")
    usable = int(((meta2["anchor"] != 0xFFFFFFFF) & (meta2["anchor_def"] == meta["anchor_def"][0])).sum())
    assert st0["hist_seeded"] == usable
    assert got == want


@pytest.mark.parametrize("W", [4096, W64])
def test_meta_for_ids_not_in_the_index_never_matches(torch_cuda, W):
    # metadata of every chunk, ids of only every other one: windows equal to the
    # chunks left out of the index must not match (findChunk has no such id)
    a = oracle.gen(A_SPEC)
    recs, meta = _first_backup(torch_cuda, a, W)
    ids = _ids(recs)
    half = ids[::2]
    want = oracle.chunk(a, W, seeds=_seed_tuples(half))
    got, st0, _ = _run(torch_cuda, a, W, half, meta, "device")
    assert st0["hist_seeded"] <= (len(meta) + 1) // 2 + 1
    assert got == want
    assert [r for r in got if r[0] == "N" and r[2] == W]  # the left-out chunks are saved again


def test_seeded_meta_rolling_hash_ids(torch_cuda):
    # the headline mode (no SHA-1 ids on the records): historic windows are
    # still confirmed by key + SHA-1 (computed per candidate window)
    W = W64
    a = oracle.gen(A_SPEC)
    b = _edited(a, 79)
    recs, meta = _first_backup(torch_cuda, a, W)
    ids = _ids(recs)
    want = oracle.chunk(b, W, seeds=_seed_tuples(ids))
    got, _, _ = _run(torch_cuda, b, W, ids, meta, "device", sha1=False)
    assert got == _strip_sha(want)


def test_seeding_order_and_forget(torch_cuda):
    from zbackup_amd import BackupCreator, ZcError
    W = W64
    a = oracle.gen(A_SPEC)
    c = oracle.gen("R31:6000000,C17:2000000")
    recs, meta = _first_backup(torch_cuda, a, W)
    ids = _ids(recs)
    want_a = oracle.chunk(a, W, seeds=_seed_tuples(ids))
    ta = torch_cuda.from_numpy(a).to("cuda")
    tc = torch_cuda.from_numpy(c).to("cuda")
    with BackupCreator(W, sha1=True) as bc:
        bc.seed_index_meta(ids["sha1"], ids["rolling"], ids["size"], meta)
        seeded = bc.stats()["hist_seeded"]
        # seeding the same ids again adds nothing (registerNewChunkId: unless present)
        bc.seed_index_meta(ids["sha1"], ids["rolling"], ids["size"], meta)
        assert bc.stats()["hist_seeded"] == seeded
        bc.chunk_device(tc.data_ptr(), c.size)  # adds its own chunks to the index
        assert bc.stats()["hist_entries"] > seeded
        with pytest.raises(ZcError):
            bc.seed_index_meta(ids["sha1"], ids["rolling"], ids["size"], meta)
        assert len(bc.export_chunk_meta()) == bc.stats()["hist_entries"] - seeded
        bc.forget_stream_chunks()  # back to the seeded index, metadata included
        assert bc.stats()["hist_entries"] == seeded
        assert len(bc.export_chunk_meta()) == 0
        bc.chunk_device(ta.data_ptr(), a.size)
        assert bc.record_tuples() == want_a
        bc.forget_stream_chunks()
        bc.seed_index_meta(ids["sha1"][:0], ids["rolling"][:0], W, meta[:0])  # allowed again


def test_export_round_trip_through_a_second_generation(torch_cuda):
    # backup 1 writes A; backup 2 (seeded from 1) writes B = A edited and exports
    # only B's new chunks; backup 3 seeded with both sidecars backs up B again
    W = W64
    a = oracle.gen(A_SPEC)
    b = _edited(a, 80)
    recs1, meta1 = _first_backup(torch_cuda, a, W)
    ids1 = _ids(recs1)
    from zbackup_amd import BackupCreator
    tb = torch_cuda.from_numpy(b).to("cuda")
    with BackupCreator(W, sha1=True) as bc:
        bc.seed_index_meta(ids1["sha1"], ids1["rolling"], ids1["size"], meta1)
        bc.chunk_device(tb.data_ptr(), b.size)
        recs2 = bc.records()
        meta2 = bc.export_chunk_meta()
    ids2 = _ids(recs2)
    assert len(meta2) == int((ids2["size"] == W).sum())
    ids = np.concatenate([ids1, ids2])
    meta = np.concatenate([meta1, meta2])
    want = oracle.chunk(b, W, seeds=_seed_tuples(ids))
    got, st0, _ = _run(torch_cuda, b, W, ids, meta, "device")
    assert st0["hist_seeded"] == int((meta["anchor"] != 0xFFFFFFFF).sum())
    assert got == want
    assert sum(1 for r in got if r[0] == "D") >= int((recs2["kind"] == 1).sum())


def _utf16_like(n, seed):
    """UTF-16LE-like text: printable bytes at even offsets, 0 at odd ones."""
    rng = np.random.default_rng(seed)
    out = np.zeros(n, dtype=np.uint8)
    out[0::2] = rng.integers(0x20, 0x7F, (n + 1) // 2, dtype=np.uint8)
    return out


def test_utf16_like_content_vs_oracle(torch_cuda):
    # content whose odd bytes are all 0: the anchor key's odd-parity half is 0
    # at every anchor; records still bit-exact, history included
    W = W64
    x = _utf16_like(12 << 20, 3)
    data = np.concatenate([x, x[5:], _edited(x, 4)])
    want = oracle.chunk(data, W)
    from zbackup_amd import BackupCreator
    t = torch_cuda.from_numpy(data).to("cuda")
    with BackupCreator(W, sha1=True) as bc:
        bc.chunk_device(t.data_ptr(), data.size)
        assert bc.record_tuples() == want
        assert bc.stats()["anchors"] > 0


def test_utf16_like_content_probe_stays_linear(torch_cuda):
    # 1 GiB: 16,384 chunks, every anchor key among 16 values.  With the anchor
    # table slotted on the key alone every chunk's anchor shared 16 probe
    # chains (inserts and walks O(refs / 16) each); slotted on key and
    # fingerprint the batch costs what it costs on random bytes
    from zbackup_amd import BackupCreator, fill_splitmix64
    W = W64
    n = 1 << 30
    half = n // 2
    u = torch_cuda.from_numpy(_utf16_like(half, 5)).to("cuda")
    buf = torch_cuda.empty(n, dtype=torch_cuda.uint8, device="cuda")
    times = {}
    for kind in ("random", "utf16"):
        if kind == "random":
            fill_splitmix64(buf.data_ptr(), half, 99)
        else:
            buf[:half].copy_(u)
        buf[half:].copy_(buf[:half])  # the second half duplicates the first: every chunk a probe hit
        torch_cuda.cuda.synchronize()
        with BackupCreator(W, sha1=False, timing=True) as bc:
            bc.chunk_device(buf.data_ptr(), n)
            bc.chunk_device(buf.data_ptr(), n)
            st = bc.stats()
            kinds = bc.records()["kind"]
        assert int((kinds == 1).sum()) == half // W, kind
        times[kind] = st["meta_ms"] + st["probe_ms"]
    assert times["utf16"] < 4 * times["random"] + 2.0, times


def test_dense_historic_candidates_vs_oracle(torch_cuda):
    # The device orders historic candidates by position in buckets of about
    # n / (2 candidates) bytes; a bucket of more than 64 is left unsorted and
    # the host sorts the whole list (zc_bucket_sort_kernel).  Stream 1 holds
    # 256 KiB of a 1024-byte period (W = 4096: one chunk, then duplicates of
    # it).  Stream 2 is 128 MiB of new random bytes around 128 KiB of the same
    # period at another phase: every historic candidate (one per period) falls
    # in that 128 KiB, about 128 to a bucket.  The records -- the first
    # matching window at each point, as BackupCreator finds it -- must equal
    # the oracle's.
    from zbackup_amd import BackupCreator
    W = 4096
    rng = np.random.default_rng(41)
    per = np.tile(rng.integers(0, 256, 1024, dtype=np.uint8), 300)
    s1 = np.concatenate([rng.integers(0, 256, 2 << 20, dtype=np.uint8), per[:256 << 10],
                         rng.integers(0, 256, 2 << 20, dtype=np.uint8)])
    s2 = np.concatenate([rng.integers(0, 256, 128 << 20, dtype=np.uint8), per[123:123 + (128 << 10)],
                         rng.integers(0, 256, 1 << 20, dtype=np.uint8)])
    t1 = torch_cuda.from_numpy(s1).to("cuda")
    t2 = torch_cuda.from_numpy(s2).to("cuda")
    with BackupCreator(W, sha1=True) as bc:
        bc.chunk_device(t1.data_ptr(), s1.size)
        r1 = bc.records()
        bc.chunk_device(t2.data_ptr(), s2.size)
        got = bc.record_tuples()
        st = bc.stats()
    want = oracle.chunk(s2, W, seeds=_seed_tuples(_ids(r1)))
    assert got == want
    assert st["candidates"] >= 64
    assert sum(1 for r in want if r[0] == "D") >= 20  # the period's windows found in the history
