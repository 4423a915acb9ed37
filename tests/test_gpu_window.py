"""GPU parity of the bounded feed window (zc_set_window): the stream goes
through BackupCreator's zero-copy feed contract (getInputBuffer /
getInputBufferSize / handleMoreData, zutils.cc:100-124) in ragged pieces, is
chunked a window half at a time during handleMoreData, and the window slides,
so chunks far back are matched by {key, SHA-1, first anchor} only (the
historic index) -- records bit-exact vs the oracle (backup_creator.cc:56-172,
chunk_index.cc:119-143), drained incrementally, with their payload bytes
readable right after they are taken; device memory flat over the stream."""
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


def _feed(bc, data, rng, max_piece, check_payload=True):
    """Ragged zero-copy feed; takes records after every piece and checks the
    payload of every taken record against the input (bytes stay readable
    until the next feed call).  Returns (records, hbm_bytes samples)."""
    taken, hbm = [], []
    pos = 0
    while pos < data.size:
        buf = bc.get_input_buffer()
        room = bc.get_input_buffer_size()
        assert room > 0
        take = min(int(rng.integers(1, max_piece + 1)), room, data.size - pos)
        np.frombuffer(buf, dtype=np.uint8, count=take)[:] = data[pos:pos + take]
        bc.handle_more_data(take)
        pos += take
        recs = bc.take_records()
        if len(recs):
            taken.append(recs)
            if check_payload:
                for r in (recs[0], recs[-1]):
                    o, n = int(r["offset"]), int(r["size"])
                    assert bc.read_stream(o, n) == data[o:o + n].tobytes()
                    assert bc.stream_data(o, n) == data[o:o + n].tobytes()  # zero-copy view
            hbm.append(bc.stats()["hbm_bytes"])
    bc.finish()
    taken.append(bc.take_records())
    return np.concatenate(taken), hbm


def _same(got, want):
    assert len(got) == len(want), (len(got), len(want))
    for f in ("offset", "size", "kind", "rolling"):
        bad = np.nonzero(got[f] != want[f])[0]
        assert bad.size == 0, f"{f} differs at {bad.size} records, first {bad[:4]}: {got[bad[:2]]} vs {want[bad[:2]]}"
    bad = np.nonzero((got["sha1"] != want["sha1"]).any(axis=1))[0]
    assert bad.size == 0, f"sha1 differs at {bad.size} records, first {bad[:4]}"


# streams whose copies reach back past the window (historic matches by
# SHA-1), zero runs (anchorless chunks: the by-value screen), shifted copies
# (grid-shifting matches across slides) and a copy of the copy
SPECS = [
    (65536, "R1:70000000,C1000:9000000,Z:3000000,R2:30000000,C5:20000000,C70000123:6000000,R3:777777"),
    (4096, "R7:30000000,C333:4000000,Z:2000000,R8:10000000,C17:3000000,B3:100000,C31000000:5000000,R9:4097"),
    (1000, "R11:25000000,C3:2000000,R12:6000000,C12345:3000000,Z:500000,C20000000:1000000"),
    (300007, "R21:40000000,C100:12000000,Z:1500000,R22:8000000,C40000000:6000000"),
]


@pytest.mark.parametrize("W,spec", SPECS)
@pytest.mark.parametrize("sha1", [True, False])
def test_window_feed_vs_oracle(torch_cuda, W, spec, sha1):
    from zbackup_amd import BackupCreator
    data = oracle.gen(spec)
    want = oracle.chunk_array(data, W)
    if not sha1:
        want["sha1"][:] = 0
    rng = np.random.default_rng(W)
    with BackupCreator(W, sha1=sha1, window=1) as bc:  # the smallest window: 8 W + 16 MiB
        got, _ = _feed(bc, data, rng, 3 << 20)
        st = bc.stats()
    assert st["segments"] >= 2 and st["window_bytes"] < data.size
    _same(got, want)


def test_window_1gib_ragged_128mib_flat_hbm(torch_cuda):
    """A 1 GiB stream through a 128 MiB window: bit-exact vs the oracle, and
    the context's device memory stays flat while the stream grows."""
    from zbackup_amd import BackupCreator
    spec = ("R41:300000000,C12345:100000000,Z:20000000,R42:200000000,C250000000:150000000,"
            "R43:100000000,C1:100000000,B7:3000000,R44:101000000")
    data = oracle.gen(spec)
    assert data.size >= 1 << 30
    want = oracle.chunk_array(data, W64)
    rng = np.random.default_rng(5)
    with BackupCreator(W64, sha1=True, window=128 << 20) as bc:
        got, hbm = _feed(bc, data, rng, 9 << 20, check_payload=False)
        st = bc.stats()
    _same(got, want)
    assert st["segments"] >= 12 and st["hist_entries"] > 0
    # flat: what the context holds late in the stream is what it held early
    quarter = hbm[len(hbm) // 4]
    assert max(hbm) <= quarter + (32 << 20), (quarter, max(hbm))
    assert max(hbm) < 4 * (128 << 20)


def test_window_second_stream_matches_first(torch_cuda):
    """With ZC_FLAG_SHA1 a stream's chunks join the context's index (Writer::add
    -> ChunkIndex::addChunk); the next stream, fed through the window, matches
    them by key and SHA-1 (historic entries) -- as a later backup matches a
    committed one's index."""
    from zbackup_amd import BackupCreator
    a = oracle.gen("R51:40000000,Z:1000000,R52:5000000")
    b = oracle.gen("R53:3000000,R51:40000000,R54:777,R52:5000000,Z:2000000")
    want_a = oracle.chunk_array(a, W64)
    seeds = [(bytes(r["sha1"]), int(r["rolling"]), int(r["size"])) for r in want_a if r["kind"] == 0]
    want_b = oracle.chunk_array(b, W64, seeds=seeds)
    assert (want_b["kind"] == 1).sum() > 500
    rng = np.random.default_rng(9)
    with BackupCreator(W64, sha1=True, window=1) as bc:
        got_a, _ = _feed(bc, a, rng, 5 << 20)
        _same(got_a, want_a)
        bc.reset()
        got_b, _ = _feed(bc, b, rng, 5 << 20)
        _same(got_b, want_b)


def test_device_second_stream_uses_historic_index(torch_cuda):
    """Device-resident streams on one context with ZC_FLAG_SHA1: the second
    stream (the first one's bytes shifted and repeated) matches the first's
    chunks through the historic index, not the by-value screen."""
    from zbackup_amd import BackupCreator
    a = oracle.gen("R61:30000000,Z:700000")
    b = oracle.gen("R62:12345,R61:30000000,Z:700000,R61:1000000")
    want_a = oracle.chunk_array(a, W64)
    seeds = [(bytes(r["sha1"]), int(r["rolling"]), int(r["size"])) for r in want_a if r["kind"] == 0]
    want_b = oracle.chunk_array(b, W64, seeds=seeds)
    ta = torch_cuda.from_numpy(a).to("cuda")
    tb = torch_cuda.from_numpy(b).to("cuda")
    with BackupCreator(W64, sha1=True) as bc:
        bc.chunk_device(ta.data_ptr(), a.size)
        _same(bc.records(), want_a)
        st = bc.stats()
        assert st["hist_entries"] > 0  # anchored chunks (the zero chunk goes by value)
        bc.reset()
        bc.chunk_device(tb.data_ptr(), b.size)
        _same(bc.records(), want_b)


def test_unbounded_window_still_works(torch_cuda):
    from zbackup_amd import BackupCreator
    data = oracle.gen("R71:5000000,C100:70000,Z:200000")
    want = oracle.chunk_array(data, 4096)
    with BackupCreator(4096, window=0) as bc:
        assert bc.window == 0
        bc.feed(data)
        bc.finish()
        _same(bc.records(), want)


@pytest.mark.parametrize("W,block,piece", [(65536, 48 << 20, 1 << 20), (4096, 24 << 20, 64 << 10)])
def test_window_edited_duplicate_vs_oracle(torch_cuda, W, block, piece):
    """An edited duplicate (a block, then the block with 1-100 random bytes
    inserted every `piece` bytes: one grid shift per insertion, walked lazily
    on the shifted grid) fed through the smallest window: the lazy-shift state
    crosses window segments and slides."""
    from zbackup_amd import BackupCreator
    rng = np.random.default_rng(W + 1)
    segs, off = [f"R77:{block}"], 0
    while off < block:
        ln = min(piece, block - off)
        segs += [f"C{off}:{ln}", f"R{int(rng.integers(1, 1 << 30))}:{int(rng.integers(1, 101))}"]
        off += ln
    data = oracle.gen(",".join(segs))
    want = oracle.chunk_array(data, W)
    assert (want["kind"] == 1).sum() > block // W // 2
    with BackupCreator(W, sha1=True, window=1) as bc:
        got, _ = _feed(bc, data, np.random.default_rng(3), 5 << 20)
        st = bc.stats()
    assert st["segments"] >= 4
    _same(got, want)
