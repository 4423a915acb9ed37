"""ChunkIndex::findChunk's exact semantics on the device (chunk_index.cc:119-143,
163-182): a window matches only when an index entry has both its 64-bit
rolling key and its 16-byte SHA-1 prefix, and several entries may share one
key (the chain walked by findChunk).  Checked on the device path, through the
smallest feed window, and through the historic index (entries whose bytes have
left HBM), with and without ZC_FLAG_SHA1, against the oracle.

Colliding keys are built, not hoped for: the rolling hash is a polynomial in
base 257 mod 2^64, and for any odd base a 1024-byte Thue-Morse block A and its
complement B have equal polynomials mod 2^64 (prod (x^(2^i) - 1) is divisible
by 2^64 at odd x).  So X+A and X+B are different W-byte windows with one key:
the "key hit, SHA-1 differs" case of findChunk."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from zbackup_amd import _build
    _build.build()
    oracle.build()
    return torch


def _tm_pair(W, seed):
    """Two W-byte chunks, equal rolling key, different bytes (and SHA-1)."""
    t = np.array([bin(i).count("1") & 1 for i in range(1024)], dtype=np.uint8)
    a = np.where(t == 0, 97, 98).astype(np.uint8)
    x = oracle.splitmix64(W - 1024, seed)
    c1, c2 = np.concatenate([x, a]), np.concatenate([x, 195 - a])
    assert oracle.digest(c1) == oracle.digest(c2) and oracle.sha1(c1) != oracle.sha1(c2)
    return c1, c2


def _rand(n, seed):
    return oracle.splitmix64(n, seed)


def _run(torch, data, W, path, sha1, seeds=()):
    from zbackup_amd import BackupCreator
    with BackupCreator(W, seeds=seeds, sha1=sha1, window=1 if path == "window" else None) as bc:
        if path == "device":
            t = torch.from_numpy(np.ascontiguousarray(data)).to("cuda")
            bc.chunk_device(t.data_ptr(), data.size)
        else:
            rng = np.random.default_rng(data.size)
            pos = 0
            while pos < data.size:
                buf = bc.get_input_buffer()
                take = min(int(rng.integers(1, 3 << 20)), bc.get_input_buffer_size(), data.size - pos)
                np.frombuffer(buf, dtype=np.uint8, count=take)[:] = data[pos:pos + take]
                bc.handle_more_data(take)
                pos += take
            bc.finish()
        got = bc.record_tuples()
        st = bc.stats()
    return got, st


def _strip_sha(recs):
    return [(k, o, s, h, "0" * 32 if k != "B" else sha) for (k, o, s, h, sha) in recs]


def _at(recs, off):
    return [r for r in recs if r[1] == off]


@pytest.mark.parametrize("W", [4096, 65536])
@pytest.mark.parametrize("path", ["device", "window"])
@pytest.mark.parametrize("sha1", [True, False])
def test_in_stream_key_collision(torch_cuda, W, path, sha1):
    # C1 on the grid, C2 (same key, other bytes) right after it on the grid
    # (an equal-key class pair that must NOT join), C2 and C1 again off the
    # grid; then ~40 MB later (past the smallest window: C1 is historic by
    # then) C2 and C1 once more
    c1, c2 = _tm_pair(W, 11)
    parts = [_rand(3 * W, 1), c1, c2, _rand(777, 2), c2, _rand(5000, 3), c1, _rand(2 * W + 17, 4), c1, c2,
             _rand(40_000_000, 5), c2, _rand(99, 6), c1, _rand(W + 3, 7)]
    data = np.concatenate(parts)
    want = oracle.chunk(data, W)
    got, st = _run(torch_cuda, data, W, path, sha1)
    assert got == (want if sha1 else _strip_sha(want))
    if path == "window":
        assert st["segments"] >= 2
    if path == "device" and sha1:
        # C1 and C2 are equal-key grid chunks: joined speculatively by key,
        # the digests then differ and the stream is redone (Respeculate)
        assert st["respeculations"] == 1
    # the window that is C2 right after C1 on the grid is no match of C1's
    o2 = 4 * W
    assert [r[0] for r in _at(want, o2)] == ["N"]


@pytest.mark.parametrize("W", [4096, 65536])
@pytest.mark.parametrize("path", ["device", "window"])
def test_static_key_with_wrong_prefix_is_no_match(torch_cuda, W, path):
    # an index entry whose key equals a real window's rolling hash, with another
    # SHA-1 prefix: findChunk finds the key, compares the prefix, no match
    c1, c2 = _tm_pair(W, 12)
    data = np.concatenate([_rand(2 * W + 5, 21), c2, _rand(3 * W, 22), c2, _rand(W, 23)])
    key = oracle.digest(c2)
    wrong = bytes(oracle.sha1(_rand(W, 24))[:16])  # no window of the stream has it
    seeds = [(wrong, key, W)]
    want = oracle.chunk(data, W, seeds=seeds)
    assert not [r for r in want if r[0] == "D"]
    got, _ = _run(torch_cuda, data, W, path, True, seeds)
    assert got == want


@pytest.mark.parametrize("W", [4096, 65536])
@pytest.mark.parametrize("path", ["device", "window"])
def test_static_chain_two_ids_one_key(torch_cuda, W, path):
    # two entries with one key (a chain): the first has a wrong prefix, the
    # second the window's -- findChunk walks the chain and matches the second
    c1, c2 = _tm_pair(W, 13)
    data = np.concatenate([_rand(2 * W + 5, 31), c2, _rand(3 * W, 32), c1, _rand(W, 33)])
    key = oracle.digest(c2)
    seeds = [(bytes(16 * [0x5A]), key, W), (bytes(oracle.sha1(c2)[:16]), key, W)]
    want = oracle.chunk(data, W, seeds=seeds)
    d = [r for r in want if r[0] == "D"]
    assert [r[1] for r in d] == [2 * W + 5]
    got, _ = _run(torch_cuda, data, W, path, True, seeds)
    assert got == want


@pytest.mark.parametrize("W", [4096, 65536])
def test_historic_key_collision_and_seeded_wrong_prefix(torch_cuda, W):
    # stream a saves C1 (a grid chunk): it joins the context's index and, as
    # the stream ends, the historic index (key, SHA-1, anchor; no bytes).  An
    # entry with C1's key and a wrong prefix is seeded next to it (a chain).
    # Stream b holds C2 (key hit, SHA-1 differs: no match) and C1 off the grid
    # (match through the historic entry), on the device and through the window.
    from zbackup_amd import BackupCreator
    c1, c2 = _tm_pair(W, 14)
    a = np.concatenate([_rand(2 * W, 41), c1, _rand(W + 9, 42)])
    b = np.concatenate([_rand(5000, 43), c2, _rand(333, 44), c1, _rand(W + 1, 45), c2, c1])
    want_a = oracle.chunk(a, W)
    key = oracle.digest(c1)
    wrong = (bytes(16 * [0xA5]), key, W)
    idx = [(bytes.fromhex(r[4]), r[3], r[2]) for r in want_a if r[0] == "N"]
    want_b = oracle.chunk(b, W, seeds=idx + [wrong])
    # C2's window is no match (it is cut as part of a saved chunk); C1's is
    assert not [r for r in want_b if r[0] == "D" and r[1] == 5000]
    assert [r for r in want_b if r[0] == "D" and r[1] == 5000 + W + 333]
    for path in ("device", "window"):
        with BackupCreator(W, sha1=True, window=1 if path == "window" else None) as bc:
            ta = torch_cuda.from_numpy(a).to("cuda")
            bc.chunk_device(ta.data_ptr(), a.size)
            assert bc.record_tuples() == want_a
            assert bc.stats()["hist_entries"] > 0
            bc.reset()
            bc.seed_index([wrong])
            if path == "device":
                tb = torch_cuda.from_numpy(b).to("cuda")
                bc.chunk_device(tb.data_ptr(), b.size)
            else:
                bc.feed(b)
                bc.finish()
            assert bc.record_tuples() == want_b, path


@pytest.mark.parametrize("W", [4096, 65536])
def test_respeculation_on_a_context_with_history_and_seeds(torch_cuda, W):
    # a refuted speculative join (equal-key grid chunks C1, C2 of different
    # bytes) redoes the stream after its historic registration has grown the
    # device index: the redo must start from the index exactly as the stream
    # found it -- earlier streams' historic entries and by-value seeds kept,
    # nothing of the refuted pass left -- and the next stream must match the
    # earlier streams' chunks, the redone stream's and the seeds (oracle)
    from zbackup_amd import BackupCreator
    c1, c2 = _tm_pair(W, 15)
    a = _rand(6 * W + 77, 51)
    s = _rand(3 * W, 52)
    seeds = [(bytes(oracle.sha1(s[W:2 * W])[:16]), oracle.digest(s[W:2 * W]), W), (bytes(16 * [0x33]), 12345, W)]
    b = np.concatenate([_rand(2 * W, 53), c1, c2, a[W:4 * W], _rand(W + 5, 54)])
    d = np.concatenate([_rand(123, 55), a[2 * W:5 * W], c2, c1, s[W:2 * W], b[:2 * W], _rand(W, 56)])
    index = list(seeds)
    wants = []
    for x in (a, b, d):
        want = oracle.chunk(x, W, seeds=list(index))
        index += [(bytes.fromhex(sha), h, sz) for (k, o, sz, h, sha) in want if k == "N" and sz == W]
        wants.append(want)
    assert sum(1 for r in wants[1] if r[0] == "D") >= 2
    assert sum(1 for r in wants[2] if r[0] == "D") >= 6
    with BackupCreator(W, seeds=seeds, sha1=True) as bc:
        for i, (x, want) in enumerate(zip((a, b, d), wants)):
            t = torch_cuda.from_numpy(np.ascontiguousarray(x)).to("cuda")
            bc.chunk_device(t.data_ptr(), x.size)
            assert bc.record_tuples() == want, i
            assert bc.stats()["respeculations"] == (1 if i == 1 else 0), i
            bc.reset()


@pytest.mark.parametrize("W", [4096, 65536])
def test_historic_grid_key_collision_refutes_speculation(torch_cuda, W):
    # stream a saves C1 as a grid chunk (it joins the historic index); stream b
    # holds C2 (C1's key, other bytes) as a grid chunk, and no in-stream pair:
    # on the device path C2's window is joined to C1's historic entry on the
    # key before the grid SHA-1 exists, the join is refuted when the digests
    # land and the stream is redone exactly -- C2 saved as new.  Stream c then
    # repeats C1 on its grid: joined the same way, confirmed, a duplicate.
    from zbackup_amd import BackupCreator
    c1, c2 = _tm_pair(W, 16)
    a = np.concatenate([_rand(2 * W, 61), c1, _rand(W, 62)])
    b = np.concatenate([_rand(3 * W, 63), c2, _rand(W + 11, 65)])
    c = np.concatenate([_rand(W, 66), c1, _rand(2 * W + 3, 67)])
    want_a = oracle.chunk(a, W)
    idx = [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in want_a if k == "N" and s == W]
    want_b = oracle.chunk(b, W, seeds=idx)
    idx += [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in want_b if k == "N" and s == W]
    want_c = oracle.chunk(c, W, seeds=idx)
    assert [r[0] for r in _at(want_b, 3 * W)] == ["N"] and [r[0] for r in _at(want_c, W)] == ["D"]
    with BackupCreator(W, sha1=True) as bc:
        ta = torch_cuda.from_numpy(a).to("cuda")
        bc.chunk_device(ta.data_ptr(), a.size)
        assert bc.record_tuples() == want_a
        bc.reset()
        tb = torch_cuda.from_numpy(b).to("cuda")
        bc.chunk_device(tb.data_ptr(), b.size)
        assert bc.record_tuples() == want_b
        assert bc.stats()["respeculations"] == 1
        bc.reset()
        tc = torch_cuda.from_numpy(c).to("cuda")
        bc.chunk_device(tc.data_ptr(), c.size)
        assert bc.record_tuples() == want_c
        assert bc.stats()["respeculations"] == 0
