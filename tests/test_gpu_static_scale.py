"""The static index at repository scale: ChunkIndex::loadIndex
registers every chunk of every index file (chunk_index.cc:26-79) and findChunk
probes all of them at every byte (chunk_index.cc:119-143).  Ids known only by
value (no bytes, no anchors) go through the exact screen; past 2048 keys it
tests a Bloom filter at every position: up to 384 K keys two levels (LDS, then
L2) whose runs are trimmed on the device to exact 64-bit key hits, beyond that
one level whose hits are checked in the kernel against a table of 16-bit check
words.  Seeded with 3,000 / 300,000 / 1 M / 2 M random ids plus the real
ids of a block and of the all-zero chunk that the stream contains: records
bit-exact vs the oracle (device-resident and through the feed window)."""
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


def _same(got, want):
    assert len(got) == len(want), (len(got), len(want))
    for f in ("offset", "size", "kind", "rolling"):
        bad = np.nonzero(got[f] != want[f])[0]
        assert bad.size == 0, f"{f} differs at {bad.size} records, first {bad[:4]}"
    bad = np.nonzero((got["sha1"] != want["sha1"]).any(axis=1))[0]
    assert bad.size == 0, f"sha1 differs at {bad.size} records, first {bad[:4]}"


def _seeds(nrand):
    real = [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in oracle.chunk(oracle.gen("R9:8000000"), W64)
            if k == "N" and s == W64]
    zero = [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in oracle.chunk(oracle.gen("Z:65536"), W64)]
    rng = np.random.default_rng(nrand)
    keys = rng.integers(1, 2**63, nrand, dtype=np.int64)
    shas = rng.integers(0, 256, (nrand, 16), dtype=np.uint8)
    rand = [(shas[i].tobytes(), int(keys[i]), W64) for i in range(nrand)]
    return real + zero + rand, len(real)


SPEC = "R5:30000000,R9:8000000,Z:1000000,R6:20000000,C40000000:3000000,R9:3000000"


@pytest.mark.parametrize("nrand", [3000, 300000, 1000000, 2000000])
def test_large_static_index_device_vs_oracle(torch_cuda, nrand):
    from zbackup_amd import BackupCreator
    seeds, nreal = _seeds(nrand)
    data = oracle.gen(SPEC)
    want = oracle.chunk_array(data, W64, seeds=seeds)
    assert (want["kind"] == 1).sum() >= nreal
    t = torch_cuda.from_numpy(data).to("cuda")
    if nrand >= 1000000:
        # the random ids through the array form (seed_index_arrays), the
        # stream's own ids as tuples
        rng = np.random.default_rng(nrand)
        keys = rng.integers(1, 2**63, nrand, dtype=np.int64)
        shas = rng.integers(0, 256, (nrand, 16), dtype=np.uint8)
        bc = BackupCreator(W64, seeds=seeds[:len(seeds) - nrand], sha1=True)
        bc.seed_index_arrays(shas, keys.astype(np.uint64), W64)
    else:
        bc = BackupCreator(W64, seeds=seeds, sha1=True)
    with bc:
        bc.chunk_device(t.data_ptr(), data.size)
        _same(bc.records(), want)


@pytest.mark.parametrize("nrand", [4000000])
def test_static_index_4m_ids_device_vs_oracle(torch_cuda, nrand):
    # 4 M random ids (a 256 GiB repository at W = 64 KiB) plus the stream's own:
    # the one-level screen with its check table at 4 M keys, every record vs
    # the oracle seeded with the same ids (as arrays: no per-id Python objects)
    from zbackup_amd import BackupCreator
    real, _ = _seeds(0)
    rng = np.random.default_rng(nrand)
    sa = np.zeros(nrand, dtype=oracle.SEED_DTYPE)
    sa["rolling"] = rng.integers(1, 2**63, nrand, dtype=np.int64).astype(np.uint64)
    sa["sha1"] = rng.integers(0, 256, (nrand, 16), dtype=np.uint8)
    sa["size"] = W64
    seeds = np.concatenate([oracle.seed_array(real), sa])
    data = oracle.gen(SPEC)
    want = oracle.chunk_array(data, W64, seeds=seeds)
    assert (want["kind"] == 1).sum() >= len(real) - 1
    t = torch_cuda.from_numpy(data).to("cuda")
    with BackupCreator(W64, sha1=True) as bc:
        bc.seed_index_arrays(seeds["sha1"], seeds["rolling"], seeds["size"])
        assert bc.stats()["by_value"] == len(seeds)
        bc.chunk_device(t.data_ptr(), data.size)
        _same(bc.records(), want)


@pytest.mark.parametrize("nrand", [300000, 1000000])
def test_large_static_index_window_vs_oracle(torch_cuda, nrand):
    from zbackup_amd import BackupCreator
    seeds, _ = _seeds(nrand)
    data = oracle.gen(SPEC)
    want = oracle.chunk_array(data, W64, seeds=seeds)
    with BackupCreator(W64, seeds=seeds, sha1=True, window=1) as bc:
        bc.feed(data)
        bc.finish()
        _same(bc.records(), want)


@pytest.mark.parametrize("W,nrand", [(1000, 3000), (4099, 3000), (300007, 3000), (1000, 700000), (4099, 700000)])
def test_bloom_screen_odd_w_vs_oracle(torch_cuda, W, nrand):
    """The Bloom mode of the staged screen (over 2048 by-value keys; two
    levels, and one level past 384 K) at chunk sizes whose out-byte funnel
    shifts differ (-W mod 16 = 8, 13, 9), on a stream long enough (> 64 MiB)
    for the staged kernel to run."""
    from zbackup_amd import BackupCreator
    old = oracle.gen("R9:8000000")
    real = [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in oracle.chunk(old, W) if k == "N" and s == W][:400]
    zero = [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in oracle.chunk(oracle.gen(f"Z:{W}"), W)]
    rng = np.random.default_rng(W)
    keys = rng.integers(1, 2**63, nrand, dtype=np.int64)
    shas = rng.integers(0, 256, (nrand, 16), dtype=np.uint8)
    seeds = real + zero + [(shas[i].tobytes(), int(keys[i]), W) for i in range(nrand)]
    data = oracle.gen("R5:40000000,R9:8000000,Z:1000000,R6:30000000,C41000000:3000000")
    want = oracle.chunk_array(data, W, seeds=seeds)
    assert (want["kind"] == 1).sum() >= len(real)
    t = torch_cuda.from_numpy(data).to("cuda")
    with BackupCreator(W, seeds=seeds, sha1=True) as bc:
        bc.chunk_device(t.data_ptr(), data.size)
        _same(bc.records(), want)


def _headed_blocks(nblk, W, seed):
    """nblk W-byte blocks, each 32 seeded random bytes then zeros: all distinct,
    none with an anchor (a chunk's first anchor sits at offset >= 63, where
    the anchor test's 31-byte window sees only zeros)."""
    rng = np.random.default_rng(seed)
    b = np.zeros((nblk, W), dtype=np.uint8)
    b[:, :32] = rng.integers(0, 256, (nblk, 32), dtype=np.uint8)
    return b.reshape(-1)


def test_check_table_overflow_rebuilds_vs_oracle(torch_cuda, monkeypatch):
    """An epoch whose own anchorless keys do not fit the one-level screen's check
    table (the by-value set's table plus room for 65,536 epoch keys): the table
    is rebuilt with room for them and the one-level screen kept.  Forced here:
    ZC_TEST_CHK_BITS starts the table's size search so small that it ends
    barely holding the 400 K seeded keys, and the 72 MB stream is ~590 K
    distinct anchorless chunks, every one of whose keys joins the epoch's copy
    of the table; 400 seeded ids are blocks the stream repeats (matches)."""
    from zbackup_amd import BackupCreator
    W = 128
    old = _headed_blocks(2000, W, 7)
    real = [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in oracle.chunk(old, W) if k == "N" and s == W][:400]
    rng = np.random.default_rng(48)
    keys = rng.integers(1, 2**63, 400000, dtype=np.int64)
    shas = rng.integers(0, 256, (400000, 16), dtype=np.uint8)
    seeds = real + [(shas[i].tobytes(), int(keys[i]), W) for i in range(400000)]
    data = np.concatenate([_headed_blocks(300000, W, 8), oracle.gen("R5:77"), old[:51200],
                           _headed_blocks(290000, W, 9)])
    want = oracle.chunk_array(data, W, seeds=seeds)
    assert (want["kind"] == 1).sum() >= len(real)
    monkeypatch.setenv("ZC_TEST_CHK_BITS", "12")
    t = torch_cuda.from_numpy(data).to("cuda")
    with BackupCreator(W, seeds=seeds, sha1=True) as bc:
        bc.chunk_device(t.data_ptr(), data.size)
        _same(bc.records(), want)
        assert bc.stats()["chk_rebuilds"] >= 1
