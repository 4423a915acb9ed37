"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference-built golden fixtures.  Integer/byte work, so the bar is bit-exact:
offsets, sizes, kinds, 64-bit rolling hashes and SHA-1 prefixes."""
import numpy as np
import pytest

from oracle import oracle
from tests import golden_io

pytestmark = pytest.mark.gpu

CASES = golden_io.case_names()
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


def _case(name):
    return golden_io.load_case(f"{golden_io.GOLDEN}/{name}.txt")


def _run_host_feed(data, W, seeds=(), chunk=None, sha1=True):
    from zbackup_amd import BackupCreator
    with BackupCreator(W, seeds=seeds, sha1=sha1) as bc:
        if chunk is None:
            bc.feed(data)
        else:
            # the zero-copy contract of zutils.cc:100-124, in ragged pieces
            rng = np.random.default_rng(len(data))
            pos = 0
            while pos < data.size:
                buf = bc.get_input_buffer()
                take = min(int(rng.integers(1, chunk + 1)), bc.get_input_buffer_size(), data.size - pos)
                np.frombuffer(buf, dtype=np.uint8, count=take)[:] = data[pos:pos + take]
                bc.handle_more_data(take)
                pos += take
        bc.finish()
        return bc.record_tuples()


def _run_device(torch, data, W, seeds=(), sha1=True):
    from zbackup_amd import BackupCreator
    t = torch.from_numpy(np.ascontiguousarray(data)).to("cuda") if data.size else torch.empty(
        0, dtype=torch.uint8, device="cuda")
    with BackupCreator(W, seeds=seeds, sha1=sha1) as bc:
        bc.chunk_device(t.data_ptr(), data.size)
        return bc.record_tuples()


@pytest.mark.parametrize("name", CASES)
def test_golden_host_feed(torch_cuda, name):
    meta, seeds, want = _case(name)
    data = oracle.gen(meta["spec"])
    assert _run_host_feed(data, meta["W"], seeds) == want


@pytest.mark.parametrize("name", CASES)
def test_golden_device_resident(torch_cuda, name):
    meta, seeds, want = _case(name)
    data = oracle.gen(meta["spec"])
    assert _run_device(torch_cuda, data, meta["W"], seeds) == want


@pytest.mark.parametrize("name", ["w4096_shift", "mixed", "frag50", "w257_periodic"])
def test_ragged_feed(torch_cuda, name):
    meta, seeds, want = _case(name)
    data = oracle.gen(meta["spec"])
    assert _run_host_feed(data, meta["W"], seeds, chunk=70001) == want


# random stress: synthetic streams built from copies at arbitrary offsets,
# zero runs and repeated bytes, checked against the oracle
def _random_spec(rng, W):
    segs, n = [], 0
    for _ in range(int(rng.integers(2, 9))):
        t = rng.integers(0, 5)
        ln = int(rng.integers(1, 5 * W))
        if t == 0 or n == 0:
            segs.append(f"R{int(rng.integers(1, 1 << 30))}:{ln}")
        elif t == 1:
            segs.append(f"Z:{ln}")
        elif t == 2:
            segs.append(f"B{int(rng.integers(0, 256))}:{ln}")
        else:
            segs.append(f"C{int(rng.integers(0, n))}:{ln}")
        n += ln
    return ",".join(segs)


@pytest.mark.parametrize("seed", range(24))
def test_random_streams_vs_oracle(torch_cuda, seed):
    rng = np.random.default_rng(1000 + seed)
    W = int(rng.choice([128, 200, 257, 1000, 1024, 4096, 4097, 65536]))
    spec = _random_spec(rng, W)
    data = oracle.gen(spec)
    want = oracle.chunk(data, W)
    assert _run_device(torch_cuda, data, W) == want, spec


# streams of several full 2 MiB scan tiles plus a partial one: the persistent
# scan kernel (not only the tail kernel) at every anchor rate, including the
# dense small-W rates where a dword holds several anchors, spans overflow
# their anchor slots and waves overflow their LDS anchor lists
@pytest.mark.parametrize("W", [128, 257, 1000, 4096, 65536])
def test_multi_tile_vs_oracle(torch_cuda, W):
    spec = f"R{W}:3000000,C1000:1500000,Z:300000,B7:100000,C5:2000000,R77:411111"
    data = oracle.gen(spec)
    want = oracle.chunk(data, W)
    assert _run_device(torch_cuda, data, W) == want


# SHA-1 ids on streams of many grid chunks per scan lane: the grid SHA-1
# (zc_sha1_grid16_kernel, queued behind the first epoch's batch) hashes every
# grid chunk, and records that are whole grid chunks take their prefix from
# it.  Cases: many chunks per scan lane (W = 128), W not a power of two
# (2944 = 16 * 184: the aligned kernel; the general one for W % 16 != 0 runs in
# the fuzz suite), a 3-byte partial last chunk (zc_sha1_one_kernel),
# duplicates moving the grid, and 260 scan tiles
@pytest.mark.parametrize("W,spec", [
    (128, "R31:50000000,C7:3000000,R32:333"),
    (1024, "R33:40000000,Z:2000000,C123:5000000,R34:77777"),
    (2944, "R35:50331648"),
    (4096, "R36:50343939"),
    (1024, "R37:545259520,R38:4321"),
])
def test_grid_sha1_many_chunks_per_lane_vs_oracle(torch_cuda, W, spec):
    data = oracle.gen(spec)
    want = oracle.chunk(data, W)
    assert _run_device(torch_cuda, data, W) == want


# tiny chunk sizes: below the anchor offset (every ref anchorless: the exact
# screen alone) and below the staged screen's 32-byte minimum
@pytest.mark.parametrize("W", [1, 2, 7, 16, 31, 32, 33, 63, 64, 65])
def test_tiny_chunk_sizes_vs_oracle(torch_cuda, W):
    spec = "R21:20000,C333:4000,Z:700,B9:300,R22:9000,C5000:6000,R23:77"
    data = oracle.gen(spec)
    want = oracle.chunk(data, W)
    assert _run_device(torch_cuda, data, W) == want


# chunk sizes above the 256 KiB wave-tile (a chunk's first anchor may lie in a
# later wave-tile; horizons of 64 W), including one that is not a multiple of
# the 1 KiB span
@pytest.mark.parametrize("W", [262144, 300007, 1 << 20])
def test_large_chunk_sizes_vs_oracle(torch_cuda, W):
    spec = f"R11:{6 * W + 12345},C{3 * W + 17}:{2 * W + 999},Z:{W + 5},R12:{2 * W},C{W // 2}:{3 * W}"
    data = oracle.gen(spec)
    want = oracle.chunk(data, W)
    assert _run_device(torch_cuda, data, W) == want


# long runs of grid chunks (>= 32,768 records at once) are written by the host
# thread pool; the runs here are cut by a same-grid match (dead refs: the
# serial path) and by a grid-shifting one (a new epoch's run)
@pytest.mark.parametrize("spec", ["R3:6000000", "R3:6000000,C1000:5120,R4:6000000",
                                  "R3:4194304,C4194300:6000,R4:4500000"])
def test_long_grid_runs_vs_oracle(torch_cuda, spec):
    W = 128
    data = oracle.gen(spec)
    want = oracle.chunk(data, W)
    assert sum(1 for r in want if r[0] == "N") >= 32768
    assert _run_device(torch_cuda, data, W) == want


def _dense_anchor_pattern(W, period=16):
    """A `period`-byte pattern whose periodic extension has an anchor in every
    period at chunk size W (the anchor state of zc_device.h: st(q) = sum_{j<16}
    b[q-2j] 2^j mod 2^16, an anchor where (int16)st(q) >= anchor_lo), so
    wave-tiles overflow their anchor-pool share."""
    rate = 16
    while rate < 4096 and rate * 2 <= W // 16:
        rate *= 2
    lo = 0x8000 - 0x10000 // rate
    rng = np.random.default_rng(77)
    for _ in range(100000):
        pat = rng.integers(0, 256, period, dtype=np.uint8)
        ext = np.tile(pat, 64 // period + 2)
        for q in range(32, 32 + period):
            st = 0
            for j in range(16):
                st = (st + (int(ext[q - 2 * j]) << j)) & 0xFFFF
            if lo <= st < 0x8000:
                return pat
    raise AssertionError("no pattern found")


@pytest.mark.parametrize("W", [4096, 65536])
def test_dense_anchor_overflow_vs_oracle(torch_cuda, W):
    # every period holds an anchor: ~16x the pool share per wave-tile at
    # W = 65536, so the side-pool rescan path runs; mixed with random bytes
    pat = _dense_anchor_pattern(W)
    body = np.tile(pat, (3 << 20) // pat.size)
    data = np.concatenate([oracle.gen("R9:1500000"), body, oracle.gen("R10:777777"), body[:1000003]])
    want = oracle.chunk(data, W)
    assert _run_device(torch_cuda, data, W) == want


def test_chunk_host_overlapped_vs_oracle(torch_cuda):
    # zc_chunk_host: several 64 MiB copy/scan segments plus a partial tile,
    # from pinned host memory; records equal the oracle's
    from zbackup_amd import BackupCreator
    data = oracle.gen("R5:80000000,C1000:50000000,Z:3000000,R6:7777777")
    want = oracle.chunk(data, W64)
    host = torch_cuda.from_numpy(data).pin_memory()
    with BackupCreator(W64) as bc:
        bc.chunk_host(host.data_ptr(), data.size)
        assert bc.record_tuples() == want


def test_index_persists_across_streams(torch_cuda):
    # ChunkStorage::Writer::add -> ChunkIndex::addChunk: a second stream on the
    # same context matches the first stream's chunks (zutils.cc:137-166 reuses
    # one index for the iterative passes)
    from zbackup_amd import BackupCreator
    a = oracle.gen("R501:700000")
    b = oracle.gen("R502:33333,R501:700000,R503:1000")
    want_a = oracle.chunk(a, W64)
    seeds = [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in want_a if k == "N"]
    want_b = oracle.chunk(b, W64, seeds=seeds)
    assert sum(1 for r in want_b if r[0] == "D") > 0
    with BackupCreator(W64, sha1=True) as bc:
        bc.feed(a)
        bc.finish()
        assert bc.record_tuples() == want_a
        bc.reset()
        bc.feed(b)
        bc.finish()
        assert bc.record_tuples() == want_b


def test_forget_stream_chunks_restores_the_seeded_index(torch_cuda):
    """zc_forget_stream_chunks: after it, a stream on a reused context chunks as
    on a fresh one with the same seeds (the stream-added entries are gone, the
    seeded ones stay)."""
    from zbackup_amd import BackupCreator
    a = oracle.gen("R601:400000")
    s = oracle.gen("R602:300000")
    want_s = oracle.chunk(s, W64)
    seeds = [(bytes.fromhex(sha), h, sz) for (k, o, sz, h, sha) in want_s if k == "N"]
    b = oracle.gen("R602:300000,R601:400000,R603:5000")
    want_b = oracle.chunk(b, W64, seeds=seeds)
    assert any(r[0] == "D" for r in want_b)
    with BackupCreator(W64, seeds=seeds, sha1=True) as bc:
        for _ in range(2):
            bc.feed(a)
            bc.finish()
            bc.reset()
            bc.forget_stream_chunks()  # a's chunks leave the index again
            bc.feed(b)
            bc.finish()
            assert bc.record_tuples() == want_b  # seeded matches only
            bc.reset()
            bc.forget_stream_chunks()


@pytest.mark.parametrize("name,path", [("frag50", "feed"), ("frag50", "device"), ("mixed", "feed"),
                                       ("mixed", "device"), ("small_tail", "window")])
def test_get_backup_data_matches_oracle_serialization(torch_cuda, name, path):
    # zc_serialize_records (Message::serialize per record, bytes_to_emit read
    # from the stream) vs the same stream serialized from the oracle's records
    from zbackup_amd import BackupCreator, chunk_id_blob, serialize_instruction
    meta, seeds, want = _case(name)
    data = oracle.gen(meta["spec"])
    expect = b""
    for (k, off, size, h, sha) in want:
        if k == "B":
            expect += serialize_instruction(raw=data[off:off + size].tobytes())
        else:
            expect += serialize_instruction(chunk_blob=chunk_id_blob(bytes.fromhex(sha), h))
    with BackupCreator(meta["W"], seeds=seeds, window=(8 * meta["W"] + (16 << 20)) if path == "window" else None) as bc:
        if path == "device":
            t = torch_cuda.from_numpy(data).to("cuda")
            bc.chunk_device(t.data_ptr(), data.size)
        else:
            bc.feed(data)
            bc.finish()
        assert bc.get_backup_data() == expect
        with pytest.raises(Exception):
            bc.get_backup_data()  # backup_creator.cc:277 CHECK: only once


@pytest.mark.parametrize("n", [0, 1, 7, 8, 1000, 4099, 1 << 20])
def test_device_filler_matches_oracle_generator(torch_cuda, n):
    from zbackup_amd import fill_splitmix64
    t = torch_cuda.empty(max(n, 1), dtype=torch_cuda.uint8, device="cuda")
    fill_splitmix64(t.data_ptr(), n, 77)
    assert np.array_equal(t.cpu().numpy()[:n], oracle.splitmix64(n, 77))


# --- BASELINE.json configs at full size: size-independent properties --------

def _sample_digests(torch, t, offsets, size):
    host = t.cpu().numpy() if t.numel() <= (1 << 24) else None
    out = []
    for off in offsets:
        chunk = host[off:off + size] if host is not None else t[off:off + size].cpu().numpy()
        out.append(oracle.digest(chunk))
    return out


@pytest.fixture(scope="module")
def big_random(torch_cuda):
    from zbackup_amd import fill_splitmix64
    n = 8 << 30
    t = torch_cuda.empty(n, dtype=torch_cuda.uint8, device="cuda")
    fill_splitmix64(t.data_ptr(), n, 2024)
    yield t
    del t
    torch_cuda.cuda.empty_cache()


def test_c2_random_8gib_grid(torch_cuda, big_random):
    from zbackup_amd import BackupCreator
    n = big_random.numel()
    with BackupCreator(W64, sha1=False) as bc:
        bc.chunk_device(big_random.data_ptr(), n)
        recs = bc.records()
    assert len(recs) == n // W64
    assert (recs["kind"] == 0).all()
    assert np.array_equal(recs["offset"], np.arange(n // W64, dtype=np.uint64) * W64)
    assert (recs["size"] == W64).all()
    rng = np.random.default_rng(5)
    idx = np.unique(np.concatenate([[0, len(recs) - 1], rng.integers(0, len(recs), 254)]))
    want = _sample_digests(torch_cuda, big_random, [int(recs["offset"][i]) for i in idx], W64)
    assert [int(recs["rolling"][i]) for i in idx] == want


def test_c3_half_duplicated_8gib(torch_cuda, big_random):
    from zbackup_amd import BackupCreator
    n = big_random.numel()
    half = n // 2
    big_random[half:].copy_(big_random[:half])
    with BackupCreator(W64, sha1=False) as bc:
        bc.chunk_device(big_random.data_ptr(), n)
        recs = bc.records()
    m = half // W64
    assert len(recs) == 2 * m
    assert (recs["kind"][:m] == 0).all() and (recs["kind"][m:] == 1).all()
    assert np.array_equal(recs["rolling"][:m], recs["rolling"][m:])
    assert np.array_equal(recs["offset"], np.arange(2 * m, dtype=np.uint64) * W64)
    rng = np.random.default_rng(6)
    idx = rng.integers(0, m, 64)
    want = _sample_digests(torch_cuda, big_random, [int(recs["offset"][i]) for i in idx], W64)
    assert [int(recs["rolling"][i]) for i in idx] == want


def test_c5_all_zero_8gib(torch_cuda, big_random):
    from zbackup_amd import BackupCreator
    n = big_random.numel()
    big_random.zero_()
    with BackupCreator(W64, sha1=False) as bc:
        bc.chunk_device(big_random.data_ptr(), n)
        recs = bc.records()
    assert len(recs) == n // W64
    assert recs["kind"][0] == 0 and (recs["kind"][1:] == 1).all()
    assert (recs["rolling"] == 0x172AEAFF81000001).all()
    assert np.array_equal(recs["offset"], np.arange(n // W64, dtype=np.uint64) * W64)


# --- edited duplicates: a copy with small insertions every piece ------------
# (each insertion moves the grid: backup_creator.cc:242-265 resets the window
# on the match after it; the walk follows the new grid lazily)

def edited_copy_spec(seed, block, piece, rng):
    """R<seed>:<block> followed by the same bytes in `piece`-byte pieces, each
    followed by 1-100 inserted random bytes."""
    segs, off = [f"R{seed}:{block}"], 0
    while off < block:
        ln = min(piece, block - off)
        segs.append(f"C{off}:{ln}")
        segs.append(f"R{int(rng.integers(1, 1 << 30))}:{int(rng.integers(1, 101))}")
        off += ln
    return ",".join(segs)


@pytest.mark.parametrize("W,block,piece", [(65536, 64 << 20, 1 << 20), (4096, 8 << 20, 64 << 10),
                                           (1000, 2 << 20, 50000)])
def test_edited_duplicate_vs_oracle(torch_cuda, W, block, piece):
    rng = np.random.default_rng(W)
    data = oracle.gen(edited_copy_spec(31, block, piece, rng))
    want = oracle.chunk(data, W)
    assert sum(1 for r in want if r[0] == "D") > block // W // 2
    assert _run_device(torch_cuda, data, W) == want
    assert _run_host_feed(data, W) == want


@pytest.mark.parametrize("sha1", [True, False])
def test_backup_data_of_a_long_windowed_stream(torch_cuda, sha1):
    # a stream many windows long whose first records are a bytes_to_emit
    # fragment (50 bytes between a chunk and its copy) and a short chunk: the
    # records are serialized as they are taken, while their bytes are still in
    # the window; getBackupData at the end equals the oracle's stream
    from zbackup_amd import BackupCreator, chunk_id_blob, serialize_instruction
    W = 4096
    data = oracle.gen("R1:4096,R2:50,C0:4096,R3:300,C4146:4096,R4:70000000,C0:4096")
    want = oracle.chunk(data, W)
    assert want[1][0] == "B" and want[1][2] == 50
    expect = b""
    for (k, off, size, h, sha) in want:
        if k == "B":
            expect += serialize_instruction(raw=data[off:off + size].tobytes())
        else:
            expect += serialize_instruction(chunk_blob=chunk_id_blob(bytes.fromhex(sha) if sha1 else bytes(16), h))
    with BackupCreator(W, sha1=sha1, window=8 * W + (16 << 20)) as bc:
        pos = 0
        while pos < data.size:
            buf = bc.get_input_buffer()
            take = min(bc.get_input_buffer_size(), data.size - pos)
            np.frombuffer(buf, dtype=np.uint8, count=take)[:] = data[pos:pos + take]
            bc.handle_more_data(take)
            pos += take
        bc.finish()
        assert bc.stats()["segments"] >= 3
        assert bc.get_backup_data() == expect
        if sha1:
            assert bc.record_tuples() == want


@pytest.mark.parametrize("path", ["device", "feed", "window"])
def test_all_duplicate_middle_stream_keeps_the_index(torch_cuda, path):
    # three (four) SHA-1 streams on one context: the second repeats the first,
    # so it saves no W-byte chunk at all; the index the first stream built
    # (keys and SHA-1 prefixes of its historic entries) must survive it, and
    # must survive the third stream growing it, so the third and fourth
    # streams match the first's chunks as ChunkIndex::findChunk would
    # (chunk_index.cc:119-143 over the entries Writer::add registered)
    from zbackup_amd import BackupCreator
    a = oracle.gen("R701:700000")
    b = oracle.gen("R702:33333,R701:700000,R703:150000")
    d = oracle.gen("R704:999,R701:500000,R703:150000,R705:7")
    index = []
    wants = []
    for s in (a, a, b, d):
        want = oracle.chunk(s, W64, seeds=list(index))
        index += [(bytes.fromhex(sha), h, sz) for (k, o, sz, h, sha) in want if k == "N" and sz == W64]
        wants.append(want)
    assert all(r[0] == "D" for r in wants[1] if r[2] == W64)
    assert sum(1 for r in wants[2] if r[0] == "D") >= 8 and sum(1 for r in wants[3] if r[0] == "D") >= 6
    with BackupCreator(W64, sha1=True, window=1 if path == "window" else None) as bc:
        for s, want in zip((a, a, b, d), wants):
            if path == "device":
                t = torch_cuda.from_numpy(s).to("cuda")
                bc.chunk_device(t.data_ptr(), s.size)
            else:
                bc.feed(s)
                bc.finish()
            assert bc.record_tuples() == want
            bc.reset()
