"""GPU parity of the bundle writer offload (§8(f)-4), through the C ABI:
zc_lzo_compress's framed lzo1x_1 output is byte-identical to liblzo2 2.10's
lzo1x_1_compress + zbackup's framing (compression.cc:435-466, 586-606) for
every payload -- six kinds of content, the block-edge sizes of
lzo1x_1_compress's 49152-byte split (20/21 bytes, 49152 + 20/21), random sizes
up to 3 MB, payloads and outputs at unaligned device offsets -- and a chunked
stream's new chunks, bundled by Writer::add's rule (chunk_storage.cc:31-46) and
gathered on the device (Bundle::Creator::addChunk, bundle.cc:30-36), give the
same bundle files' payload bytes as the oracle's records do."""
import numpy as np
import pytest

from oracle import lzo_oracle, oracle
from tests.lzo_inputs import KINDS, payload

pytestmark = pytest.mark.gpu

EDGE_SIZES = [0, 1, 3, 4, 17, 20, 21, 22, 40, 41, 100, 1000, 49151, 49152, 49153, 49172, 49173, 49174, 98304,
              98324, 98325, 100000, 262144, 2097152]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    if lzo_oracle.lzo_lib() is None:
        pytest.skip("liblzo2 not in this image")
    from zbackup_amd import _build
    _build.build()
    oracle.build()
    return torch


@pytest.fixture(scope="module")
def comp(torch_cuda):
    from zbackup_amd.bundle import BundleCompressor
    with BundleCompressor() as c:
        yield c


def _compress(torch, comp, payloads, rng):
    """All payloads in one zc_lzo_compress call, at odd offsets in and out."""
    from zbackup_amd.bundle import lzo_capacity
    pay_off, pos = [], 0
    for p in payloads:
        pos += int(rng.integers(0, 16))
        pay_off.append(pos)
        pos += len(p)
    host = np.zeros(pos + 1, dtype=np.uint8)
    for o, p in zip(pay_off, payloads):
        host[o:o + len(p)] = p
    out_off, opos = [], 0
    for p in payloads:
        opos += int(rng.integers(0, 16))
        out_off.append(opos)
        opos += lzo_capacity(len(p))
    d_in = torch.from_numpy(host).cuda()
    d_out = torch.full((opos + 1,), 0xEE, dtype=torch.uint8, device="cuda")
    sizes = comp.compress(d_in.data_ptr(), pay_off, [len(p) for p in payloads], d_out.data_ptr(), out_off)
    out = d_out.cpu().numpy()
    return [out[o:o + int(s)].tobytes() for o, s in zip(out_off, sizes)]


def _check(payloads, got):
    for i, (p, g) in enumerate(zip(payloads, got)):
        want = lzo_oracle.frame(p.tobytes())
        assert g == want, f"payload {i}: {len(p)} bytes, got {len(g)} framed bytes, want {len(want)}"


def test_lzo_edge_sizes_every_kind(torch_cuda, comp):
    rng = np.random.default_rng(1)
    payloads = [payload(k, n, 100 + i) for i, (n, k) in enumerate((n, k) for n in EDGE_SIZES for k in KINDS)]
    _check(payloads, _compress(torch_cuda, comp, payloads, rng))


def test_lzo_random_sizes(torch_cuda, comp):
    # ZC_LZO_SWEEP=<rounds> repeats this with other seeds (a longer run by hand)
    import os
    for rnd in range(int(os.environ.get("ZC_LZO_SWEEP", "1"))):
        rng = np.random.default_rng(2 + 1000 * rnd)
        payloads = [payload(KINDS[i % len(KINDS)], int(rng.integers(0, 3_000_000)), 200 + i + 100000 * rnd)
                    for i in range(48)]
        got = _compress(torch_cuda, comp, payloads, rng)
        _check(payloads, got)
    for p, g in zip(payloads[:12], got):  # and the library decompresses them
        assert lzo_oracle.unframe(g) == p.tobytes()


def test_lzo_repeated_calls_reuse_dictionaries(torch_cuda, comp):
    # the dictionaries are not cleared between calls (generation tags): a
    # second call over different bytes must not see the first call's entries
    rng = np.random.default_rng(3)
    for rep in range(3):
        payloads = [payload(k, 150000 + 977 * rep, 300 + 10 * rep + j) for j, k in enumerate(KINDS)]
        _check(payloads, _compress(torch_cuda, comp, payloads, rng))


def test_lzo_compress_host(torch_cuda, comp):
    payloads = [payload(k, 70000 + 4099 * i, 400 + i) for i, k in enumerate(KINDS)] + [np.zeros(0, np.uint8)]
    _check(payloads, comp.compress_host([p.tobytes() for p in payloads]))


def test_lzo_256mib_text_bundles(torch_cuda, comp):
    rng = np.random.default_rng(4)
    data = payload("text", 256 << 20, 5)
    n = 0x200000
    payloads = [data[i:i + n] for i in range(0, len(data), n)]
    _check(payloads, _compress(torch_cuda, comp, payloads, rng))


@pytest.mark.parametrize("spec_kind", ["mixed", "text"])
def test_bundles_of_a_chunked_stream(torch_cuda, comp, spec_kind):
    """stream -> records (GPU) -> NEW chunks the index accepts -> Writer::add
    bundles -> device gather -> lzo1x_1: every bundle equals the oracle's."""
    from zbackup_amd import ZC_CHUNK_NEW, BackupCreator
    from zbackup_amd.bundle import lzo_capacity, plan_bundles
    torch = torch_cuda
    W = 65536
    if spec_kind == "mixed":  # text, random, a repeat of both, zeros
        a, b = payload("text", 9 << 20, 11), payload("random", 7 << 20, 12)
        data = np.concatenate([a, b, a[3:5 << 20], np.zeros(3 << 20, np.uint8), b[:4 << 20], payload("runs", 5 << 20, 13)])
    else:
        data = payload("text", 40 << 20, 14)
    want_recs = oracle.chunk_array(data, W)
    d = torch.from_numpy(data).cuda()
    with BackupCreator(chunk_max_size=W, sha1=True) as bc:
        bc.chunk_device(d.data_ptr(), len(data))
        recs = bc.records()
    assert len(recs) == len(want_recs)
    for f in ("offset", "size", "kind", "rolling", "sha1"):
        assert np.array_equal(recs[f], want_recs[f]), f
    # Writer::add: saved chunks whose id the index does not hold yet
    seen, offs, sizes = set(), [], []
    for r in recs:
        if r["kind"] != ZC_CHUNK_NEW:
            continue
        cid = bytes(r["sha1"]) + int(r["rolling"]).to_bytes(8, "little")
        if cid in seen:
            continue
        seen.add(cid)
        offs.append(int(r["offset"]))
        sizes.append(int(r["size"]))
    bundle_of, nb = plan_bundles(sizes)
    saved = [r for r in want_recs if r["kind"] == ZC_CHUNK_NEW]
    want_b = lzo_oracle.writer_bundles(
        [(bytes(r["sha1"]) + int(r["rolling"]).to_bytes(8, "little"), int(r["size"])) for r in saved])
    assert nb == len(want_b) and nb > 4
    d_payload = torch.empty(max(sum(sizes), 1), dtype=torch.uint8, device="cuda")
    comp.gather(d.data_ptr(), offs, sizes, d_payload.data_ptr())
    pay_size = np.bincount(bundle_of, weights=sizes, minlength=nb).astype(np.uint64)
    pay_off = np.concatenate([[0], np.cumsum(pay_size)[:-1]]).astype(np.uint64)
    out_off = np.concatenate([[0], np.cumsum([lzo_capacity(int(s)) for s in pay_size])]).astype(np.uint64)
    d_out = torch.empty(int(out_off[-1]), dtype=torch.uint8, device="cuda")
    out_size = comp.compress(d_payload.data_ptr(), pay_off, pay_size, d_out.data_ptr(), out_off[:-1])
    out = d_out.cpu().numpy()
    for b, members in enumerate(want_b):
        pl = b"".join(data[int(saved[m]["offset"]):int(saved[m]["offset"]) + int(saved[m]["size"])].tobytes()
                      for m in members)
        got = out[int(out_off[b]):int(out_off[b]) + int(out_size[b])].tobytes()
        assert got == lzo_oracle.frame(pl), f"bundle {b}"


def test_adler32_of_device_ranges(torch_cuda, comp):
    """zc_adler32 == zlib.adler32 (the library Adler32 wraps, adler32.hh) for
    ranges of every alignment and length, incl. empty, a few bytes inside one
    16-byte slot, and a 96 MiB range; and of framed bundle outputs."""
    import zlib
    rng = np.random.default_rng(6)
    host = rng.integers(0, 256, 100 << 20, dtype=np.uint8)
    host[5 << 20:7 << 20] = 0xFF  # long runs of the largest byte (the sums' worst case)
    d = torch_cuda.from_numpy(host).cuda()
    offs, lens = [], []
    for ln in [0, 1, 2, 3, 15, 16, 17, 31, 33, 255, 4096, 65537, 2097152, 3000001]:
        for _ in range(3):
            o = int(rng.integers(0, len(host) - ln - 1))
            offs.append(o)
            lens.append(ln)
    offs += [3, 5 << 20, 0]
    lens += [12, 2 << 20, 96 << 20]
    got = comp.adler32(d.data_ptr() + 1, offs, lens)  # an unaligned base pointer: range = host[o + 1 ..]
    for o, ln, g in zip(offs, lens, got):
        assert int(g) == zlib.adler32(host[o + 1:o + 1 + ln].tobytes()), (o, ln)
    payloads = [payload(k, 300000 + 7 * i, 500 + i) for i, k in enumerate(KINDS)]
    framed = _compress(torch_cuda, comp, payloads, rng)
    blob = np.frombuffer(b"".join(framed), dtype=np.uint8)
    dd = torch_cuda.from_numpy(blob.copy()).cuda()
    fo = np.concatenate([[0], np.cumsum([len(f) for f in framed])[:-1]])
    got = comp.adler32(dd.data_ptr(), fo, [len(f) for f in framed])
    assert [int(g) for g in got] == [zlib.adler32(f) for f in framed]


def test_lzo_many_tiny_bundles(torch_cuda, comp):
    """5,000 payloads of 0-300 bytes in one call (bundles below one 48 KiB
    block, at and around the 20/21-byte edge, most without any match)."""
    rng = np.random.default_rng(7)
    sizes = rng.integers(0, 300, 5000)
    sizes[:64] = np.arange(64)
    payloads = [payload(KINDS[i % len(KINDS)], int(n), 700 + i) for i, n in enumerate(sizes)]
    _check(payloads, _compress(torch_cuda, comp, payloads, rng))


def test_lzo_short_last_blocks_and_random_sweep(torch_cuda, comp):
    """Every short last block (49152 * k + 21 .. 40, k = 1, 2) for every kind,
    and 300 payloads of random size up to 200 KB: the block loop's guard on
    short blocks, with the pending literals the full blocks leave."""
    rng = np.random.default_rng(8)
    payloads = [payload(kind, 49152 * k + r, 800 + 100 * k + r + 1000 * i)
                for i, kind in enumerate(KINDS) for k in (1, 2) for r in range(21, 41)]
    payloads += [payload(KINDS[i % len(KINDS)], int(rng.integers(0, 200000)), 5000 + i) for i in range(300)]
    _check(payloads, _compress(torch_cuda, comp, payloads, rng))


def test_lzo_call_split_into_batches(torch_cuda, comp, monkeypatch):
    """A call larger than one device batch (normally 2^18 blocks = 12 GiB)
    runs batch after batch, each a new dictionary generation: here batches of
    at most 5 blocks (ZC_LZO_BATCH_BLOCKS), payloads of 0-400 KB."""
    monkeypatch.setenv("ZC_LZO_BATCH_BLOCKS", "5")
    rng = np.random.default_rng(9)
    payloads = [payload(KINDS[i % len(KINDS)], int(rng.integers(0, 400000)), 900 + i) for i in range(40)]
    _check(payloads, _compress(torch_cuda, comp, payloads, rng))


@pytest.mark.parametrize("shared", [False, True])
def test_compressor_threads_beside_a_feed(torch_cuda, shared):
    # Bundle::Creator::write runs on several compressor threads at once
    # (chunk_storage.cc:133-141,175) while the main thread is inside
    # handleMoreData.  Own contexts (shared=False, GpuLzoBundleCompressor's pool)
    # run concurrently; one context shared by every thread (shared=True) is
    # serialized by the per-context lock.  Every frame equals liblzo2's and the
    # fed stream's records equal the oracle's.
    import threading

    from zbackup_amd import BackupCreator
    from zbackup_amd.bundle import BundleCompressor
    W = 4096
    data = oracle.gen("R5:9000000,C100:3000000,Z:500000,R6:4000000")
    want = oracle.chunk(data, W)
    payloads = [[payload(k, int(s), 31 * t + i) for i, (k, s) in
                 enumerate(zip(KINDS * 2, [2097152, 700001, 49173, 1234567, 98304, 2000000, 5, 333333, 49152,
                                           1 << 20, 77777, 600000]))] for t in range(4)]
    shared_comp = BundleCompressor() if shared else None
    errors, results = [], [None] * 4

    def compressor(t):
        try:
            comp = shared_comp or BundleCompressor()
            out = []
            for _ in range(3):
                out = comp.compress_host([p.tobytes() for p in payloads[t]])
            results[t] = out
            if not shared:
                comp.close()
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(repr(e))

    threads = [threading.Thread(target=compressor, args=(t,)) for t in range(4)]
    with BackupCreator(W, window=8 * W + (16 << 20)) as bc:
        for th in threads:
            th.start()
        pos = 0
        while pos < data.size:  # the main thread feeds meanwhile
            buf = bc.get_input_buffer()
            take = min(bc.get_input_buffer_size(), 1 << 20, data.size - pos)
            np.frombuffer(buf, dtype=np.uint8, count=take)[:] = data[pos:pos + take]
            bc.handle_more_data(take)
            pos += take
        bc.finish()
        got = bc.record_tuples()
        for th in threads:
            th.join()
    if shared_comp is not None:
        shared_comp.close()
    assert not errors, errors
    assert got == want
    for t in range(4):
        _check(payloads[t], results[t])
