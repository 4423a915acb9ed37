"""GPU parity of the exact-hash screen (keys without content anchors: all-zero
and other low-entropy chunks, and the static index of earlier backups).

The screen runs on two kernels -- zc_fscan_staged over whole 512 KiB screen
wave-tiles, zc_fscan (lane per KiB) over the head and tail of the stream and
over wave-tiles whose runs overflow -- so these streams are several MiB long,
use chunk sizes W whose -W mod 16 covers every funnel shift of the staged
kernel's out-byte stream, and start new epochs mid-stream (grid-shifting
matches move p_start inside a wave-tile).  Every case is checked against the
oracle and against the lane-per-KiB screen alone (ZC_FLAG_NO_STAGED_SCREEN)."""
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


def _device(torch, data, W, seeds=(), staged=True):
    from zbackup_amd import BackupCreator
    t = torch.from_numpy(np.ascontiguousarray(data)).to("cuda")
    with BackupCreator(W, seeds=seeds, sha1=True, staged_screen=staged) as bc:
        bc.chunk_device(t.data_ptr(), data.size)
        return bc.record_tuples()


def _check(torch, data, W, seeds=()):
    want = oracle.chunk(data, W, seeds=seeds)
    got = _device(torch, data, W, seeds)
    assert got == want
    assert _device(torch, data, W, seeds, staged=False) == want
    return want


# -W mod 16 = 0, 12, 8, 15, 4, 3, 1, 10, 11: the (Q, s) shapes of the out-byte funnel
@pytest.mark.parametrize("W", [65536, 4100, 1000, 65537, 300, 77773, 143, 65542, 1029])
def test_zero_runs_vs_oracle(torch_cuda, W):
    # the stream starts with W zero bytes: grid chunk 0 is all zero (no
    # anchor), so every later all-zero window is found by the screen only
    spec = (f"Z:{W + 3000000},R{W}:700001,Z:2500000,B9:40000,Z:1800000,C17:900000,"
            f"Z:{3 * W + 5},R{W + 1}:333,Z:1200000")
    data = oracle.gen(spec)
    recs = _check(torch_cuda, data, W)
    assert sum(1 for r in recs if r[0] == "D") > 10


@pytest.mark.parametrize("W", [4096, 65536])
def test_constant_byte_chunks_vs_oracle(torch_cuda, W):
    # chunks of one repeated byte value (two distinct anchorless keys), with
    # random bursts that shift the grid (new epochs start mid wave-tile)
    spec = (f"B200:{2 * W},B17:{2 * W},R1:100003,B200:2000000,R2:77,B17:1500000,"
            f"R3:1000,B200:{W + 11},B17:1000000,R4:5")
    data = oracle.gen(spec)
    recs = _check(torch_cuda, data, W)
    assert sum(1 for r in recs if r[0] == "D") > 10


def test_many_runs_per_span_overflow(torch_cuda):
    # zero runs slightly longer than W between short random bursts: every
    # 8 KiB lane span holds many separate hit runs, so the staged kernel's
    # wave-tiles overflow their run slots and are redone by zc_fscan
    # (every zero window after a burst is a grid-shifting match: ~4500 epochs,
    # each bounded by its horizon)
    W = 200
    parts = [f"Z:{W + 50}"]
    for i in range(4500):
        parts.append(f"R{i + 7}:{7 + i % 13}")
        parts.append(f"Z:{W + 40 + i % 37}")
    data = oracle.gen(",".join(parts))
    assert data.size > (1 << 20)
    _check(torch_cuda, data, W)


@pytest.mark.parametrize("nseeds,nfake", [(1, 0), (3, 0), (9, 0), (40, 0), (40, 300), (40, 1900), (40, 2100)])
def test_static_index_vs_oracle(torch_cuda, nseeds, nfake):
    # the static index (ChunkIndex::loadIndex of earlier backups) has no
    # anchors on our side: its keys go through the screen -- compared
    # directly (1..4 keys), or the 2^17-bit key map confirmed by 16 compares
    # (5..16) or a binary search in LDS (17..2048), or the map alone (more) --
    # and hits are confirmed by SHA-1 (chunk_index.cc:130-139); `nfake` keys
    # of chunks that do not occur widen the index
    W = 65536
    old = oracle.gen("R901:3000000")
    old_recs = oracle.chunk(old, W)
    seeds = [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in old_recs if k == "N" and s == W][:nseeds]
    rng = np.random.default_rng(nfake)
    seeds += [(rng.bytes(16), int(x), W) for x in rng.integers(1, 2**63, nfake, dtype=np.int64)]
    # the new backup holds the old content at a shifted offset, plus fresh bytes
    data = np.concatenate([oracle.gen("R902:1234567"), old[: 40 * W], oracle.gen("R903:2100003"),
                           old[5 * W: 9 * W], oracle.gen("Z:700000")])
    recs = _check(torch_cuda, data, W, seeds)
    assert sum(1 for r in recs if r[0] == "D") >= min(nseeds, 4)
