"""GPU: the scan's content anchors against a numpy model of their definition
(zc_device.h: st(q) = sum_{j<16} b[q-2j] 2^j mod 2^16, q an anchor iff
(int16)st(q) >= anchor_lo and q >= 63).  Anchors are internal to the engine
(the reference has none), so this pins the per-byte packed form the scan
computes -- the fast path's tile end, the partial-tile kernel and the exact
rescan of overflowed wave-tiles -- to the one definition the records' parity
tests rely on.  Counts are exact (zc_stats.anchors)."""
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
    return torch


def _rate_inv(W):
    r = 16
    while r < 4096 and r * 2 <= W // 16:
        r *= 2
    return r


def model_anchors(data, W):
    """The anchor positions of `data` at chunk size W (a bool per position)."""
    b = data.astype(np.uint32)
    st = np.zeros(b.size, dtype=np.uint32)
    for j in range(16):
        st[2 * j:] += b[:b.size - 2 * j] << np.uint32(j)
    s16 = (st & 0xFFFF).astype(np.uint16).view(np.int16)
    lo = 0x8000 - 0x10000 // _rate_inv(W)
    hit = s16 >= lo
    hit[:63] = False
    return hit


def model_anchor_count(data, W):
    return int(model_anchors(data, W).sum())


def _device_anchors(torch, data, W):
    from zbackup_amd import BackupCreator
    t = torch.from_numpy(np.ascontiguousarray(data)).to("cuda")
    with BackupCreator(W, sha1=False) as bc:
        bc.chunk_device(t.data_ptr(), data.size)
        return bc.stats()["anchors"]


@pytest.mark.parametrize("W", [65536, 4096, 256])
def test_anchor_count_random_vs_model(torch_cuda, W):
    # whole 2 MiB scan tiles plus a partial last tile (the tail kernel)
    data = oracle.gen("R21:37000011")
    assert _device_anchors(torch_cuda, data, W) == model_anchor_count(data, W)


def test_anchor_count_constant_runs_hold_none(torch_cuda):
    # a run of one repeated byte never anchors (st = 0 or -c), at the densest
    # rate: every anchor lies in the 31 bytes after a change of byte value
    data = np.repeat(np.arange(256, dtype=np.uint8), 65536)
    hit = model_anchors(data, 128)
    assert not np.any(hit.reshape(256, 65536)[:, 31:])
    assert _device_anchors(torch_cuda, data, 128) == int(hit.sum())


def test_anchor_count_dense_overflow_vs_model(torch_cuda):
    # a 16-byte pattern with an anchor in every period: the wave-tiles'
    # lists and pool shares overflow, the exact rescan (zc_anchor_rescan)
    # counts them, mixed with random bytes the fast path takes
    from tests.test_gpu_parity import _dense_anchor_pattern
    pat = _dense_anchor_pattern(65536)
    body = np.tile(pat, (3 << 20) // pat.size)
    data = np.concatenate([oracle.gen("R9:1500000"), body, oracle.gen("R10:777777")])
    assert _device_anchors(torch_cuda, data, 65536) == model_anchor_count(data, 65536)
