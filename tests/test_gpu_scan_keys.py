"""GPU parity of the grid-chunk keys the scan writes (GridKeysOut).

With W a multiple of the 4 KiB lane span that divides the 256 KiB wave-tile,
the scan folds each grid chunk's span digests into its RollingHash digest at
the wave-tile's end (2^k lanes per chunk, k = 0 .. 6) and the chunk-metadata
kernel computes only the keys of chunks in the stream's partial last tile.
Every record's rolling hash must equal the oracle's (rolling_hash.cc digest,
backup_creator.cc:127-141), for each such W, through the device path and
zc_chunk_host's segmented scan, with and without SHA-1 ids -- and for W the
scan does not handle, through the metadata kernel alone.
"""
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


# three full 2 MiB scan tiles and more, a duplicated range (DUP records whose
# keys come from the scan), zeros, and a partial last tile
SPEC = "R21:5000000,C777:2500000,Z:300000,R22:1111111"


@pytest.mark.parametrize("W", [4096, 8192, 16384, 32768, 65536, 131072, 262144, 12288, 1 << 20])
@pytest.mark.parametrize("sha1", [False, True])
def test_scan_written_grid_keys_vs_oracle(torch_cuda, W, sha1):
    from zbackup_amd import BackupCreator
    data = oracle.gen(SPEC)
    assert data.size > 4 * (2 << 20) and data.size % (2 << 20)
    want = oracle.chunk(data, W)
    if not sha1:
        want = [(k, o, s, h, "0" * 32 if k != "B" else sha) for (k, o, s, h, sha) in want]
    t = torch_cuda.from_numpy(data).to("cuda")
    with BackupCreator(W, sha1=sha1) as bc:
        bc.chunk_device(t.data_ptr(), data.size)
        assert bc.record_tuples() == want
        # the same again on the context (its index now holds the chunks)
        bc.forget_stream_chunks()
        bc.chunk_device(t.data_ptr(), data.size)
        assert bc.record_tuples() == want
    host = torch_cuda.from_numpy(data).pin_memory()
    with BackupCreator(W, sha1=sha1) as bc:
        bc.chunk_host(host.data_ptr(), data.size)
        assert bc.record_tuples() == want
