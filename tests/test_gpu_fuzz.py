"""Randomized GPU parity sweep of the chunking engine (records, including SHA-1
prefixes, vs the oracle's BackupCreator restatement, backup_creator.cc:56-272,
chunk_index.cc:119-202): 400 seeded streams of 2-14 segments -- random bytes,
zero runs, repeated bytes, copies of earlier ranges (so copies of copies) and
short pieces -- at random chunk sizes W in [64, 70000] besides the usual ones,
device-resident; every fifth also seeded with the ids of another stream's
chunks (ChunkIndex::loadIndex), every seventh fed through the host feed in
ragged pieces through the smallest window."""
import os

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


def _spec(rng, W):
    segs, n = [], 0
    for _ in range(int(rng.integers(2, 15))):
        t = int(rng.integers(0, 6))
        u = rng.random()
        ln = int(rng.integers(1, 300)) if u < 0.25 else int(rng.integers(1, (12 if u > 0.9 else 4) * W + 2))
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


# ZC_FUZZ_SEEDS / ZC_FUZZ_BASE widen or move the sweep (a longer run by hand)
@pytest.mark.parametrize("seed", range(int(os.environ.get("ZC_FUZZ_SEEDS", "400"))))
def test_fuzz_vs_oracle(torch_cuda, seed):
    from zbackup_amd import BackupCreator
    seed += int(os.environ.get("ZC_FUZZ_BASE", "0"))
    rng = np.random.default_rng(77000 + seed)
    W = int(rng.choice([64, 65, 127, 128, 255, 256, 999, 4095, 4096, 65536])) if seed % 2 else int(
        rng.integers(64, 70001))
    spec = _spec(rng, W)
    data = oracle.gen(spec)
    seeds = ()
    if seed % 5 == 0:
        other = oracle.gen(_spec(np.random.default_rng(88000 + seed), W))
        seeds = [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in oracle.chunk(np.concatenate([other, data[:W * 2]]), W)
                 if k == "N"]
    want = oracle.chunk(data, W, seeds=seeds)
    if seed % 7 == 0:
        with BackupCreator(W, seeds=seeds, sha1=True, window=8 * W + (16 << 20)) as bc:
            pos = 0
            while pos < data.size:
                buf = bc.get_input_buffer()
                take = min(int(rng.integers(1, 200000)), bc.get_input_buffer_size(), data.size - pos)
                np.frombuffer(buf, dtype=np.uint8, count=take)[:] = data[pos:pos + take]
                bc.handle_more_data(take)
                pos += take
            bc.finish()
            got = bc.record_tuples()
    else:
        t = torch_cuda.from_numpy(np.ascontiguousarray(data)).to("cuda") if data.size else torch_cuda.empty(
            0, dtype=torch_cuda.uint8, device="cuda")
        with BackupCreator(W, seeds=seeds, sha1=True) as bc:
            bc.chunk_device(t.data_ptr(), data.size)
            got = bc.record_tuples()
    assert got == want, (spec, W, len(seeds))
