"""Multi-GPU path on CPU: bench.py's replica logic under a world-size-2 gloo
group (BASELINE.json configs[3]: independent buffers, one per GPU, no
data-path collective).  Each rank chunks its own stream (seed = base + rank)
with the oracle as a stand-in for the device engine; the job time is the max
over ranks and the value counts every rank's bytes."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from oracle import oracle

BASE_SEED = 2024
N = 1 << 20
W = 4096


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = oracle.splitmix64(N, bench.rank_seed(BASE_SEED, rank))
        recs = oracle.chunk(data, W)
        elapsed = 0.25 * (rank + 1)  # a deterministic per-rank "time"
        job = bench.job_elapsed(elapsed, world)
        gathered = [None] * world
        dist.all_gather_object(gathered, (rank, elapsed, job, recs))
        if rank == 0:
            import pickle
            with open(os.path.join(out_dir, "result.pkl"), "wb") as f:
                pickle.dump(gathered, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_replicas_gloo(tmp_path):
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    import pickle
    with open(tmp_path / "result.pkl", "rb") as f:
        gathered = pickle.load(f)
    assert [g[0] for g in gathered] == [0, 1]
    # the job time is the slowest rank's, on every rank
    assert all(g[2] == pytest.approx(0.5) for g in gathered)
    # independent streams: each rank's records equal a single-process run of
    # its own seed, and the two streams differ
    for rank, _, _, recs in gathered:
        want = oracle.chunk(oracle.splitmix64(N, BASE_SEED + rank), W)
        assert recs == want
        assert len(recs) == N // W and all(r[0] == "N" for r in recs)
    assert gathered[0][3] != gathered[1][3]
    # whole-job value: every rank's bytes over the job time
    assert bench.job_value(N, world, 3, 0.5) == pytest.approx(N * 2 * 3 / 0.5 / 2**30)


def test_single_rank_helpers():
    assert bench.rank_seed(7, 0) == 7 and bench.rank_seed(7, 3) == 10
    assert bench.job_elapsed(1.5, 1) == 1.5
