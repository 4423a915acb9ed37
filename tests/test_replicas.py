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
    assert bench.job_gather(2.5, 1) == [2.5]
    env = bench.child_env({"PATH": "/bin"}, 3, 8, 1234)
    assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"], env["MASTER_PORT"]) == ("3", "3", "8", "1234")
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["PATH"] == "/bin"


@pytest.mark.timeout(300)
def test_bench_self_launches_ranks_on_cpu():
    """`python bench.py --gpus 2` with no torchrun environment starts two rank
    processes itself (bench.launch); --dry-run has each rank chunk its own
    seeded stream with the oracle, so the launch, the gloo bookkeeping (max
    over ranks, per-rank gathers) and rank 0's one JSON line run on CPU."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    out = subprocess.run([sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py"),
                          "--gpus", "2", "--dry-run", "--gib", str(2 * W / 2**30 * 64), "--steps", "2",
                          "--warmup", "1"], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["dry_run"] and d["n_gpus"] == 2 and d["steps"] == 2 and d["value"] > 0
    assert d["seeds"] == [2024, 2025]
    n = int(2 * W * 64)
    assert d["records_per_rank"] == [n // 65536 + (n % 65536 > 0)] * 2
    # independent streams: the ranks' first chunk keys differ
    assert d["first_key_per_rank"][0] != d["first_key_per_rank"][1]


def test_bench_rejects_world_size_mismatch():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py"),
                          "--gpus", "2", "--dry-run"], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr
