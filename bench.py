#!/usr/bin/env python3
"""Benchmark: device-resident rolling-hash chunking GiB/s (BASELINE.json metric).

A step = one full pass of the engine (zc_chunk_device: scan, grid keys, anchor
probe, verification, boundary resolution, records to host) over one resident
8 GiB synthetic stream.  Workload = BASELINE.json configs[1] (C2: 8 GiB seeded
random bytes, W = chunk.max_size = 65536).  Multi-GPU: one process per GPU,
each with its own independent 8 GiB stream (seed = base + rank), no
data-path collective (configs[3]); the value is the sum of bytes over the max
of the per-rank times.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c5] [--e2e]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

W64 = 65536
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
CONFIGS = {
    "c2": "C2: 1 x 8 GiB seeded random stream, device-resident, W=65536",
    "c3": "C3: 8 GiB = two copies of a 4 GiB seeded random block, W=65536",
    "c5": "C5: 8 GiB all-zero stream, W=65536",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--gib", type=float, default=8.0, help="stream size per GPU")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--cpu-sample-mib", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e", action="store_true", help="also time host(pinned)->HBM + chunking")
    ap.add_argument("--sha1", action="store_true",
                    help="records carry SHA-1 chunk ids (ZC_FLAG_SHA1; the full chunk_to_emit content)")
    return ap.parse_args()


def cpu_baseline(sample_bytes, seed):
    """The oracle port (per-byte rotate + identity-hash hash_map probe + SHA-1
    per chunk, single thread) on the first `sample_bytes` of the same stream."""
    from oracle import oracle
    data = oracle.splitmix64(sample_bytes, seed)
    t0 = time.perf_counter()
    recs = oracle.chunk(data, W64)
    dt = time.perf_counter() - t0
    return {"value": round(sample_bytes / dt / 2**30, 5), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"first {sample_bytes >> 20} MiB of the C2 stream (seed {seed}), "
                      f"{len(recs)} records in {dt:.2f} s, oracle/zc_oracle.cpp single thread",
            "chunks_per_s": round(len(recs) / dt, 1)}


def rank_seed(base, rank):
    """Replica streams are independent: rank r chunks the stream seeded base + r
    (BASELINE.json configs[3]: one 8 GiB buffer per GPU, seed = base + gpu)."""
    return base + rank


def job_elapsed(elapsed, world):
    """Whole-job time of the timed region = the max over ranks (each rank
    brackets its own steps with a barrier and a device sync)."""
    if world <= 1:
        return elapsed
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_value(n_bytes_per_rank, world, steps, elapsed):
    """Aggregate GiB/s: the bytes every rank chunked over the job time."""
    return n_bytes_per_rank * world * steps / elapsed / 2**30


def pmc_traffic(n_bytes):
    """HBM bytes per zc_scan launch from the committed rocprofv3 --pmc summary
    (FETCH_SIZE doubled per the gfx950 correction + WRITE_SIZE), if present."""
    path = os.path.join(ROOT, "profiles", "scan_pmc.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        if int(d.get("bytes", -1)) != int(n_bytes):
            return None
        return d.get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)

    from zbackup_amd import BackupCreator, fill_splitmix64

    n = int(args.gib * 2**30)
    buf = torch.empty(n, dtype=torch.uint8, device=f"cuda:{local}")
    seed = rank_seed(args.seed, rank)
    if args.config == "c5":
        buf.zero_()
    elif args.config == "c3":
        fill_splitmix64(buf.data_ptr(), n // 2, seed, local)
        buf[n // 2:].copy_(buf[: n // 2])
    else:
        fill_splitmix64(buf.data_ptr(), n, seed, local)
    torch.cuda.synchronize()

    # with --sha1 a context's chunks join its index (Writer::add ->
    # ChunkIndex::addChunk), so chunking the same stream again would measure
    # an incremental backup of identical data: each step first drops them
    # (zc_forget_stream_chunks), so every step is a first backup of the stream
    # against the index a fresh ZBackup instance loads, on warm buffers
    bc = BackupCreator(W64, device=local, sha1=args.sha1, timing=True)

    def step():
        if args.sha1:
            bc.forget_stream_chunks()
        bc.chunk_device(buf.data_ptr(), n)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    for k in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    scan_ms = []
    for k in range(args.steps):
        step()
        scan_ms.append(bc.scan_ms())
    barrier()
    elapsed = time.perf_counter() - t0
    st = bc.stats()
    nrec = len(bc.records())
    elapsed = job_elapsed(elapsed, world)
    ms_step = elapsed / args.steps * 1e3
    value = job_value(n, world, args.steps, elapsed)

    e2e = None
    if args.e2e:
        # the stream starts in (pinned) host memory, as in zutils.cc:100-124
        host = buf.cpu().pin_memory()
        reps = 3
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(reps):
            buf.copy_(host, non_blocking=True)
        torch.cuda.synchronize()
        h2d = n * reps / (time.perf_counter() - t1) / 2**30
        t1 = time.perf_counter()
        for _ in range(reps):
            buf.copy_(host, non_blocking=True)
            torch.cuda.synchronize()
            bc.chunk_device(buf.data_ptr(), n)
        serial = n * reps / (time.perf_counter() - t1) / 2**30
        t1 = time.perf_counter()
        for _ in range(reps):
            bc.chunk_host(host.data_ptr(), n)
        overlapped = n * reps / (time.perf_counter() - t1) / 2**30
        e2e = {"GiB_per_s": round(overlapped, 3), "path": "pinned host buffer -> zc_chunk_host: 64 MiB H2D "
               "segments on a side stream, each scanned as it lands, then resolve + records to host",
               "serial_GiB_per_s": round(serial, 3), "h2d_only_GiB_per_s": round(h2d, 3)}
        del host

    if rank == 0:
        scan_avg = sum(scan_ms) / len(scan_ms)
        achieved = n / (scan_avg * 1e-3) / 1e9
        out = {
            "metric": "rolling-hash chunking GiB/s (device-resident)",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64-seeded bytes generated in HBM)",
            "config": {"workload": CONFIGS[args.config], "stream_bytes_per_gpu": n,
                       "chunk_max_size": W64, "parallelism": f"replicas x{world} (independent streams)",
                       "chunk_ids": "SHA-1 prefix + rolling hash" if args.sha1 else "rolling hash"},
            "chunks_per_s": round(nrec * world * args.steps / elapsed, 1),
            "records_per_stream": nrec,
            "roofline": {"bound": "hbm", "kernel": "zc_scan_kernel", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": pmc_traffic(n), "bytes_per_launch": n,
                         "scan_ms_avg": round(scan_avg, 4)},
            "stages": {"scan_ms": round(st["scan_ms"], 4), "resolve_ms": round(st["resolve_ms"], 4),
                       "total_ms": round(st["total_ms"], 4), "anchors": st["anchors"],
                       "candidates": st["candidates"], "epochs": st["epochs"],
                       "meta_ms": round(st["meta_ms"], 4), "probe_ms": round(st["probe_ms"], 4),
                       "fscan_ms": round(st["fscan_ms"], 4), "walk_ms": round(st["walk_ms"], 4),
                       "finalize_ms": round(st["finalize_ms"], 4), "fbatch_ms": round(st["fbatch_ms"], 4)},
        }
        if e2e:
            out["end_to_end"] = e2e
        if world == 1 and not args.no_cpu_baseline and args.config == "c2":
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample_mib << 20, seed)
        print(json.dumps(out), flush=True)
    bc.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
