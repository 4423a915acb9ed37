#!/usr/bin/env python3
"""Benchmark: device-resident rolling-hash chunking GiB/s (BASELINE.json metric).

A step = one full pass of the engine (zc_chunk_device: scan, grid keys, anchor
probe, verification, boundary resolution, records to host) over one resident
8 GiB synthetic stream.  Workload = BASELINE.json configs[1] (C2: 8 GiB seeded
random bytes, W = chunk.max_size = 65536).  Multi-GPU (configs[3], C4): one
process per GPU, each with its own independent 8 GiB stream (seed = base +
rank), no data-path collective; the value is the sum of bytes over the max of
the per-rank times.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c5]

With --gpus N > 1 and no torchrun environment, this process starts N rank
processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set per child)
before anything touches a GPU, and exits with their status; under
`torch.distributed.run` each rank reads those variables from the environment.

Besides the headline `value` (chunk ids = rolling hash, as BASELINE's metric
names), the same line carries, driver-observed:
  value_c3, value_c5
               BASELINE configs[2] and [4] (C3: two copies of 4 GiB; C5: all
               zeros) in the headline mode, timed as the headline
  value_sha1   the same streams with complete ChunkIds (SHA-1 prefix + rolling
               hash on every record: backup_creator.cc:130-131, chunk_id.cc:19-27)
  end_to_end   the stream starting in pinned host memory (zc_chunk_host: H2D
               overlapped with the scan), the zutils.cc:100-124 path
  bundle_lzo   the bundle writer offload: saved chunks bundled (Writer::add),
               gathered and lzo1x_1-compressed on the GPU (bundle.cc:30-36,
               96-155), with liblzo2 on one core beside it
  static_index the first GiB against 300 K and 2 M ids known by value only
               (an index loaded from earlier backups, chunk_index.cc:26-79)
"""
import argparse
import json
import os
import socket
import subprocess
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
    "edit": "edited duplicate: 4 GiB seeded random, then the same 4 GiB with 1-100 random bytes inserted "
            "every 1 MiB (~4096 grid shifts), 8 GiB in all, W=65536",
}
C4 = "C4: N x 8 GiB independent seeded random streams, one per GPU, W=65536"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--gib", type=float, default=8.0, help="stream size per GPU")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--cpu-sample-mib", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-lzo", dest="lzo", action="store_false",
                    help="skip the bundle_lzo (bundle writer offload) pass")
    ap.add_argument("--no-extras", action="store_true",
                    help="headline only (skip the value_sha1 and end_to_end passes)")
    ap.add_argument("--sha1-steps", type=int, default=5)
    ap.add_argument("--sha1", action="store_true",
                    help="the headline itself with SHA-1 chunk ids (ZC_FLAG_SHA1)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the launch and rank bookkeeping: each rank chunks its "
                         "stream with the oracle instead of the GPU (no measurement)")
    return ap.parse_args(argv)


# --------------------------------------------------------------------------
# replica helpers (pure; tests/test_replicas.py runs them under gloo)

def rank_seed(base, rank):
    """Replica streams are independent: rank r chunks the stream seeded base + r
    (BASELINE.json configs[3]: one 8 GiB buffer per GPU, seed = base + gpu)."""
    return base + rank


def job_max(x, world):
    """Max of a per-rank float over the job (gloo all-reduce; identity at N=1)."""
    if world <= 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_elapsed(elapsed, world):
    """Whole-job time of the timed region = the max over ranks (each rank
    brackets its own steps with a barrier and a device sync)."""
    return job_max(elapsed, world)


def job_gather(x, world):
    """Per-rank values, rank order (gloo all-gather; [x] at N=1)."""
    if world <= 1:
        return [x]
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    out = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


def job_value(n_bytes_per_rank, world, steps, elapsed):
    """Aggregate GiB/s: the bytes every rank chunked over the job time."""
    return n_bytes_per_rank * world * steps / elapsed / 2**30


def child_env(base_env, rank, world, port):
    """Environment of rank `rank` of a self-launched N-process job."""
    env = dict(base_env)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(argv, world, script=None, extra_env=None):
    """Start `world` rank processes of `script` (this file) with `argv`, one per
    GPU, and wait for all of them.  Nothing here touches a GPU: each child
    initialises its own device.  Returns the worst exit status."""
    script = script or os.path.abspath(__file__)
    port = free_port()
    base = dict(os.environ)
    if extra_env:
        base.update(extra_env)
    procs = [subprocess.Popen([sys.executable, script] + list(argv), env=child_env(base, r, world, port))
             for r in range(world)]
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


# --------------------------------------------------------------------------

def cpu_sample_bytes(sample_bytes, seed, config):
    """The first `sample_bytes` of the config's stream, on the host: C2 random;
    C3 a random block and its copy (sample_bytes / 2 each, the duplicated shape
    at sample scale); C5 zeros."""
    import numpy as np
    from oracle import oracle
    if config == "c5":
        return np.zeros(sample_bytes, dtype=np.uint8)
    if config == "c3":
        half = oracle.splitmix64(sample_bytes // 2, seed)
        return np.concatenate([half, half])
    return oracle.splitmix64(sample_bytes, seed)


def cpu_baseline(sample_bytes, seed, config="c2"):
    """The oracle port (per-byte rotate + identity-hash hash_map probe + SHA-1
    per chunk, single thread) on a sample of the same stream."""
    from oracle import oracle
    data = cpu_sample_bytes(sample_bytes, seed, config)
    t0 = time.perf_counter()
    recs = oracle.chunk(data, W64)
    dt = time.perf_counter() - t0
    return {"value": sample_bytes / dt / 2**30, "seconds": dt, "records": len(recs)}


def host_cpu():
    """The host CPU this process runs on: model name, logical CPUs the machine
    has and the ones this process may use (read at run time, on the GPU box)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = None
    return {"model": model, "nproc": os.cpu_count(), "usable_cpus": usable}


def committed_profile(build_id):
    """The newest committed profiles/rNN_scan_profile.json (tools/collect_profiles.py)
    of THIS build of libzchunk.so, or None: a profile of other sources is never
    quoted for this binary."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_scan_profile.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:
            continue
        if d.get("build_id") == build_id:
            d["path"] = os.path.relpath(path, ROOT)
            return d
    return None


def pmc_traffic(prof, n_bytes):
    """HBM bytes per zc_scan launch from the build's committed rocprofv3 --pmc
    passes (FETCH_SIZE doubled per the gfx950 correction + WRITE_SIZE)."""
    if not prof or "pmc" not in prof or int(prof.get("bytes", -1)) != int(n_bytes):
        return None
    return prof["pmc"]["hbm_bytes_per_launch"]


def rocprof_scan_ms(prof):
    """Average zc_scan_kernel duration (ms) under rocprofv3 --kernel-trace --stats
    of the C2 bench, from the build's committed summary."""
    if not prof or "rocprof" not in prof:
        return None, None
    return prof["rocprof"]["avg_ms"], prof["rocprof"]["source"]


def fill_edited(torch, buf, n, seed, local):
    """4 GiB seeded random block A, then A again in 1 MiB pieces each followed
    by 1-100 random bytes, cut at n bytes (the grid moves at every insertion)."""
    from zbackup_amd import fill_splitmix64
    import numpy as np
    half = n // 2
    fill_splitmix64(buf.data_ptr(), half, seed, local)
    rng = np.random.default_rng(seed)
    noise = torch.empty(1 << 20, dtype=torch.uint8, device=buf.device)
    fill_splitmix64(noise.data_ptr(), noise.numel(), seed + 7919, local)
    pos, src, piece = half, 0, 1 << 20
    while pos < n:
        ln = min(piece, half - src, n - pos)
        if ln <= 0:
            break
        buf[pos:pos + ln].copy_(buf[src:src + ln])
        pos += ln
        src += ln
        k = min(int(rng.integers(1, 101)), n - pos)
        o = int(rng.integers(0, noise.numel() - 128))
        buf[pos:pos + k].copy_(noise[o:o + k])
        pos += k
    if pos < n:
        fill_splitmix64(buf.data_ptr() + pos, n - pos, seed + 1, local)


def fill_stream(torch, buf, n, config, seed, local):
    from zbackup_amd import fill_splitmix64
    if config == "edit":
        fill_edited(torch, buf, n, seed, local)
    elif config == "c5":
        buf.zero_()
    elif config == "c3":
        fill_splitmix64(buf.data_ptr(), n // 2, seed, local)
        buf[n // 2:].copy_(buf[: n // 2])
    else:
        fill_splitmix64(buf.data_ptr(), n, seed, local)
    torch.cuda.synchronize()


# Untimed warm-up: at least W steps and at least this long.  The GPU takes
# ~10-20 ms of sustained load to reach its steady clock: in a kernel trace of
# the headline (round 4, 1.9 ms steps) the scan ran 1.86-1.91 ms for the
# first launches and settled at 1.53-1.58 ms from the eighth on.
MIN_WARMUP_S = 0.25


def timed_steps(torch, world, step, warmup, steps, min_warmup_s=MIN_WARMUP_S):
    """W untimed steps (repeated until min_warmup_s has passed), then K timed
    steps between barriers + device syncs; returns (job time = max over ranks,
    per-step scan ms of this rank)."""
    import torch.distributed as dist

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    t_w = time.perf_counter()
    for _ in range(warmup):
        step()
    if warmup > 0:
        while True:
            torch.cuda.synchronize()
            if time.perf_counter() - t_w >= min_warmup_s:
                break
            step()
    barrier()
    t0 = time.perf_counter()
    scan = [step() for _ in range(steps)]
    barrier()
    return job_elapsed(time.perf_counter() - t0, world), scan


def static_leg(torch, buf, local, ks=(300000, 2000000, 8000000), nbytes=1 << 30, reps=3):
    """The static index at repository scale: the first GiB of
    the stream against K random ids known by value only (ChunkIndex::loadIndex
    of earlier backups' index files, chunk_index.cc:26-79), rolling-hash ids;
    the best of `reps` whole zc_chunk_device calls after one warm-up."""
    import numpy as np
    from zbackup_amd import BackupCreator
    out = {"unit": "GiB/s", "stream_bytes": nbytes, "chunk_max_size": W64,
           "note": "two-level Bloom screen below 384 K ids, one-level with the in-kernel check table above (DESIGN 4.3); "
                   "8 M ids: a 512 GiB repository at W = 64 KiB"}
    for k in ks:
        rng = np.random.default_rng(k)
        keys = rng.integers(1, 2**63, k, dtype=np.int64).astype(np.uint64)
        shas = rng.integers(0, 256, (k, 16), dtype=np.uint8)
        with BackupCreator(W64, device=local, sha1=False, timing=True) as bc:
            bc.seed_index_arrays(shas, keys, W64)
            bc.chunk_device(buf.data_ptr(), nbytes)
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t1 = time.perf_counter()
                bc.chunk_device(buf.data_ptr(), nbytes)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t1)
            st = bc.stats()
        out[f"ids_{k}"] = {"value": round(nbytes / min(ts) / 2**30, 2), "ms": round(min(ts) * 1e3, 3),
                           "screen_ms": round(st["fscan_ms"], 3), "screen_runs": int(st["fscan_runs"])}
    return out


def synthetic_meta(rng, k, W=W64):
    """Anchor metadata of k chunks this process never holds (ids of a large
    repository's earlier backups): first anchor at a random offset >= 63, a key
    shaped like a real anchor's ({st(q-1), st(q)}, st(q) passing the anchor
    test at W's rate), a random fingerprint -- entries that fill the historic
    index and its probe filter but match no window of the stream."""
    import numpy as np
    from zbackup_amd import META_DTYPE, anchor_def
    rate = 4096  # anchor_rate_inv(65536)
    lo = 0x8000 - 0x10000 // rate
    m = np.zeros(k, dtype=META_DTYPE)
    m["size"] = W
    m["anchor_def"] = anchor_def(W)
    m["anchor"] = rng.integers(63, W, k, dtype=np.uint32)
    st_q = rng.integers(lo, 0x8000, k, dtype=np.uint32)
    m["gear"] = (st_q << 16) | rng.integers(0, 1 << 16, k, dtype=np.uint32)
    m["fingerprint"] = rng.integers(0, 2**63, k, dtype=np.int64).astype(np.uint64)
    return m


def seeded_repo_leg(torch, buf, n, seed, local, reps=4):
    """A non-empty repository opened by a new process (ChunkIndex::loadIndex,
    chunk_index.cc:26-79, zbackup_base.cc:87-100) with the content-anchor
    metadata an earlier backup exported beside its index (zc_export_chunk_meta ->
    zc_seed_index_meta, ABI 5): a fresh context seeded with the ids and metadata
    of an earlier context's backup of (i) the same 8 GiB stream (every chunk a
    duplicate) and (ii) a different one (none), then the C2 stream backed up with
    SHA-1 ids.  The first call on the context is timed apart (its buffers are
    made then); the value is the best of `reps` calls, each from the seeded
    index (zc_forget_stream_chunks drops what the previous call added)."""
    import numpy as np
    from zbackup_amd import BackupCreator
    out = {"unit": "GiB/s", "stream_bytes": n, "chunk_max_size": W64,
           "path": "ids + anchor metadata of an earlier context's backup -> zc_seed_index_meta on a fresh context "
                   "-> zc_chunk_device with SHA-1 ids (historic index probed by content anchors; no per-byte screen)"}
    other = torch.empty(n, dtype=torch.uint8, device=buf.device)
    fill_stream(torch, other, n, "c2", seed + 1000003, local)
    for label, src in (("same_stream", buf), ("other_stream", other)):
        with BackupCreator(W64, device=local, sha1=True) as a:
            a.chunk_device(src.data_ptr(), n)
            recs = a.records()
            meta = a.export_chunk_meta()
        ids = recs[recs["kind"] == 0]
        with BackupCreator(W64, device=local, sha1=True, timing=True) as b:
            b.seed_index_meta(ids["sha1"], ids["rolling"], ids["size"], meta)
            seeded = b.stats()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            b.chunk_device(buf.data_ptr(), n)
            torch.cuda.synchronize()
            first_ms = (time.perf_counter() - t1) * 1e3
            ts = []
            for _ in range(reps):
                b.forget_stream_chunks()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                b.chunk_device(buf.data_ptr(), n)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t1)
            st = b.stats()
            kinds = b.records()["kind"]
        out[label] = {"value": round(n / min(ts) / 2**30, 3), "ms": round(min(ts) * 1e3, 3),
                      "first_call_ms": round(first_ms, 3), "seeded_ids": int(len(ids)),
                      "hist_seeded": int(seeded["hist_seeded"]), "by_value": int(seeded["by_value"]),
                      "dup_records": int((kinds == 1).sum()), "new_records": int((kinds == 0).sum()),
                      "stages": stage_dict(st)}
    del other
    # a 2 M-id repository partly written by stock zbackup: 99 % of the ids with
    # metadata (the historic index: 2 M entries), 1 % by value (the exact
    # screen runs at every byte for them), on the first GiB
    rng = np.random.default_rng(2000000)
    k = 2_000_000
    keys = rng.integers(1, 2**63, k, dtype=np.int64).astype(np.uint64)
    shas = rng.integers(0, 256, (k, 16), dtype=np.uint8)
    meta = synthetic_meta(rng, k)
    meta["sha1"] = shas
    meta["rolling"] = keys
    nb = 1 << 30
    for label, frac in (("ids_2000000_all_meta", 1.0), ("ids_2000000_99pct_meta", 0.99)):
        with BackupCreator(W64, device=local, sha1=True, timing=True) as b:
            b.seed_index_meta(shas, keys, W64, meta[: int(k * frac)])
            seeded = b.stats()
            b.chunk_device(buf.data_ptr(), nb)
            ts = []
            for _ in range(3):
                b.forget_stream_chunks()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                b.chunk_device(buf.data_ptr(), nb)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t1)
            st = b.stats()
        out[label] = {"value": round(nb / min(ts) / 2**30, 3), "ms": round(min(ts) * 1e3, 3), "stream_bytes": nb,
                      "hist_seeded": int(seeded["hist_seeded"]), "by_value": int(seeded["by_value"]),
                      "screen_ms": round(st["fscan_ms"], 3), "stages": stage_dict(st)}
    return out


def bundle_leg(torch, buf, n, recs, world, local, cpu_sample):
    """Bundle writer offload (§8(f)-4) over the stream's saved chunks: Writer::add's
    bundling (2 MiB bundles), the payloads gathered on the device and lzo1x_1
    compressed with zbackup's framing -- for the C2 stream (random: LZO finds
    nothing to match) and for 4 GiB of text-like data (compresses ~3x); liblzo2
    on one core over 64 MiB of each as the CPU baseline."""
    import numpy as np

    from tests.lzo_inputs import payload
    from zbackup_amd import ZC_CHUNK_NEW
    from zbackup_amd.bundle import BundleCompressor, lzo_capacity, plan_bundles
    res = {}
    with BundleCompressor(device=local) as comp:
        for kind in ("random", "text"):
            if kind == "random":
                src, nbytes = buf, n
                sel = recs[recs["kind"] == ZC_CHUNK_NEW]
                offs, sizes = sel["offset"].astype(np.uint64), sel["size"].astype(np.uint64)
            else:
                nbytes = 4 << 30
                base = torch.from_numpy(payload("text", 128 << 20, 21)).to(buf.device)
                src = base.repeat(nbytes // base.numel())  # built in HBM (no 4 GiB host array per rank)
                del base
                offs = np.arange(0, nbytes, W64, dtype=np.uint64)
                sizes = np.full(len(offs), W64, dtype=np.uint64)
            bundle_of, nb = plan_bundles(sizes)
            pay_size = np.bincount(bundle_of, weights=sizes, minlength=nb).astype(np.uint64)
            caps = np.array([lzo_capacity(int(x)) for x in pay_size], dtype=np.uint64)
            out_off = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.uint64)
            # a bundle whose chunks lie back to back in the stream has the
            # stream range itself as its payload (Bundle::Creator::addChunk's
            # appends would rebuild those bytes): compressed in place; the
            # others are gathered into a payload buffer first
            first = np.searchsorted(bundle_of, np.arange(nb))
            ends = offs + sizes
            adj = np.ones(len(offs), dtype=bool)
            adj[1:] = (offs[1:] == ends[:-1]) | (bundle_of[1:] != bundle_of[:-1])
            inplace = np.logical_and.reduceat(adj, first) if nb else np.zeros(0, bool)
            g_sel = np.nonzero(~inplace[bundle_of])[0]
            g_size = pay_size[~inplace]
            g_off = np.concatenate([[0], np.cumsum(g_size)[:-1]]).astype(np.uint64)
            d_pay = torch.empty(max(int(g_size.sum()), 1), dtype=torch.uint8, device=buf.device)
            d_out = torch.empty(int(caps.sum()), dtype=torch.uint8, device=buf.device)
            out_size = np.zeros(nb, dtype=np.uint64)

            def step():
                if inplace.any():
                    out_size[inplace] = comp.compress(src.data_ptr(), offs[first[inplace]], pay_size[inplace],
                                                      d_out.data_ptr(), out_off[inplace])
                if len(g_sel):
                    comp.gather(src.data_ptr(), offs[g_sel], sizes[g_sel], d_pay.data_ptr())
                    out_size[~inplace] = comp.compress(d_pay.data_ptr(), g_off, g_size, d_out.data_ptr(),
                                                       out_off[~inplace])
                return 0.0

            el, _ = timed_steps(torch, world, step, 1, 3)
            parse_ms, blocks = comp.last_stats()
            # the gather alone (every bundle assembled, as if none were in place)
            d_all = torch.empty(int(pay_size.sum()), dtype=torch.uint8, device=buf.device)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            comp.gather(src.data_ptr(), offs, sizes, d_all.data_ptr())
            torch.cuda.synchronize()
            gather_ms = (time.perf_counter() - t0) * 1e3
            in_bytes = int(sizes.sum())
            r = {"value": round(job_value(in_bytes, world, 3, el), 3), "unit": "GiB/s",
                 "ms_per_step": round(el / 3 * 1e3, 3), "bundles": int(nb), "in_place_bundles": int(inplace.sum()),
                 "blocks_48k": int(blocks), "parse_ms": round(parse_ms, 3),
                 "gather_all_ms": round(gather_ms, 3), "ratio": round(float(out_size.sum()) / in_bytes, 4)}
            if cpu_sample:
                from oracle import lzo_oracle
                if lzo_oracle.lzo_lib() is not None:
                    host = d_all[:64 << 20].cpu().numpy()
                    t0 = time.perf_counter()
                    for i in range(0, len(host), 0x200000):
                        lzo_oracle.frame(host[i:i + 0x200000].tobytes())
                    r["cpu_liblzo2_1core"] = round(len(host) / (time.perf_counter() - t0) / 2**30, 4)
            res[kind] = r
            del d_pay, d_out, d_all, src
    res["path"] = ("saved chunks -> Writer::add bundles (2 MiB) -> payload in place when the chunks are adjacent, "
                   "else zc_bundle_gather (HBM) -> zc_lzo_compress (lzo1x_1 + zbackup framing, byte-identical to "
                   "liblzo2 2.10)")
    return res


def stage_dict(st):
    return {"scan_ms": round(st["scan_ms"], 4), "resolve_ms": round(st["resolve_ms"], 4),
            "total_ms": round(st["total_ms"], 4), "anchors": st["anchors"],
            "candidates": st["candidates"], "epochs": st["epochs"],
            "meta_ms": round(st["meta_ms"], 4), "probe_ms": round(st["probe_ms"], 4),
            "fscan_ms": round(st["fscan_ms"], 4), "walk_ms": round(st["walk_ms"], 4),
            "finalize_ms": round(st["finalize_ms"], 4), "fbatch_ms": round(st["fbatch_ms"], 4),
            "sha_wait_ms": round(st["sha_wait_ms"], 4), "sha_fill_ms": round(st["sha_fill_ms"], 4),
            "hist_ms": round(st["hist_ms"], 4)}


def feed_bench(n, seed, sha1, copy_threads=8, sha256=2):
    """tools/feedbench/feed_bench (built in-tree by build()): the zutils.cc read
    loop over the C++ binding, one process; the input copy is split over
    copy_threads threads and reported apart from the engine's time.  sha256:
    the backup's whole-stream SHA-256 (zutils.cc:119), 1 inline after each read
    as the reference does, 2 on a helper thread beside handleMoreData, 0 none."""
    exe = os.path.join(ROOT, "tools", "feedbench", "feed_bench")
    if not os.path.exists(exe):
        return None
    out = subprocess.run([exe, str(W64), str(n), str(seed), "1" if sha1 else "0", str(copy_threads), str(sha256)],
                         capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        return {"error": out.stderr.strip()[-300:]}
    d = json.loads(out.stdout.strip().splitlines()[-1])
    eng = d["engine_and_adapter_s"]
    return {"value": round(n / d["loop_s"] / 2**30, 3), "unit": "GiB/s",
            "engine_and_adapter_GiB_per_s": round(n / eng / 2**30, 3) if eng > 0 else None,
            "engine_and_adapter_note": "loop minus the input copies, Writer::add's payload appends, the SHA-256 and "
                                      "the feed window's one-time setup (window_setup_s: pinning its host mirror)",
            "window_setup_s": d.get("window_setup_s"), "segments": d.get("segments"),
            "engine_resolve_ms": d.get("engine_total_ms"),
            "loop_s": d["loop_s"], "copy_s": d["copy_s"], "copy_threads": d["copy_threads"],
            "writer_add_s": d["writer_add_s"], "engine_and_adapter_s": eng, "shrink_s": d["shrink_s"],
            "shrink_iterations": d["shrink_iterations"], "writer_chunks": d["writer_chunks"],
            "bundles": d["bundles"], "window_bytes": d["window_bytes"], "pieces": d["pieces"],
            "sha256": {0: "none", 1: "inline after each read (zutils.cc:119)",
                       2: "helper thread beside handleMoreData"}[sha256], "sha256_s": d["sha256_s"],
            "path": "zutils.cc read loop over integration/gpu_backup_creator.hh: memcpy into getInputBuffer "
                    f"({copy_threads} threads, standing for fread), handleMoreData through the bounded window, "
                    "records drained as cut (zc_take_records, zc_read_stream -> Writer::add into 2 MiB bundle "
                    "payloads, Message::serialize), finish, getBackupData; shrink passes timed apart"}


def rank_env(args):
    """(world, rank, local rank) from the environment; joins the gloo group
    the replicas use for their barriers and max/gather reductions."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return world, rank, local


def dry_rank(args):
    """--dry-run: the replica job of run_rank with the oracle (CPU) standing in
    for the device engine, so the self-launch and the rank bookkeeping run on a
    machine without a GPU.  Prints a line marked dry_run; not a measurement."""
    import torch.distributed as dist
    from oracle import oracle
    world, rank, _ = rank_env(args)
    n = max(int(args.gib * 2**30), 1)
    data = oracle.splitmix64(n, rank_seed(args.seed, rank))
    box = {}

    def step():
        box["recs"] = oracle.chunk_array(data, W64)
        return 0.0

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    elapsed = job_elapsed(time.perf_counter() - t0, world)
    nrec = job_gather(float(len(box["recs"])), world)
    first = job_gather(float(box["recs"]["rolling"][0]) if len(box["recs"]) else 0.0, world)
    if rank == 0:
        print(json.dumps({"dry_run": True, "metric": "rolling-hash chunking GiB/s (oracle rehearsal)",
                          "value": job_value(n, world, args.steps, elapsed), "unit": "GiB/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "records_per_rank": [int(v) for v in nrec], "first_key_per_rank": first,
                          "seeds": [rank_seed(args.seed, r) for r in range(world)]}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_rank(args):
    import torch
    import torch.distributed as dist

    world, rank, local = rank_env(args)
    # one GPU per rank; more ranks than visible GPUs (a rehearsal of the
    # multi-rank path on a smaller box) share them, and say so
    ndev = torch.cuda.device_count()
    if ndev and local >= ndev:
        print(f"bench.py: rank {rank} shares GPU {local % ndev} ({ndev} visible for {world} ranks)",
              file=sys.stderr, flush=True)
        local %= ndev
    torch.cuda.set_device(local)

    from zbackup_amd import BackupCreator

    n = int(args.gib * 2**30)
    buf = torch.empty(n, dtype=torch.uint8, device=f"cuda:{local}")
    seed = rank_seed(args.seed, rank)
    fill_stream(torch, buf, n, args.config, seed, local)

    # with SHA-1 ids a context's chunks join its index (Writer::add ->
    # ChunkIndex::addChunk), so chunking the same stream again would measure
    # an incremental backup of identical data: each step first drops them
    # (zc_forget_stream_chunks), so every step is a first backup of the stream
    # against the index a fresh ZBackup instance loads, on warm buffers
    def make_step(bc, sha1):
        def step():
            if sha1:
                bc.forget_stream_chunks()
            bc.chunk_device(buf.data_ptr(), n)
            return bc.scan_ms()
        return step

    bc = BackupCreator(W64, device=local, sha1=args.sha1, timing=True)
    elapsed, scan_ms = timed_steps(torch, world, make_step(bc, args.sha1), args.warmup, args.steps)
    st = bc.stats()
    recs = bc.records().copy()
    nrec = len(recs)
    bc.close()
    ms_step = elapsed / args.steps * 1e3
    value = job_value(n, world, args.steps, elapsed)
    scan_avg = sum(scan_ms) / len(scan_ms)
    fracs = [n / (s * 1e-3) / 1e9 / HBM_PEAK_GBS for s in job_gather(scan_avg, world)]

    extras = {}
    # the extra passes are single-GPU measurements: a multi-GPU run (C4) keeps
    # to the headline, the per-GPU fractions and the concurrent CPU baseline, so
    # N ranks do not each pin 8 GiB of host memory for the end-to-end legs
    if not args.no_extras and world == 1:
        # BASELINE configs[2] (C3, 50 % duplicated) and configs[4] (C5, all
        # zeros) in the headline's own mode (rolling-hash ids), timed exactly as
        # the headline: W untimed + K timed steps between barriers and syncs
        if args.config == "c2" and not args.sha1:
            other = torch.empty(n, dtype=torch.uint8, device=buf.device)
            for cfg in ("c3", "c5"):
                fill_stream(torch, other, n, cfg, seed, local)
                bo = BackupCreator(W64, device=local, sha1=False, timing=True)

                def step_cfg():
                    bo.chunk_device(other.data_ptr(), n)
                    return bo.scan_ms()

                elo, scan_o = timed_steps(torch, world, step_cfg, args.warmup, args.steps)
                sto = bo.stats()
                nrec_o = len(bo.records())
                bo.close()
                extras[f"value_{cfg}"] = {"value": round(job_value(n, world, args.steps, elo), 3), "unit": "GiB/s",
                                          "ms_per_step": round(elo / args.steps * 1e3, 3), "steps": args.steps,
                                          "warmup": args.warmup, "workload": CONFIGS[cfg],
                                          "chunks_per_s": round(nrec_o * args.steps / elo, 1),
                                          "scan_ms_avg": round(sum(scan_o) / len(scan_o), 4),
                                          "stages": stage_dict(sto)}
            del other
        # complete ChunkIds on every record (the mode the zbackup binding runs,
        # integration/gpu_backup_creator.hh): C2, and C3 / C5 in a second buffer
        if not args.sha1 and args.sha1_steps > 0:
            b2 = BackupCreator(W64, device=local, sha1=True, timing=True)
            el2, _ = timed_steps(torch, world, make_step(b2, True), 2, args.sha1_steps)
            st2 = b2.stats()
            extras["value_sha1"] = job_value(n, world, args.sha1_steps, el2)
            extras["sha1_ms_per_step"] = el2 / args.sha1_steps * 1e3
            extras["sha1_stages"] = stage_dict(st2)
            if args.config == "c2":
                other = torch.empty(n, dtype=torch.uint8, device=buf.device)
                for cfg in ("c3", "c5"):
                    fill_stream(torch, other, n, cfg, seed, local)

                    def step_other():
                        b2.forget_stream_chunks()
                        b2.chunk_device(other.data_ptr(), n)
                        return 0.0

                    elc, _ = timed_steps(torch, world, step_other, 2, args.sha1_steps)
                    extras[f"value_sha1_{cfg}"] = {"value": round(job_value(n, world, args.sha1_steps, elc), 3),
                                                   "unit": "GiB/s",
                                                   "ms_per_step": round(elc / args.sha1_steps * 1e3, 3),
                                                   "workload": CONFIGS[cfg], "stages": stage_dict(b2.stats())}
                del other
            b2.close()
        # incremental backups on one context: with SHA-1 ids a stream's chunks
        # stay in the context's index (Writer::add -> ChunkIndex::addChunk), so
        # a later stream is matched against them through the historic index --
        # the same 8 GiB again (every chunk a duplicate), and the stream after a
        # different 8 GiB one (131,072 historic entries, none matching)
        if not args.sha1:
            other = torch.empty(n, dtype=torch.uint8, device=buf.device)
            fill_stream(torch, other, n, args.config, seed + 1000003, local)
            inc = {}
            for label, first in (("same_stream_again", buf), ("after_other_stream", other)):
                # same data again: 3 repeats on one context (nothing new joins
                # the index); after another stream: each repeat on a fresh
                # context (the measured stream adds 131,072 entries)
                ts = []
                b5 = None
                for rep in range(3):
                    if b5 is None:
                        b5 = BackupCreator(W64, device=local, sha1=True, timing=True)
                        b5.chunk_device(first.data_ptr(), n)
                        torch.cuda.synchronize()
                    t1 = time.perf_counter()
                    b5.chunk_device(buf.data_ptr(), n)
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter() - t1)
                    if label == "after_other_stream" and rep < 2:
                        b5.close()
                        b5 = None
                st5 = b5.stats()
                kinds = b5.records()["kind"]
                b5.close()
                inc[label] = {"value": round(job_value(n, world, 1, job_max(min(ts), world)), 3), "unit": "GiB/s",
                              "ms": round(min(ts) * 1e3, 3), "dup_records": int((kinds == 1).sum()),
                              "new_records": int((kinds == 0).sum()), "hist_entries": st5["hist_entries"],
                              "stages": stage_dict(st5)}
            del other
            extras["incremental"] = inc
            if args.config == "c2" and n == 8 << 30:
                extras["seeded_repo"] = seeded_repo_leg(torch, buf, n, seed, local)
        # the stream starts in (pinned) host memory, as in zutils.cc:100-124:
        # rolling-hash ids and complete ChunkIds
        host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        host.copy_(buf)
        reps = 3
        for sha1 in (False, True):
            b3 = BackupCreator(W64, device=local, sha1=sha1, timing=True)

            def e2e_step():
                if sha1:
                    b3.forget_stream_chunks()
                b3.chunk_host(host.data_ptr(), n)
                return 0.0

            el3, _ = timed_steps(torch, world, e2e_step, 1, reps)
            b3.close()
            extras["end_to_end_sha1" if sha1 else "end_to_end"] = {
                "value": job_value(n, world, reps, el3), "unit": "GiB/s", "ms_per_step": el3 / reps * 1e3,
                "path": "pinned host buffer -> zc_chunk_host: 64 MiB H2D segments on a side stream, each scanned "
                        "as it lands, then resolve + records to host" + (" + SHA-1 chunk ids" if sha1 else "")}
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(reps):
            buf.copy_(host, non_blocking=True)
        torch.cuda.synchronize()
        h2d = job_gather(n * reps / (time.perf_counter() - t1) / 2**30, world)
        extras["end_to_end"]["h2d_only_GiB_per_s_per_gpu"] = [round(v, 2) for v in h2d]
        fill_stream(torch, buf, n, args.config, seed, local)  # buf held the host copy's bytes anyway
        del host
        # the drop-in feed (zutils.cc:100-127 over integration/gpu_backup_creator.hh,
        # tools/feedbench): input copied into getInputBuffer() (standing for fread),
        # handleMoreData through the bounded window, the adapter taking the records
        # as they are cut (Writer::add of each new chunk's bytes into a 2 MiB bundle
        # payload, Message::serialize of every record), finish, getBackupData, the
        # shrink passes; rolling-hash ids and complete ChunkIds
        if args.config == "c2":
            # feed: the engine's part alone (no whole-stream SHA-256); feed_sha1:
            # the reference loop whole -- complete ChunkIds and the backup's
            # SHA-256 of every piece, on a helper thread (and inline, as
            # zutils.cc:119 runs it, in feed_sha1_inline_sha256)
            for key, sha1, s256 in (("feed", False, 0), ("feed_sha1", True, 2), ("feed_sha1_inline_sha256", True, 1)):
                fb = feed_bench(n, seed, sha1, sha256=s256)
                if fb:
                    extras[key] = fb
        if args.config == "c2" and args.lzo:
            extras["bundle_lzo"] = bundle_leg(torch, buf, n, recs, world, local, rank == 0)
        if args.config == "c2" and n >= 1 << 30:
            extras["static_index"] = static_leg(torch, buf, local)

    cpu = None
    if not args.no_cpu_baseline and args.config == "c2":
        # the reference path is one thread per stream (zutils.cc:100-124): N
        # ranks run N single-thread oracle processes concurrently, one each
        if world > 1:
            dist.barrier()
        c = cpu_baseline(args.cpu_sample_mib << 20, seed)
        per = job_gather(c["value"], world)
        cpu = {"value": round(sum(per), 5), "unit": "GiB/s", "cores": world, "kind": "port",
               "sample": f"first {args.cpu_sample_mib} MiB of each rank's C2 stream (seed {args.seed}+rank), "
                         f"oracle/zc_oracle.cpp single thread per rank, {world} concurrent; rank 0: "
                         f"{c['records']} records in {c['seconds']:.2f} s",
               "per_process": [round(v, 5) for v in per], "host": host_cpu()}
        if world == 1 and not args.no_extras:
            # the other single-GPU configs' shapes at sample scale
            for cfg in ("c3", "c5"):
                co = cpu_baseline(args.cpu_sample_mib << 20, seed, cfg)
                cpu[f"value_{cfg}"] = {"value": round(co["value"], 5), "unit": "GiB/s", "cores": 1,
                                       "sample": f"{args.cpu_sample_mib} MiB of the {cfg.upper()} shape "
                                                 f"({CONFIGS[cfg]}), {co['records']} records in "
                                                 f"{co['seconds']:.2f} s"}

    if rank == 0:
        from zbackup_amd import _lib
        build_id = _lib.build_id()
        prof = committed_profile(build_id)
        achieved = n / (scan_avg * 1e-3) / 1e9
        rp_ms, rp_src = rocprof_scan_ms(prof)
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
            "config": {"workload": C4 if world > 1 and args.config == "c2" else CONFIGS[args.config],
                       "stream_bytes_per_gpu": n, "chunk_max_size": W64,
                       "parallelism": f"replicas x{world} (independent streams)",
                       "chunk_ids": "SHA-1 prefix + rolling hash" if args.sha1 else "rolling hash"},
            "chunks_per_s": round(nrec * world * args.steps / elapsed, 1),
            "records_per_stream": nrec,
            "roofline": {"bound": "hbm", "kernel": "zc_scan_kernel", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": pmc_traffic(prof, n), "bytes_per_launch": n,
                         "scan_ms_avg": round(scan_avg, 4)},
            "build_id": build_id,
            "per_gpu_frac": [round(f, 4) for f in fracs],
            "stages": stage_dict(st),
        }
        if rp_ms and args.config == "c2" and n == 8 << 30:
            # the headline fraction is the committed rocprofv3 --kernel-trace
            # --stats average of THIS build's scan (the profile is keyed on the
            # build id); this run's own HIP-event average stays beside it as
            # events_frac (it is another box's clock)
            out["roofline"]["events_achieved"] = out["roofline"]["achieved"]
            out["roofline"]["events_frac"] = out["roofline"]["frac"]
            out["roofline"]["achieved"] = round(n / (rp_ms * 1e-3) / 1e9, 1)
            out["roofline"]["frac"] = round(n / (rp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            out["roofline"]["frac_source"] = "rocprof"
            out["roofline"]["rocprof"] = {"scan_ms_avg": round(rp_ms, 4),
                                          "achieved": round(n / (rp_ms * 1e-3) / 1e9, 1),
                                          "frac": round(n / (rp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                          "source": rp_src}
        else:
            out["roofline"]["frac_source"] = "events (no committed rocprof profile of this build)"
        if prof is None:
            out["roofline"]["profile"] = f"no committed profiles/rNN_scan_profile.json of build {build_id}"
        else:
            out["roofline"]["profile"] = prof["path"]
        if "value_sha1" in extras:
            out["value_sha1"] = round(extras["value_sha1"], 3)
            out["sha1_ms_per_step"] = round(extras["sha1_ms_per_step"], 3)
            out["sha1_stages"] = extras["sha1_stages"]
        for key in ("value_c3", "value_c5", "value_sha1_c3", "value_sha1_c5"):
            if key in extras:
                out[key] = extras[key]
        for key in ("end_to_end", "end_to_end_sha1"):
            if key in extras:
                e = extras[key]
                e["value"] = round(e["value"], 3)
                e["ms_per_step"] = round(e["ms_per_step"], 3)
                out[key] = e
        if "incremental" in extras:
            out["incremental_sha1"] = extras["incremental"]
        if "seeded_repo" in extras:
            out["seeded_repo_sha1"] = extras["seeded_repo"]
        for key in ("feed", "feed_sha1", "feed_sha1_inline_sha256"):
            if key in extras:
                out[key] = extras[key]
        if "bundle_lzo" in extras:
            out["bundle_lzo"] = extras["bundle_lzo"]
        if "static_index" in extras:
            out["static_index"] = extras["static_index"]
        if cpu:
            out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # self-launched multi-GPU run: one child process per GPU
        sys.exit(launch(sys.argv[1:], args.gpus))
    if args.dry_run:
        dry_rank(args)
    else:
        run_rank(args)


if __name__ == "__main__":
    main()
