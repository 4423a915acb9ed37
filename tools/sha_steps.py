#!/usr/bin/env python3
"""SHA-1-mode step times (tooling only): C2, C3 and C5 at 8 GiB, each step a
first backup of the stream (forget + zc_chunk_device with ZC_FLAG_SHA1), the
configs interleaved round by round; per config the median / min wall time of
a step and the median of the engine's phase timings.

  python tools/sha_steps.py [rounds]
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from zbackup_amd import BackupCreator
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    n = 8 << 30
    cfgs = ("c2", "c3", "c5")
    bufs = {}
    for cfg in cfgs:
        bufs[cfg] = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        bench.fill_stream(torch, bufs[cfg], n, cfg, 2024, 0)
    bc = BackupCreator(65536, device=0, sha1=True, timing=True)
    times = {c: [] for c in cfgs}
    st = {c: [] for c in cfgs}
    for r in range(rounds + 1):
        for cfg in cfgs:
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                bc.forget_stream_chunks()
                bc.chunk_device(bufs[cfg].data_ptr(), n)
                torch.cuda.synchronize()
                if r:
                    times[cfg].append((time.perf_counter() - t0) * 1e3)
                    st[cfg].append(bc.stats())
    bc.close()
    out = {}
    for cfg in cfgs:
        t = sorted(times[cfg])
        ph = {k: round(statistics.median(s[k] for s in st[cfg]), 3)
              for k in ("scan_ms", "meta_ms", "walk_ms", "finalize_ms", "sha_wait_ms", "sha_fill_ms", "hist_ms",
                        "total_ms")}
        out[cfg] = {"median_ms": round(statistics.median(t), 3), "min_ms": round(t[0], 3),
                    "GiB_per_s_median": round(8 / (statistics.median(t) * 1e-3), 1), **ph}
        print(cfg, json.dumps(out[cfg]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
