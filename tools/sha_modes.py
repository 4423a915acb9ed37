#!/usr/bin/env python3
"""Experiment (tooling only): the ZC_FLAG_SHA1 pipeline's SHA-1 schedules
(ZC_SHA_MODE, zc_engine.cpp) interleaved in one process on the same 8 GiB
streams: per config and mode the median / min wall time of a step (forget +
zc_chunk_device), and the median of the host phases.

  python tools/sha_modes.py [rounds] [modes]
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
    modes = [int(m) for m in (sys.argv[2] if len(sys.argv) > 2 else "0,1,3").split(",")]
    n = 8 << 30
    buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    out = {}
    for cfg in ("c2", "c3", "c5"):
        bench.fill_stream(torch, buf, n, cfg, 2024, 0)
        bc = BackupCreator(65536, device=0, sha1=True, timing=True)
        times = {m: [] for m in modes}
        st = {m: [] for m in modes}
        for r in range(rounds + 1):
            for m in modes:
                os.environ["ZC_SHA_MODE"] = str(m)
                for _ in range(3):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    bc.forget_stream_chunks()
                    bc.chunk_device(buf.data_ptr(), n)
                    torch.cuda.synchronize()
                    dt = (time.perf_counter() - t0) * 1e3
                    if r:
                        times[m].append(dt)
                        st[m].append(bc.stats())
        bc.close()
        for m in modes:
            t = sorted(times[m])
            ph = {k: round(statistics.median(s[k] for s in st[m]), 3)
                  for k in ("scan_ms", "meta_ms", "walk_ms", "finalize_ms", "sha_wait_ms", "sha_fill_ms", "hist_ms",
                            "total_ms")}
            out[f"{cfg}_mode{m}"] = {"median_ms": round(statistics.median(t), 3), "min_ms": round(t[0], 3),
                                     "GiB_per_s_median": round(8 / (statistics.median(t) * 1e-3), 1), **ph}
            print(cfg, m, json.dumps(out[f"{cfg}_mode{m}"]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
