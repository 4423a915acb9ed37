#!/usr/bin/env python3
"""Run some of bench.py's extra legs alone on one GPU (tooling only):

  python tools/run_legs.py seeded_repo incremental static_index ...

Prints one JSON line per leg."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def incremental(torch, buf, n, seed):
    import bench
    from zbackup_amd import BackupCreator
    other = torch.empty(n, dtype=torch.uint8, device=buf.device)
    bench.fill_stream(torch, other, n, "c2", seed + 1000003, 0)
    inc = {}
    for label, first in (("same_stream_again", buf), ("after_other_stream", other)):
        ts = []
        b5 = None
        for rep in range(3):
            if b5 is None:
                b5 = BackupCreator(65536, device=0, sha1=True, timing=True)
                b5.chunk_device(first.data_ptr(), n)
                torch.cuda.synchronize()
            t1 = time.perf_counter()
            b5.chunk_device(buf.data_ptr(), n)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t1)
            if label == "after_other_stream" and rep < 2:
                b5.close()
                b5 = None
        st = b5.stats()
        b5.close()
        inc[label] = {"ms": [round(t * 1e3, 3) for t in ts], "stages": bench.stage_dict(st)}
    return inc


def main():
    import torch
    import bench
    n = 8 << 30
    seed = 2024
    buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    bench.fill_stream(torch, buf, n, "c2", seed, 0)
    for leg in sys.argv[1:]:
        t0 = time.perf_counter()
        if leg == "seeded_repo":
            r = bench.seeded_repo_leg(torch, buf, n, seed, 0)
        elif leg == "incremental":
            r = incremental(torch, buf, n, seed)
        elif leg == "static_index":
            r = bench.static_leg(torch, buf, 0)
        else:
            raise SystemExit(f"unknown leg {leg}")
        print(json.dumps({"leg": leg, "seconds": round(time.perf_counter() - t0, 1), **r}), flush=True)


if __name__ == "__main__":
    main()
