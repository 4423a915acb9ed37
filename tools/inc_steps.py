#!/usr/bin/env python3
"""Incremental-backup step times (tooling only): an 8 GiB C2 stream chunked
with SHA-1 ids on a context, then the same stream again `reps` times (every
chunk a historic duplicate), each repeat's wall time and engine phases printed.

  python tools/inc_steps.py [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KEYS = ("total_ms", "scan_ms", "meta_ms", "probe_ms", "walk_ms", "finalize_ms", "sha_wait_ms", "sha_fill_ms",
        "hist_ms", "candidates", "respeculations", "hist_entries")


def main():
    import torch
    import bench
    from zbackup_amd import BackupCreator
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    n = 8 << 30
    buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    bench.fill_stream(torch, buf, n, "c2", 2024, 0)
    bc = BackupCreator(65536, device=0, sha1=True, timing=True)
    bc.chunk_device(buf.data_ptr(), n)
    torch.cuda.synchronize()
    print("first", json.dumps({k: bc.stats()[k] for k in KEYS}), flush=True)
    for i in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bc.chunk_device(buf.data_ptr(), n)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        st = bc.stats()
        kinds = bc.records()["kind"]
        print("again", i, round(ms, 3), "dup", int((kinds == 1).sum()),
              json.dumps({k: (round(st[k], 3) if isinstance(st[k], float) else st[k]) for k in KEYS}), flush=True)
    bc.close()


if __name__ == "__main__":
    main()
