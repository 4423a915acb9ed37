#!/usr/bin/env python3
"""SHA-1 kernel in the two SHA-1-mode steps (tooling only; run under
`rocprofv3 --kernel-trace`): a first backup of the 8 GiB C2 stream (forget +
zc_chunk_device, the bench's value_sha1 step) and an incremental backup of the
same stream again (every chunk a historic duplicate), `reps` of each,
interleaved on one box, with each step's wall time printed.

  python tools/sha_inc_trace.py [reps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from zbackup_amd import BackupCreator
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    n = 8 << 30
    buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    bench.fill_stream(torch, buf, n, "c2", 2024, 0)
    first = BackupCreator(65536, device=0, sha1=True, timing=True)
    inc = BackupCreator(65536, device=0, sha1=True, timing=True)
    inc.chunk_device(buf.data_ptr(), n)
    for r in range(reps + 1):
        for label, bc in (("first", first), ("again", inc)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if label == "first":
                bc.forget_stream_chunks()
            bc.chunk_device(buf.data_ptr(), n)
            torch.cuda.synchronize()
            st = bc.stats()
            print(label, r, round((time.perf_counter() - t0) * 1e3, 3), "sha_wait", round(st["sha_wait_ms"], 3),
                  "probe", round(st["probe_ms"], 3), "walk", round(st["walk_ms"], 3), "fin",
                  round(st["finalize_ms"], 3), flush=True)
    first.close()
    inc.close()


if __name__ == "__main__":
    main()
