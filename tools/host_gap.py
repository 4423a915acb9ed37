#!/usr/bin/env python3
"""Where the headline step's time outside the device work goes (tooling only).

For the 8 GiB C2 stream, rolling-hash ids: per call, the wall time of the
zc_chunk_device ctypes call, the engine's own total_ms (run_final), scan_ms,
meta_ms, and the gap from one call's return to the next call's entry; then
the cost of the Python side of bench.py's step (the wrapper, zc_get_stats).

  python tools/host_gap.py [reps]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from zbackup_amd import BackupCreator
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = 8 << 30
    buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    bench.fill_stream(torch, buf, n, "c2", 2024, 0)
    torch.cuda.synchronize()
    bc = BackupCreator(65536, device=0, sha1=False, timing=True)
    L, ctx, ptr = bc._L, bc._ctx, ctypes.c_void_p(buf.data_ptr())
    for _ in range(10):
        L.zc_chunk_device(ctx, ptr, n)
    rows = []
    t_prev = time.perf_counter()
    for _ in range(reps):
        t0 = time.perf_counter()
        rc = L.zc_chunk_device(ctx, ptr, n)
        t1 = time.perf_counter()
        assert rc == 0
        st = bc.stats()
        rows.append(((t1 - t0) * 1e3, st["total_ms"], st["scan_ms"], st["meta_ms"], st["walk_ms"],
                     st["finalize_ms"], (t0 - t_prev) * 1e3))
        t_prev = time.perf_counter()
    rows.sort()
    print("call_ms total_ms scan_ms meta_ms walk_ms finalize_ms  (sorted by call_ms)")
    for r in rows:
        print(" ".join(f"{v:8.4f}" for v in r[:6]))
    med = rows[len(rows) // 2]
    print(f"median: call {med[0]:.4f} ms, engine total {med[1]:.4f} ms, outside run_final "
          f"{(med[0] - med[1]) * 1e3:.1f} us, after the scan {(med[1] - med[2]) * 1e3:.1f} us "
          f"(batch from the scan's end {med[3] * 1e3:.1f} us)")
    # bench.py's step, back to back: wrapper + call + scan_ms read
    steps = []
    for _ in range(reps):
        t0 = time.perf_counter()
        bc.chunk_device(buf.data_ptr(), n)
        bc.scan_ms()
        steps.append((time.perf_counter() - t0) * 1e3)
    steps.sort()
    print(f"bench-style step (wrapper + call + scan_ms), median {steps[len(steps) // 2]:.4f} ms")
    k = 2000
    t0 = time.perf_counter()
    for _ in range(k):
        bc.scan_ms()
    print(f"scan_ms() read: {(time.perf_counter() - t0) / k * 1e6:.2f} us per call")
    t0 = time.perf_counter()
    for _ in range(k):
        bc._new_stream()
    print(f"_new_stream(): {(time.perf_counter() - t0) / k * 1e6:.2f} us per call")
    t0 = time.perf_counter()
    for _ in range(k):
        L.zc_chunk_device(ctx, ptr, 0)
    print(f"zc_chunk_device of 0 bytes: {(time.perf_counter() - t0) / k * 1e6:.2f} us per call")
    ab = os.environ.get("HOST_GAP_AB")  # an engine A/B switch read at zc_create: "NAME" of the env var
    if ab:
        os.environ[ab] = "1"
        bb = BackupCreator(65536, device=0, sha1=False, timing=True)
        del os.environ[ab]
        res = {"A": [], "B": []}
        for _ in range(10):
            L.zc_chunk_device(bb._ctx, ptr, n)
        for _ in range(reps):
            for label, b in (("A", bc), ("B", bb)):
                t0 = time.perf_counter()
                assert L.zc_chunk_device(b._ctx, ptr, n) == 0
                t1 = time.perf_counter()
                st = b.stats()
                res[label].append(((t1 - t0) * 1e3, st["scan_ms"], st["meta_ms"]))
        for label, rs in res.items():
            rs.sort()
            m = rs[len(rs) // 2]
            post = sorted(r[0] - r[1] for r in rs)[len(rs) // 2]
            meta = sorted(r[2] for r in rs)[len(rs) // 2]
            print(f"{label} ({ab}={'1' if label == 'B' else 'unset'}): call median {m[0]:.4f} ms, "
                  f"call - scan median {post * 1e3:.1f} us, meta median {meta * 1e3:.1f} us")
        bb.close()
    bc.close()


if __name__ == "__main__":
    main()
