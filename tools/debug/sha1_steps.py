"""Per-step timing of repeated SHA-1 steps on one context (debug tooling)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from zbackup_amd import BackupCreator, fill_splitmix64

n = 8 << 30
buf = torch.empty(n, dtype=torch.uint8, device="cuda")
fill_splitmix64(buf.data_ptr(), n, 2024, 0)
torch.cuda.synchronize()
for label, sha in (("plain", False), ("sha1", True), ("sha1-b", True)):
    bc = BackupCreator(65536, sha1=sha, timing=True)
    for i in range(8):
        t0 = time.perf_counter()
        if sha:
            bc.forget_stream_chunks()
        t1 = time.perf_counter()
        bc.chunk_device(buf.data_ptr(), n)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        st = bc.stats()
        print(label, i, f"forget {1e3 * (t1 - t0):.2f} ms chunk {1e3 * (t2 - t1):.2f} ms", {k: round(v, 3) if isinstance(v, float) else v for k, v in st.items() if k.endswith("_ms") or k in ("hist_entries", "statics")}, flush=True)
    bc.close()
