"""Where a --sha1 bench step's time goes on the host: forget / chunk_device / stats."""
import sys
import time

import torch

sys.path.insert(0, ".")
from zbackup_amd import BackupCreator, fill_splitmix64  # noqa: E402

n = 8 << 30
buf = torch.empty(n, dtype=torch.uint8, device="cuda")
fill_splitmix64(buf.data_ptr(), n, 2024, 0)
torch.cuda.synchronize()
bc = BackupCreator(65536, sha1=True, timing=True)
for k in range(8):
    t0 = time.perf_counter()
    bc.forget_stream_chunks()
    t1 = time.perf_counter()
    bc.chunk_device(buf.data_ptr(), n)
    t2 = time.perf_counter()
    s = bc.scan_ms()
    t3 = time.perf_counter()
    st = bc.stats()
    print(f"forget {1e3*(t1-t0):.3f} chunk {1e3*(t2-t1):.3f} scan_ms() {1e3*(t3-t2):.3f} total_ms {st['total_ms']:.3f}",
          flush=True)
