"""Stage timings of incremental backups on one context (ZC_FLAG_SHA1): the same
8 GiB stream again, and a stream after a different one.  Debug tooling."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from zbackup_amd import BackupCreator, fill_splitmix64  # noqa: E402

n = int(float(sys.argv[1]) * 2**30) if len(sys.argv) > 1 else 8 << 30
a = torch.empty(n, dtype=torch.uint8, device="cuda")
b = torch.empty(n, dtype=torch.uint8, device="cuda")
fill_splitmix64(a.data_ptr(), n, 2024, 0)
fill_splitmix64(b.data_ptr(), n, 77, 0)
torch.cuda.synchronize()
for label, first in (("same", a), ("other", b)):
    bc = BackupCreator(65536, sha1=True, timing=True)
    bc.chunk_device(first.data_ptr(), n)
    for i in range(3):
        t = time.perf_counter()
        bc.chunk_device(a.data_ptr(), n)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        st = bc.stats()
        print(label, i, f"{dt * 1e3:.2f} ms", {k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()},
              flush=True)
    bc.close()
