import os, sys, time, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, bench
from zbackup_amd import BackupCreator
mode = sys.argv[1]
n = 8 << 30
buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
bench.fill_stream(torch, buf, n, "c2", 2024, 0)
bc = BackupCreator(65536, device=0, sha1=True, timing=True)
bc.chunk_device(buf.data_ptr(), n)
torch.cuda.synchronize()
out = []
for i in range(6):
    if mode == "sleep":
        time.sleep(0.03)
    if mode == "records":
        bc.stats(); bc.records()
    ts = time.perf_counter()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bc.chunk_device(buf.data_ptr(), n)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out.append((round((t0 - ts) * 1e3, 3), round((t1 - t0) * 1e3, 3), round((t2 - t1) * 1e3, 3), round(bc.stats()["total_ms"], 3)))
print(mode, out, flush=True)
bc.close()
