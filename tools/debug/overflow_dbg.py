"""Debug helper (tooling only): time the run-overflow screen case of
tests/test_gpu_screen.py and print the engine's stage stats."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from oracle import oracle
from zbackup_amd import BackupCreator
W = int(sys.argv[1]) if len(sys.argv) > 1 else 200
parts = [f"Z:{W + 50}"]
for i in range(9000):
    parts.append(f"R{i + 7}:{7 + i % 13}")
    parts.append(f"Z:{W + 40 + i % 37}")
data = oracle.gen(",".join(parts))
t = torch.from_numpy(data).to("cuda")
for staged in (True, False):
    t0 = time.time()
    with BackupCreator(W, sha1=True, timing=True, staged_screen=staged) as bc:
        bc.chunk_device(t.data_ptr(), data.size)
        recs = bc.record_tuples()
        st = bc.stats()
    print("staged" if staged else "lane", round(time.time() - t0, 2), "s", len(recs), {k: (round(v, 2) if isinstance(v, float) else v) for k, v in st.items()}, flush=True)
t0 = time.time(); want = oracle.chunk(data, W); print("oracle", round(time.time() - t0, 2), recs == want, flush=True)
