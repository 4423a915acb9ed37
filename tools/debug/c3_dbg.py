"""Debug helper: C3-style stream (second half = first half), report records
that are not DUP in the second half, and compare small sizes with the oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from zbackup_amd import BackupCreator, fill_splitmix64
W = 65536
for gib in [float(a) for a in sys.argv[1:]] or [0.25, 8.0]:
    n = int(gib * 2**30)
    buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    fill_splitmix64(buf.data_ptr(), n // 2, 2024, 0)
    buf[n // 2:].copy_(buf[: n // 2])
    torch.cuda.synchronize()
    with BackupCreator(W, sha1=False) as bc:
        bc.chunk_device(buf.data_ptr(), n)
        recs = bc.records()
        st = bc.stats()
    m = (n // 2) // W
    bad = np.nonzero(recs["kind"][m:] != 1)[0]
    print(gib, len(recs), 2 * m, st, "bad", len(bad), bad[:10], recs[m + bad[:5]] if len(bad) else "")
    if gib <= 0.5:
        from oracle import oracle
        host = buf.cpu().numpy()
        ref = oracle.chunk(host, W)
        print("oracle", len(ref), "equal", len(ref) == len(recs) and all(
            (a[1], a[2], "NDB".index(a[0])) == (int(b["offset"]), int(b["size"]), int(b["kind"])) for a, b in zip(ref, recs)))
    del buf
