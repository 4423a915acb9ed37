"""Time zc_chunk_device on a seeded random stream against K random static keys
(an index loaded from earlier backups, no content): how the exact screen's
key map behaves as K grows.  Tooling only.

  python tools/static_scale.py [GiB] K1 K2 ...
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zbackup_amd import BackupCreator, fill_splitmix64  # noqa: E402


def main():
    gib = float(sys.argv[1])
    ks = [int(k) for k in sys.argv[2:]]
    n = int(gib * 2**30)
    buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    fill_splitmix64(buf.data_ptr(), n, 99, 0)
    torch.cuda.synchronize()
    rng = np.random.default_rng(5)
    for k in ks:
        seeds = [(bytes(16), int(x), 65536) for x in rng.integers(0, 2**63, k, dtype=np.int64)]
        with BackupCreator(65536, seeds=seeds, sha1=False, timing=True) as bc:
            bc.chunk_device(buf.data_ptr(), n)  # warm-up
            t = time.perf_counter()
            bc.chunk_device(buf.data_ptr(), n)
            dt = time.perf_counter() - t
            st = bc.stats()
        print(f"K={k:8d}  {n / dt / 2**30:8.1f} GiB/s  total {dt * 1e3:8.2f} ms  fscan {st['fscan_ms']:.2f} ms"
              f"  runs {st['fscan_runs']}  walk {st['walk_ms']:.2f} ms  fbatch {st['fbatch_ms']:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
