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
        keys = rng.integers(1, 2**63, k, dtype=np.int64).astype(np.uint64)
        shas = rng.integers(0, 256, (k, 16), dtype=np.uint8)
        with BackupCreator(65536, sha1=False, timing=True) as bc:
            t0 = time.perf_counter()
            bc.seed_index_arrays(shas, keys, 65536)
            seed_s = time.perf_counter() - t0
            bc.chunk_device(buf.data_ptr(), n)  # warm-up (builds the screen's filters)
            dts = []
            for _ in range(3):
                torch.cuda.synchronize()
                t = time.perf_counter()
                bc.chunk_device(buf.data_ptr(), n)
                torch.cuda.synchronize()
                dts.append(time.perf_counter() - t)
            dt = min(dts)
            st = bc.stats()
        print(f"K={k:8d}  {n / dt / 2**30:8.1f} GiB/s  total {dt * 1e3:8.2f} ms  fscan {st['fscan_ms']:.2f} ms"
              f"  runs {st['fscan_runs']}  walk {st['walk_ms']:.2f} ms  fbatch {st['fbatch_ms']:.2f} ms"
              f"  seed {seed_s:.2f} s", flush=True)


if __name__ == "__main__":
    main()
