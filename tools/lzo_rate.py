"""Rate of the GPU bundle compressor (tooling): payload kinds x sizes, 2 MiB
bundles, device-resident, plus liblzo2 on one core over a sample.
   python tools/lzo_rate.py [GiB] [kinds...]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import lzo_oracle  # noqa: E402
from tests.lzo_inputs import payload  # noqa: E402
from zbackup_amd import fill_splitmix64  # noqa: E402
from zbackup_amd.bundle import BundleCompressor, lzo_capacity  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
kinds = sys.argv[2:] or ["random", "text"]
B = 0x200000
for kind in kinds:
    n = int(gib * (1 << 30)) // B * B
    if kind == "random":
        d = torch.empty(n, dtype=torch.uint8, device="cuda")
        fill_splitmix64(d.data_ptr(), n, 7)
        sample = d[:64 << 20].cpu().numpy()
    else:
        base = payload(kind, 256 << 20, 3)
        d = torch.from_numpy(np.resize(base, n)).cuda()
        sample = base[:64 << 20]
    nb = n // B
    pay_off = np.arange(nb, dtype=np.uint64) * B
    cap = lzo_capacity(B)
    out_off = np.arange(nb, dtype=np.uint64) * cap
    d_out = torch.empty(nb * cap, dtype=torch.uint8, device="cuda")
    with BundleCompressor() as c:
        for it in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sizes = c.compress(d.data_ptr(), pay_off, np.full(nb, B, np.uint64), d_out.data_ptr(), out_off)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            pms, blocks = c.last_stats()
            print(f"{kind} {n / 2**30:.2f} GiB: {t * 1e3:.2f} ms = {n / t / 2**30:.1f} GiB/s, parse {pms:.2f} ms, "
                  f"ratio {sizes.sum() / n:.3f}, blocks {blocks}", flush=True)
    t0 = time.perf_counter()
    for i in range(0, len(sample), B):
        lzo_oracle.frame(sample[i:i + B].tobytes())
    t = time.perf_counter() - t0
    print(f"{kind}: liblzo2 1 core {len(sample) / t / 2**30:.3f} GiB/s on {len(sample) >> 20} MiB", flush=True)
    del d, d_out
