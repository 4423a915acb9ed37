"""Host rate of the whole-stream SHA-256 (zc_sha256_add) vs hashlib (OpenSSL, the
reference's implementation).  python tools/sha256_rate.py [MiB]"""
import ctypes
import hashlib
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from zbackup_amd.chunker import Sha256  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 512
buf = np.random.default_rng(1).integers(0, 256, mib << 20, dtype=np.uint8)
ptr = buf.ctypes.data
for name in ("zc_sha256", "hashlib"):
    t = time.perf_counter()
    if name == "hashlib":
        d = hashlib.sha256(memoryview(buf)).digest()
    else:
        h = Sha256()
        step = 64 << 20
        for o in range(0, buf.size, step):
            h.add(ptr + o, min(step, buf.size - o))
        d2 = h.finish()
    dt = time.perf_counter() - t
    print(f"{name}: {mib / 1024 / dt:.3f} GiB/s ({mib} MiB, 1 thread)")
assert d == d2
