"""Debug helper: the dense-anchor overflow case vs the oracle, first mismatch
with context and engine stats."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from oracle import oracle
from zbackup_amd import BackupCreator

src = open(os.path.join(os.path.dirname(__file__), "..", "..", "tests", "test_gpu_parity.py")).read()
ns = {}
exec(src[src.index("def _dense_anchor_pattern"):src.index('@pytest.mark.parametrize("W", [4096, 65536])')],
     {"np": np}, ns)
for W in [int(a) for a in sys.argv[1:]] or [4096]:
    pat = ns["_dense_anchor_pattern"](W)
    body = np.tile(pat, (3 << 20) // pat.size)
    parts = {"full": np.concatenate([oracle.gen("R9:1500000"), body, oracle.gen("R10:777777"), body[:1000003]]),
             "rand+body": np.concatenate([oracle.gen("R9:1500000"), body]),
             "body": body.copy(),
             "body_small": body[: 1 << 20].copy()}
    for name, data in parts.items():
        want = oracle.chunk(data, W)
        t = torch.from_numpy(data).to("cuda")
        with BackupCreator(W) as bc:
            bc.chunk_device(t.data_ptr(), data.size)
            got = bc.record_tuples()
            st = bc.stats()
        bad = next((i for i, (a, b) in enumerate(zip(got, want)) if a != b), None)
        if bad is None and len(got) != len(want):
            bad = min(len(got), len(want))
        print(W, name, data.size, "records", len(got), len(want), "first mismatch", bad,
              {k: st[k] for k in ("anchors", "candidates", "epochs", "fscan_runs")})
        if bad is not None:
            for i in range(max(0, bad - 3), min(bad + 4, len(want))):
                print("  ", i, "got", got[i][:4] if i < len(got) else None, "want", want[i][:4])
