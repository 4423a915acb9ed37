#!/usr/bin/env python3
"""Per-launch durations of the grid SHA-1 kernel from a rocprofv3 kernel
trace, in launch order, with the kernels that overlapped each launch and for
how long (tooling only).

  python tools/sha_launches.py PATH/TO/x_kernel_trace.csv
"""
import csv
import sys
from collections import Counter


def name(r):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0].split("::")[-1]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name(r)) for r in rows)
    t0 = ks[0][0]
    durs = []
    for s in ks:
        if s[2] != "zc_sha1_grid16_kernel":
            continue
        ov = Counter()
        for k in ks:
            if k is not s:
                o = min(k[1], s[1]) - max(k[0], s[0])
                if o > 0:
                    ov[k[2]] += o / 1e3
        d = (s[1] - s[0]) / 1e3
        durs.append(d)
        top = ", ".join(f"{a} {b:.1f}" for a, b in ov.most_common(3))
        print(f"{len(durs):3d} at {(s[0] - t0) / 1e6:8.2f} ms: {d:7.1f} us  beside: {top}")
    if durs:
        rest = durs[1:] or durs
        print(f"launches {len(durs)}: avg {sum(durs) / len(durs):.1f} us, max {max(durs):.1f} (launch "
              f"{durs.index(max(durs)) + 1}); without the first: avg {sum(rest) / len(rest):.1f}, max {max(rest):.1f}; "
              f"last 20: avg {sum(durs[-20:]) / len(durs[-20:]):.1f}, max {max(durs[-20:]):.1f}")


if __name__ == "__main__":
    main()
