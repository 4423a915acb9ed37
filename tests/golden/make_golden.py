#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ (run in the survey container,
where /root/reference exists).

Generator: oracle/_ref/liboracle_ref.so = the restated BackupCreator state
machine (oracle/zc_oracle.cpp) driving the reference's OWN RollingHash, compiled
from /root/reference/rolling_hash.cc by `make -C oracle ref`.  So every rolling
hash in these files comes from the reference's code; the boundary rules come
from the restatement (backup_creator.cc itself cannot be built here: it needs
the generated zbackup.pb.h and the libprotobuf runtime, which the image lacks).

`make_golden.py [OUTDIR]` writes into OUTDIR (default: this directory);
tests/test_oracle_ref.py regenerates into a temporary directory and diffs the
result against the committed files.

Each case is a synthetic stream spec (grammar: oracle/zc_oracle.h), so the GPU
box regenerates the exact bytes without /root/reference.  Fixture format:
  # key: value        header (case, spec, W, seed_spec)
  S <sha1_16> <rolling> <size>            static-index seed (ChunkIndex::loadIndex)
  N|D|B <offset> <size> <rolling> <sha1_16>
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import oracle  # noqa: E402

W64 = 65536

# (name, spec, W, seed_spec)
CASES = [
    # BASELINE.json configs[0]: 16 MiB random stream, W = 64 KiB
    ("c1_rand16m", "R1:16777216", W64, None),
    ("zero16m", "Z:16777216", W64, None),
    ("dup16m", "R2:8388608,C0:8388608", W64, None),
    ("shiftdup", "R3:300000,R4:1000,C0:300000", W64, None),
    ("frag50", "R5:196608,R6:50,C0:196608", W64, None),
    ("finish_big", "R7:360448", W64, None),
    ("small_tail", "R8:131172", W64, None),
    ("empty", "", W64, None),
    ("tiny100", "R9:100", W64, None),
    ("tiny1000", "R9:1000", W64, None),
    ("exact_w", "R10:65536", W64, None),
    ("w_minus_1", "R10:65535", W64, None),
    ("w_plus_1", "R10:65537", W64, None),
    ("two_w_minus_1", "R10:131071", W64, None),
    ("periodic1000", "R11:1000,C0:400000", W64, None),
    ("const255", "B255:300000", W64, None),
    ("mixed", "R12:100000,Z:200000,C50000:150000,B7:70000,C0:90000,R13:5000,C100000:140000", W64, None),
    ("seeded", "R15:12345,R14:400000,R16:70000,R14:200000", W64, "R14:400000"),
    ("w257_rand", "R20:100000", 257, None),
    ("w257_periodic", "R21:3000,C0:60000", 257, None),
    ("w1000_mixed", "R22:50000,C10000:30000,Z:5000,C0:40000", 1000, None),
    ("w4096_periodic3000", "R23:3000,C0:200000", 4096, None),
    ("w4096_shift", "R24:20000,R25:77,C0:20000,R26:300,C5:20000", 4096, None),
    ("w4096_zero_rand", "Z:40000,R31:30000,Z:50000,C0:90000", 4096, None),
    ("w1", "R27:300", 1, None),
    ("w127", "R28:5000", 127, None),
    ("w128", "R29:5000,C0:5000", 128, None),
    ("w65537", "R30:300000,C1:300000", 65537, None),
]

KAT_SPECS = [("empty", ""), ("zero65536", "Z:65536"), ("zero4464", "Z:4464"),
             ("zero3392", "Z:3392"), ("one_byte_ff", "B255:1"), ("rand100", "R99:100"),
             ("rand65536", "R1:65536"), ("rand1000003", "R98:1000003")]


def seeds_from(spec, W):
    data = oracle.gen(spec, ref=True)
    recs = oracle.chunk(data, W, ref=True)
    return [(bytes.fromhex(sha), h, s) for (k, o, s, h, sha) in recs if k == "N"]


def main(out_dir=HERE):
    oracle.build(ref=True)
    for name, spec, W, seed_spec in CASES:
        data = oracle.gen(spec, ref=True)
        seeds = seeds_from(seed_spec, W) if seed_spec else []
        recs = oracle.chunk(data, W, seeds=seeds, ref=True)
        with open(os.path.join(out_dir, f"{name}.txt"), "w") as f:
            f.write(f"# case: {name}\n# spec: {spec}\n# W: {W}\n# n: {data.size}\n")
            f.write(f"# seed_spec: {seed_spec or '-'}\n")
            f.write("# generator: oracle/_ref (restated BackupCreator + reference rolling_hash.cc)\n")
            for sha, h, s in seeds:
                f.write(f"S {sha.hex()} {h:016x} {s}\n")
            for line in oracle.format_records(recs):
                f.write(line + "\n")
        kinds = {c: sum(1 for r in recs if r[0] == c) for c in "NDB"}
        print(f"{name:22s} n={data.size:9d} W={W:6d} records={len(recs):6d} {kinds}")
    L = oracle.lib(ref=True)
    with open(os.path.join(out_dir, "kat_digest.txt"), "w") as f:
        f.write("# RollingHash::digest(buf, size) known answers, computed by the reference's\n")
        f.write("# rolling_hash.cc (oracle/_ref/liboracle_ref.so).  <name> <spec> <digest>\n")
        for name, spec in KAT_SPECS:
            d = oracle.gen(spec, ref=True)
            f.write(f"{name} {spec or '-'} {L.zco_digest(d.ctypes.data, d.size):016x}\n")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else HERE)
