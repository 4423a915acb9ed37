"""Readers for the committed golden fixtures (tests/golden/*.txt)."""
import glob
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_case(path):
    meta, seeds, recs = {}, [], []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if line.startswith("# ") and ":" in line:
                k, v = line[2:].split(":", 1)
                meta[k.strip()] = v.strip()
            elif line.startswith("S "):
                _, sha, h, size = line.split()
                seeds.append((bytes.fromhex(sha), int(h, 16), int(size)))
            elif line and line[0] in "NDB":
                k, off, size, h, sha = line.split()
                recs.append((k, int(off), int(size), int(h, 16), sha))
    meta["W"] = int(meta["W"])
    meta["n"] = int(meta["n"])
    if meta.get("spec") is None:
        meta["spec"] = ""
    return meta, seeds, recs


def case_paths():
    return sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.txt")) if not p.endswith("kat_digest.txt"))


def case_names():
    return [os.path.basename(p)[:-4] for p in case_paths()]


def kats():
    out = []
    with open(os.path.join(GOLDEN, "kat_digest.txt")) as f:
        for line in f:
            if line.startswith("#") or not line.strip():
                continue
            name, spec, d = line.split()
            out.append((name, "" if spec == "-" else spec, int(d, 16)))
    return out
