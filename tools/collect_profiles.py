#!/usr/bin/env python3
"""Copy one round's profile set (tools/profile_round.sh OUTDIR, run on the GPU
box) into profiles/ and write profiles/rNN_scan_profile.json: the scan's
rocprofv3 average duration, its PMC HBM bytes per launch and the build id of
the libzchunk.so that was profiled.  bench.py reports roofline.rocprof and
roofline.traffic only from a summary whose build id equals the loaded
library's, so a profile of another build is never quoted.  Tooling only.

  python tools/collect_profiles.py gpurun_out/prof_r04 4
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
SCAN = "zc_scan_kernel"


def kernel_rows(path, name):
    with open(path) as f:
        return [r for r in csv.DictReader(f) if name in r["Name"]]


def pmc_avg(path, counter, kernel=SCAN):
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None


def main():
    src, rnd = sys.argv[1], int(sys.argv[2])
    tag = f"r{rnd:02d}"
    bid = open(os.path.join(src, "build_id.txt")).read().strip()
    out = {"round": rnd, "build_id": bid, "kernel": SCAN, "bytes": 8 << 30}
    copied = []

    def copy(rel, name):
        p = os.path.join(src, rel)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(PROF, name))
            copied.append(name)
            return os.path.join(PROF, name)
        return None

    for c in ("c2", "c3", "c5", "c2sha"):
        copy(f"trace_{c}/{c}_kernel_stats.csv", f"{tag}_{c}_kernel_stats.csv")
    copy("trace_lzo/lzo_kernel_stats.csv", f"{tag}_lzo_kernel_stats.csv")
    copy("bench.jsonl", f"{tag}_bench.jsonl")
    copy("host_cpu.txt", f"{tag}_host_cpu.txt")
    stats = os.path.join(PROF, f"{tag}_c2_kernel_stats.csv")
    if os.path.exists(stats):
        rows = kernel_rows(stats, SCAN)
        if rows:
            r = rows[0]
            out["rocprof"] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) * 1e-6,
                              "min_ms": float(r["MinNs"]) * 1e-6, "max_ms": float(r["MaxNs"]) * 1e-6,
                              "source": os.path.relpath(stats, ROOT)}
    fpath = os.path.join(src, "pmc_fetch", "f_counter_collection.csv")
    wpath = os.path.join(src, "pmc_write", "w_counter_collection.csv")
    if os.path.exists(fpath) and os.path.exists(wpath):
        fk, wk = pmc_avg(fpath, "FETCH_SIZE"), pmc_avg(wpath, "WRITE_SIZE")
        if fk is not None and wk is not None:
            out["pmc"] = {"FETCH_SIZE_kB_avg": fk, "WRITE_SIZE_kB_avg": wk,
                          "hbm_bytes_per_launch": int(round((2 * fk + wk) * 1024)),
                          "correction": "gfx950: FETCH_SIZE reports 1/2 of a wide streaming read -> doubled "
                                        "(MI355X_MICROARCH.md, HBM); WRITE_SIZE exact for 16 B stores; kB = 1024 B"}
            with open(os.path.join(PROF, f"{tag}_c2_scan_pmc.csv"), "w", newline="") as f:
                w = csv.writer(f)
                w.writerow(["counter", "dispatch", "kernel", "value_kB"])
                for path, cn in ((fpath, "FETCH_SIZE"), (wpath, "WRITE_SIZE")):
                    with open(path) as g:
                        for r in csv.DictReader(g):
                            if SCAN in r["Kernel_Name"] and r["Counter_Name"] == cn:
                                w.writerow([cn, r["Dispatch_Id"], SCAN, r["Counter_Value"]])
            copied.append(f"{tag}_c2_scan_pmc.csv")
    spath = os.path.join(src, "pmc_sq", "s_counter_collection.csv")
    if os.path.exists(spath):
        sq = {}
        with open(spath) as f:
            for r in csv.DictReader(f):
                if SCAN in r["Kernel_Name"]:
                    sq.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        out["sq"] = {k: sum(v) / len(v) for k, v in sorted(sq.items())}
        with open(os.path.join(PROF, f"{tag}_c2_scan_sq_counters.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["counter", "avg_per_launch"])
            for k, v in out["sq"].items():
                w.writerow([k, v])
        copied.append(f"{tag}_c2_scan_sq_counters.csv")
    out["files"] = copied
    with open(os.path.join(PROF, f"{tag}_scan_profile.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
