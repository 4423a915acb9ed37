#!/usr/bin/env python3
"""Per-kernel summary (calls, total/avg/min/max us) from a rocprofv3 rocpd
SQLite database (run_results.db).  Tooling only.

  python tools/prof_summary.py gpurun_out/prof_c2/run_results.db [--csv out.csv]
"""
import sqlite3
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:60]


def summary(db_path):
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                      "from kernels group by name order by sum(duration) desc").fetchall()
    return [(short(n), c, s / 1e3, a / 1e3, mn / 1e3, mx / 1e3) for n, c, s, a, mn, mx in rows]


def main():
    rows = summary(sys.argv[1])
    out = ["kernel,calls,total_us,avg_us,min_us,max_us"]
    out += [f"{n},{c},{s:.1f},{a:.1f},{mn:.1f},{mx:.1f}" for n, c, s, a, mn, mx in rows]
    if "--csv" in sys.argv:
        with open(sys.argv[sys.argv.index("--csv") + 1], "w") as f:
            f.write("\n".join(out) + "\n")
    for n, c, s, a, mn, mx in rows:
        print(f"{n:60s} {c:6d} {s:10.1f} {a:9.1f} {mn:9.1f} {mx:9.1f}")


if __name__ == "__main__":
    main()
