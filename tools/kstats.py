#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 results database (rocpd SQLite, the default output of
`rocprofv3 --kernel-trace`): calls, total and average duration, share. Optionally only dispatches
whose kernel name contains a substring.

    python tools/kstats.py gpurun_out/<dir>/<name>_results.db [--top 40] [--match ct_] [--csv out.csv]
"""
import argparse
import csv
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--match", default="")
    ap.add_argument("--csv", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start) from kernels "
                     "group by name order by sum(end - start) desc").fetchall()
    rows = [r for r in rows if a.match in r[0]]
    tot = sum(r[2] for r in rows) or 1
    out = [("kernel", "calls", "total_ms", "avg_us", "pct")]
    for name, n, s, avg in rows:
        short = name.replace("(anonymous namespace)::", "").split("(")[0][:90]
        out.append((short, n, round(s / 1e6, 3), round(avg / 1e3, 2), round(100 * s / tot, 2)))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            csv.writer(f).writerows(out)
    for r in out[:a.top + 1]:
        print(f"{r[0]:<92} {r[1]:>7} {r[2]:>10} {r[3]:>9} {r[4]:>6}")


if __name__ == "__main__":
    sys.exit(main())
