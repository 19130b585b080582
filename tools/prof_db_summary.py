#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace results database (rocpd sqlite):
launches, total and average duration, and time per step per rank (--steps, --ranks)."""
import argparse
import re
import sqlite3


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    if "rocprim" in name:
        return "rocprim::" + ("init_lookback_scan_state" if "init_lookback" in name else "scan")
    return re.sub(r"\(.*", "", name)[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--csv", default="", help="also write every kernel's row to this CSV file")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, count(*), sum(duration) from kernels group by name "
                       "order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':70s} {'launches':>8s} {'avg_us':>9s} {'us/step/rank':>13s} {'share':>6s}")
    for n, c, d in rows[:a.top]:
        print(f"{short(n):70s} {c:8d} {d / c / 1e3:9.2f} {d / 1e3 / (a.steps * a.ranks):13.2f} {d / tot:6.1%}")
    if a.csv:
        import csv
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "launches", "avg_us", "us_per_step_per_rank", "share"])
            for n, c, d in rows:
                w.writerow([n, c, round(d / c / 1e3, 3), round(d / 1e3 / (a.steps * a.ranks), 3), round(d / tot, 5)])


if __name__ == "__main__":
    main()
