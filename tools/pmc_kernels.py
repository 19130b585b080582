#!/usr/bin/env python3
"""Per-kernel HBM traffic from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs and a kernel
trace of the same command (profiling helper, not part of the product).

Averages FETCH_SIZE and WRITE_SIZE per dispatch for every kernel whose name contains one of
--kernels (the counters' raw values are bytes x the gfx950 factors measured by tools/pmc_calib.hip:
FETCH_SIZE counts 1/2 of the bytes of coalesced reads, WRITE_SIZE counts writes exactly), and the
kernel trace's average duration, and prints one JSON object: bytes per launch and GB/s per kernel.

  python tools/pmc_kernels.py --fetch DIR --write DIR --kt DIR --kernels k_element_pipe,k_nodal
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def rows(d, suffix):
    f = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    if not f:
        raise SystemExit(f"no *{suffix} under {d}")
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


def per_kernel(d, counter, keys):
    acc = defaultdict(lambda: defaultdict(float))
    for r in rows(d, "counter_collection.csv"):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        if any(k in name for k in keys):
            acc[name][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {n: (sum(v.values()) / len(v), len(v)) for n, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kt", required=True)
    ap.add_argument("--kernels", default="k_element_pipe,k_nodal")
    ap.add_argument("--fetch-factor", type=float, default=0.5, help="FETCH_SIZE per byte read (pmc_calib)")
    ap.add_argument("--write-factor", type=float, default=1.0, help="WRITE_SIZE per byte written (pmc_calib)")
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    keys = a.kernels.split(",")
    fe = per_kernel(a.fetch, "FETCH_SIZE", keys)
    wr = per_kernel(a.write, "WRITE_SIZE", keys)
    dur = defaultdict(list)
    for r in rows(a.kt, "kernel_trace.csv"):
        if any(k in r["Kernel_Name"] for k in keys):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    out = {"label": a.label, "units": "FETCH_SIZE/WRITE_SIZE are KB in rocprofv3; bytes = KB*1024/factor",
           "kernels": {}}
    for n in sorted(set(fe) | set(wr)):
        rb = fe.get(n, (0.0, 0))[0] * 1024.0 / a.fetch_factor
        wb = wr.get(n, (0.0, 0))[0] * 1024.0 / a.write_factor
        ms = sum(dur[n]) / len(dur[n]) if dur.get(n) else None
        out["kernels"][n] = {"dispatches_fetch": fe.get(n, (0, 0))[1], "dispatches_write": wr.get(n, (0, 0))[1],
                             "read_bytes_per_launch": rb, "write_bytes_per_launch": wb,
                             "hbm_bytes_per_launch": rb + wb, "trace_avg_ms": ms, "trace_dispatches": len(dur.get(n, [])),
                             "GBs": (rb + wb) / (ms * 1e-3) / 1e9 if ms else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
