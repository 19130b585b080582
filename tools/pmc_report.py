#!/usr/bin/env python3
"""Turn rocprofv3 outputs into the bench's roofline evidence (profiles/).

1. Calibration (tools/pmc_calib.hip): FETCH_SIZE / WRITE_SIZE per known byte for each access width.
2. Element kernel: average FETCH_SIZE / WRITE_SIZE per launch over the hot instantiation's
   dispatches of the bench's timed region -- k_element_pipe with STORE_TRIAX = false (a call's last
   step stores triaxiality and the element forces too, a different, heavier instantiation), the last
   `--steps - 1` of them (bench.py --breakdown 0 --compare-fused 0: nothing runs after the timed
   call) -- corrected by the factor of the kernel's dominant access pattern (8-B-per-lane coalesced
   SoA loads / stores) -> HBM bytes per launch ("traffic"), reported against the algorithmic bytes
   both without and with the owner-assembly outputs (entry lists, Q, exported rows).
3. Kernel trace: average duration of the same dispatches, to compare with the HIP-event average the
   bench reports.
Writes profiles/element_pmc.json (read by bench.py) and prints a summary.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

CALIB = {  # kernel-name prefix -> (counter, bytes per dispatch, pattern)
    "void calib_read<double>": ("FETCH_SIZE", 1 << 30, "read 8B/lane"),
    "void calib_read<int>": ("FETCH_SIZE", 1 << 30, "read 4B/lane"),
    "calib_read_d2": ("FETCH_SIZE", 1 << 30, "read 16B/lane"),
    "calib_read_aos3": ("FETCH_SIZE", ((1 << 30) // 24) * 24, "read 3x8B/lane stride 24B"),
    "void calib_write<double>": ("WRITE_SIZE", 1 << 30, "write 8B/lane"),
    "void calib_write<int>": ("WRITE_SIZE", 1 << 30, "write 4B/lane"),
    "calib_write_d2": ("WRITE_SIZE", 1 << 30, "write 16B/lane"),
    "calib_write_aos3": ("WRITE_SIZE", ((1 << 30) // 24) * 24, "write 3x8B/lane stride 24B"),
    "calib_read_nt": ("FETCH_SIZE", 1 << 30, "read 8B/lane nontemporal"),
    "calib_write_nt": ("WRITE_SIZE", 1 << 30, "write 8B/lane nontemporal"),
}


def _rows(d, suffix):
    fs = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    if not fs:
        raise SystemExit(f"no *{suffix} under {d}")
    with open(fs[0]) as f:
        return list(csv.DictReader(f))


def counters(d):
    """{(dispatch_id): (kernel, {counter: value})} in dispatch order."""
    out = {}
    for r in _rows(d, "counter_collection.csv"):
        k = int(r["Dispatch_Id"])
        ent = out.setdefault(k, (r["Kernel_Name"], defaultdict(float)))
        ent[1][r["Counter_Name"]] += float(r["Counter_Value"])
    return [out[k] for k in sorted(out)]


def calib_factors(fetch_dir, write_dir):
    fac = {}
    for d in (fetch_dir, write_dir):
        for name, cs in counters(d):
            for pre, (cn, nbytes, pat) in CALIB.items():
                if name.startswith(pre) and cn in cs:
                    fac.setdefault(pat, []).append(cs[cn] * 1024.0 / nbytes)
    return {p: min(v) if v else None for p, v in fac.items()}  # min over the two repetitions


def hot(name):
    """The timed region's instantiation: k_element_pipe<DO_DELETE, STORE_TRIAX = false, ...>."""
    if "k_element_pipe<" not in name:
        return False
    args = name.split("k_element_pipe<", 1)[1].split(">", 1)[0].split(",")
    return len(args) > 1 and args[1].strip() == "false"


def last_element(d, cn, steps):
    vals = [cs[cn] for name, cs in counters(d) if hot(name) and cn in cs]
    vals = vals[-(steps - 1):]
    return sum(vals) / len(vals) * 1024.0 if vals else None


def trace_avg_ms(kt_dir, steps):
    rows = [r for r in _rows(kt_dir, "kernel_trace.csv") if hot(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-(steps - 1):]
    ns = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    return sum(ns) / len(ns) / 1e6, rows[-1]["Kernel_Name"] if rows else "", len(rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calib-fetch", required=True)
    ap.add_argument("--calib-write", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kt", required=True)
    ap.add_argument("--pmc-steps", type=int, required=True, help="timed steps of the PMC bench runs")
    ap.add_argument("--kt-steps", type=int, required=True, help="timed steps of the kernel-trace bench run")
    ap.add_argument("--alg-bytes", type=float, default=None, help="algorithmic bytes per element launch")
    ap.add_argument("--alg-bytes-own", type=float, default=None,
                    help="the same plus the owner-assembly outputs (entry lists, Q, exported rows)")
    ap.add_argument("--element-mode", default=None, help="bench element mode the counters were taken in")
    ap.add_argument("--elements", type=int, default=None, help="elements of the profiled model (bench checks it)")
    ap.add_argument("--out", default="profiles/element_pmc.json")
    ap.add_argument("--round", default=None, help="round / tree label recorded in the file")
    a = ap.parse_args()
    fac = calib_factors(a.calib_fetch, a.calib_write)
    fr, fw = fac.get("read 8B/lane"), fac.get("write 8B/lane")
    raw_f = last_element(a.fetch, "FETCH_SIZE", a.pmc_steps)
    raw_w = last_element(a.write, "WRITE_SIZE", a.pmc_steps)
    traffic = None
    if fr and fw and raw_f is not None and raw_w is not None:
        traffic = raw_f / fr + raw_w / fw
    avg_ms, kname, n_kt = trace_avg_ms(a.kt, a.kt_steps)
    res = {
        "kernel": kname,
        "round": a.round,
        "element_mode": a.element_mode,
        "elements": a.elements,
        "calibration_counter_bytes_per_byte": fac,
        "fetch_size_bytes_raw_per_launch": raw_f,
        "write_size_bytes_raw_per_launch": raw_w,
        "hbm_read_bytes_per_launch": raw_f / fr if raw_f is not None and fr else None,
        "hbm_write_bytes_per_launch": raw_w / fw if raw_w is not None and fw else None,
        "hbm_bytes_per_launch": traffic,
        "correction": "FETCH_SIZE / f(read 8B/lane) + WRITE_SIZE / f(write 8B/lane), factors from tools/pmc_calib.hip",
        "hbm_bytes_per_launch_nt_factors": (raw_f / fac["read 8B/lane nontemporal"] + raw_w / fac["write 8B/lane nontemporal"])
        if fac.get("read 8B/lane nontemporal") and fac.get("write 8B/lane nontemporal") and raw_f and raw_w else None,
        "algorithmic_bytes_per_launch": a.alg_bytes,
        "traffic_over_algorithmic": traffic / a.alg_bytes if traffic and a.alg_bytes else None,
        "algorithmic_bytes_per_launch_with_assembly_outputs": a.alg_bytes_own,
        "traffic_over_algorithmic_with_assembly_outputs": traffic / a.alg_bytes_own
        if traffic and a.alg_bytes_own else None,
        "kernel_trace_avg_ms": avg_ms,
        "kernel_trace_dispatches": n_kt,
        "dispatches_used": "the hot instantiation (STORE_TRIAX=false) of the timed call, no breakdown pass",
    }
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
