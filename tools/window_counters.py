#!/usr/bin/env python3
"""Per-dispatch counters of the element kernel across bench.py's deletion window.

`tools/gpu_r6.sh windowsq` runs `bench.py --deletion-window 1 --compare-fused 0 --breakdown 0
--cpu-baseline 0` under `rocprofv3 --pmc` (one pass with SQ instruction counters, one with
FETCH_SIZE). As in tools/window_trace.py, the element dispatches are, from the end: the other
mode's window (`steps`), its planning step, the headline mode's window (`steps`), its planning
step, and the run-up (steps 7921-7940). Prints, per group and per step, the counters per dispatch
(VALU / SALU / LDS / vector-memory instructions per wave, FETCH_SIZE), so a change of the element
time inside the window can be told apart as more instructions (work) or as the same instructions
waiting longer (memory, latency)."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def dispatches(d):
    fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        raise SystemExit(f"no counter_collection.csv under {d}")
    out = {}
    for f in fs:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "k_element_pipe<" not in r["Kernel_Name"]:
                    continue
                k = int(r["Dispatch_Id"])
                ent = out.setdefault(k, {"kernel": r["Kernel_Name"].split("(")[0], "c": defaultdict(float)})
                ent["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    return [out[k] for k in sorted(out)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dirs", nargs="+", required=True)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    n = a.steps
    merged = None
    for d in a.dirs:
        ds = dispatches(d)
        tail = ds[-(3 * n + 2):]
        if merged is None:
            merged = [{"kernel": x["kernel"], "c": dict(x["c"])} for x in tail]
        else:
            for m, x in zip(merged, tail):
                m["c"].update(x["c"])
    groups = {"run_up_7921_7940": merged[0:n], "headline_window_7941_7960": merged[n + 1:2 * n + 1],
              "other_window_7941_7960": merged[2 * n + 2:3 * n + 2]}
    res = {"source": "rocprofv3 --pmc passes over bench.py --deletion-window 1 (tools/gpu_r6.sh windowsq)",
           "per_dispatch": {}}
    for name, g in groups.items():
        rows = []
        for x in g:
            c = x["c"]
            w = c.get("SQ_WAVES", 0.0) or 1.0
            rows.append({"valu_per_wave": round(c.get("SQ_INSTS_VALU", 0) / w, 1),
                         "salu_per_wave": round(c.get("SQ_INSTS_SALU", 0) / w, 1),
                         "lds_per_wave": round(c.get("SQ_INSTS_LDS", 0) / w, 1),
                         "vmem_rd_per_wave": round(c.get("SQ_INSTS_VMEM_RD", 0) / w, 1),
                         "vmem_wr_per_wave": round(c.get("SQ_INSTS_VMEM_WR", 0) / w, 1),
                         "wave_cycles_per_wave": round(c.get("SQ_WAVE_CYCLES", 0) / w, 0),
                         "fetch_size_raw": c.get("FETCH_SIZE"), "kernel": x["kernel"].split("<")[1]})
        res["per_dispatch"][name] = rows
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
