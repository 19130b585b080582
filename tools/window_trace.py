#!/usr/bin/env python3
"""Kernel-trace summary of bench.py's deletion window.

`tools/gpu_r6.sh window` runs `bench.py --deletion-window 1 --compare-fused 0 --breakdown 0
--cpu-baseline 0` under `rocprofv3 --kernel-trace`. Nothing runs after the window, so the last
2 x steps + 2 element dispatches (k_element_pipe, any instantiation) are, per mode, one untimed
planning step and the window (headline mode, then the other; bench.deletion_window), and the `steps`
element dispatches before them are
the last steps of the run-up (steps 7921-7940: the same bar just before its first deletion, no
deletion yet). Prints one JSON object: per mode the element kernel's duration per window step (so the
deletion steps show), their mean against the run-up's, and the nodal/BC time per step."""
import argparse
import csv
import glob
import json
import os
import statistics


def rows(d):
    fs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not fs:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    out = []
    for f in fs:
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    out.sort(key=lambda r: int(r["Start_Timestamp"]))
    return out


def dur_ms(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kt", required=True)
    ap.add_argument("--log", default=None, help="bench output (its JSON line carries config.deletion_window)")
    ap.add_argument("--first", type=int, default=0, help="without --log (tools/window_control.py): first window step")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    if a.log:
        line = json.loads([l for l in open(a.log) if l.startswith("{")][-1])
        win = line["config"]["deletion_window"]
        steps, first = win["steps"], win["first_step"]
        head = line["config"]["element_mode"]
    else:  # the control sequence: fused, then reference order
        win, steps, first, head = None, a.steps, a.first, "fused"
    modes = [head, "exact" if head == "fused" else "fused"]
    rs = rows(a.kt)
    el_idx = [i for i, r in enumerate(rs) if "k_element_pipe<" in r["Kernel_Name"]]
    warm = win.get("warm_steps_per_mode") if win else None
    if warm:
        # bench.deletion_window (round 6): headline run on to the hand-off, 'warm' more steps (the
        # checker's start), then per mode 'warm' untimed steps from the hand-off and the timed window,
        # then the checked reference-order run from the checker's start (after an upload)
        n = steps
        if len(el_idx) < 2 * n + 2 * (warm + n) + warm:
            raise SystemExit("too few element dispatches in the trace")
        k_other = len(el_idx) - n - n              # other mode's timed window
        k_head = k_other - warm - n                # headline's timed window
        k_cont = k_head - warm - warm              # continuation after the hand-off
        groups = {"run_up": el_idx[k_cont + warm - n:k_cont + warm], modes[0]: el_idx[k_head:k_head + n],
                  modes[1]: el_idx[k_other:k_other + n], "checked_run_after_upload": el_idx[-n:]}
    else:
        if len(el_idx) < 3 * steps + 2:
            raise SystemExit("too few element dispatches in the trace")
        # one untimed planning step per mode from the hand-off state, then the timed window (round-6
        # first protocol, and tools/window_control.py): run-up, warm, headline window, warm, other window
        groups = {"run_up": el_idx[-3 * steps - 2:-2 * steps - 2], modes[0]: el_idx[-2 * steps - 1:-steps - 1],
                  modes[1]: el_idx[-steps:]}
    out = {"source": "rocprofv3 --kernel-trace of bench.py --deletion-window 1 (tools/gpu_r6.sh window)",
           "window_first_step": first, "steps": steps, "bench_deletion_window": win}
    for name, idx in groups.items():
        el = [dur_ms(rs[i]) for i in idx]
        # the nodal / BC kernels of a step run before its element kernel (k_nodal -> k_bc -> element)
        other = []
        for j, i in enumerate(idx):
            lo = idx[j - 1] + 1 if j > 0 else i
            other.append(sum(dur_ms(rs[k]) for k in range(lo, i)
                             if "k_nodal" in rs[k]["Kernel_Name"] or "k_bc" in rs[k]["Kernel_Name"]) if j > 0 else None)
        step0 = first - steps if name == "run_up" else first
        out[name] = {"steps": [step0, step0 + steps - 1],
                     "element_ms_per_step": [round(x, 4) for x in el],
                     "element_mean_ms": round(statistics.mean(el), 4),
                     "element_median_ms": round(statistics.median(el), 4),
                     "element_max_ms": round(max(el), 4),
                     "step_of_max": step0 + el.index(max(el)),
                     "nodal_bc_mean_ms": round(statistics.mean([x for x in other if x is not None]), 4),
                     "instantiations": sorted({rs[i]["Kernel_Name"].split("(")[0] for i in idx})}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
