#!/usr/bin/env python3
"""Reference decks (tests/golden/deck_*.npz) end to end: GPU steps/s (reference-order element
arithmetic and the fused kernel, whole deck, hakai_step in chunks) beside the CPU oracle's
steps/s on a bounded sample of the same deck (first --cpu-steps steps, single thread: the
reference's CPU loop is serial, v2/HAKAI_j.jl:497-764). The oracle is the CPU baseline here, never
the product path. One JSON line per deck.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("hakai-fem_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))


def gpu_run(m, steps, exact, chunk, tuning=()):
    from hakai.solver import Solver
    with Solver(m) as sv:
        sv.set_tuning("elem_exact", exact)
        for k, v in tuning:
            sv.set_tuning(k, v)
        sv.step(1, min(steps, 200))  # warm-up (allocations, first graph capture)
        sv.sync()
    with Solver(m) as sv:
        sv.set_tuning("elem_exact", exact)
        for k, v in tuning:
            sv.set_tuning(k, v)
        t0 = time.perf_counter()
        t = 1
        while t <= steps:
            n = min(chunk, steps - t + 1)
            sv.step(t, n)
            t += n
        sv.sync()
        el = time.perf_counter() - t0
        st = sv.download()
    return el, st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--decks", default="car_crash_N2k,car_wall_N2k,Charpy_test,bullet_impact,crash_tube_80_350_solid")
    ap.add_argument("--cpu-steps", type=int, default=2000)
    ap.add_argument("--chunk", type=int, default=10000, help="steps per hakai_step call (output cadence)")
    ap.add_argument("--tuning", default="", help="extra hakai_set_tuning keys, e.g. contact_fuse_small=0")
    ap.add_argument("--modes", default="1,0", help="elem_exact values to time")
    ap.add_argument("--max-steps", type=int, default=0, help="cap the GPU steps (profiling runs)")
    a = ap.parse_args()
    tuning = [(kv.split("=")[0], int(kv.split("=")[1])) for kv in a.tuning.split(",") if kv]
    import numpy as np
    from deck_fixtures import model_from_arrays
    for name in a.decks.split(","):
        z = np.load(os.path.join(ROOT, "tests", "golden", f"deck_{name}.npz"))
        m = model_from_arrays(z, name)
        steps = int(z["steps"]) if a.max_steps <= 0 else min(int(z["steps"]), a.max_steps)
        out = {"deck": name, "elements": int(m.nElement), "nodes": int(m.nNode), "steps": steps,
               "contact_flag": int(m.contact_flag), "tuning": dict(tuning)}
        for exact in [int(x) for x in a.modes.split(",")]:
            el, st = gpu_run(m, steps, exact, a.chunk, tuning)
            key = "gpu_exact" if exact else "gpu_fused"
            out[key] = {"s": round(el, 3), "steps_per_s": round(steps / el, 1),
                        "us_per_step": round(el / steps * 1e6, 2),
                        "disp_bitexact_vs_golden": bool(np.array_equal(st.disp, z["disp"]))}
        if a.cpu_steps > 0:
            import oracle as O
            o = O.Oracle(m)
            n = min(a.cpu_steps, steps)
            t0 = time.perf_counter()
            o.run(1, n)
            el = time.perf_counter() - t0
            out["cpu_oracle"] = {"sample_steps": n, "s": round(el, 3), "steps_per_s": round(n / el, 1),
                                 "us_per_step": round(el / n * 1e6, 2), "threads": 1,
                                 "kind": "port (oracle/, single thread)"}
            if "gpu_exact" in out:
                out["gpu_exact_over_cpu"] = round(out["gpu_exact"]["steps_per_s"] / out["cpu_oracle"]["steps_per_s"], 2)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
