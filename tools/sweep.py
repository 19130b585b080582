#!/usr/bin/env python3
"""A/B timing of tuning variants on C3 in ONE process, interleaved rounds (guide §5.4 rule 24).

  python tools/sweep.py --variants "simple:elem_pipe_blocks=0;pipe512:elem_pipe_blocks=512"
Each variant is name:key=value[,key=value]; keys are hakai_set_tuning keys. Prints the median and
min per-step kernel times (HIP events) and whole-step wall time per variant."""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
from hakai import mesh  # noqa: E402
from hakai._abi import K_ELEMENT, K_NODAL  # noqa: E402
from hakai.solver import Solver  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layers", type=int, default=5000)
ap.add_argument("--config", choices=("c3", "c4", "c5slab", "c5"), default="c3",
                help="c3: 20x20xlayers bar; c4: two-body impact with contact; c5slab: 100x100x200; c5: 100x100x1600")
ap.add_argument("--preload", type=int, default=400)
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--variants", default="simple:elem_pipe_blocks=0;pipe512:elem_pipe_blocks=512")
ap.add_argument("--settle", type=int, default=30,
                help="untimed steps after each variant's settings (a re-plan idles the GPU, and the steps after "
                     "an idle gap run slow for ~20 steps: profiles/r06_window_control_trace.json)")
a = ap.parse_args()

variants = []
for spec in a.variants.split(";"):
    name, _, kv = spec.partition(":")
    settings = [(k, int(v)) for k, v in (x.split("=") for x in kv.split(",") if x)]
    variants.append((name, settings))

if a.config == "c3":
    m = mesh.bar_model(20, 20, a.layers, mesh.steel_ductile(), lambda z, L: 5e5 * z / L, name="C3")
elif a.config == "c4":
    m = mesh.config_c4()
else:
    m = mesh.config_c5(layers=200 if a.config == "c5slab" else 1600)
diag, _ = m.lumped_mass()
sv = Solver(m, diag_M=diag)
sv.step(1, a.preload)
sv.sync()
t = a.preload + 1
res = {n: {"el": [], "nd": [], "step": []} for n, _ in variants}
DEFAULTS = {"elem_exact": 0, "fuse_bc": 1, "elem_pipe_blocks": 512, "elem_pipe_min": 2, "elem_gp_nt": 1,
            "own_assembly": 1, "own_pass_batches": 0}
for r in range(a.rounds):
    for name, settings in variants:
        for k, v in {**DEFAULTS, **dict(settings)}.items():  # every variant from the same baseline
            sv.set_tuning(k, v)
        if a.settle:
            sv.step(t, a.settle)
            t += a.settle
        sv.profile(True)
        sv.sync()
        sv.step(t, a.steps)
        sv.sync()
        t += a.steps
        el, nd = sv.profile_read(K_ELEMENT), sv.profile_read(K_NODAL)
        sv.profile(False)
        res[name]["el"].append(el[0] / a.steps)
        res[name]["nd"].append(nd[0] / a.steps)
        sv.sync()  # wall time without profiling events
        t0 = time.perf_counter()
        sv.step(t, a.steps)
        sv.sync()
        dt = time.perf_counter() - t0
        t += a.steps
        res[name]["step"].append(dt / a.steps * 1e3)
        print(f"round {r} {name:10s} element {el[0] / a.steps:.4f} nodal {nd[0] / a.steps:.4f} step {dt / a.steps * 1e3:.4f} "
              f"superbatch {sv.stat('own_superbatch')}", flush=True)
        res[name]["own"] = {k: sv.stat(k) for k in ("own_steps", "own_rows", "own_entries", "own_banded", "own_grid", "own_round2", "own_superbatch", "own_slots")}
for name, d in res.items():
    print(f"{name:10s} element {statistics.median(d['el']):.4f} ms/step (min {min(d['el']):.4f})  "
          f"nodal {statistics.median(d['nd']):.4f} ms/step  step {statistics.median(d['step']):.4f} ms (unprofiled wall)  "
          f"{d.get('own')}")
