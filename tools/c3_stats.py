#!/usr/bin/env python3
"""Owner-assembly list statistics of the C3 bench workload (and optional other configs): own_slots
(LDS running sums a block keeps open), rows, entries, super-batch size, and the element kernel's
LDS budget in each mode."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
from hakai import mesh  # noqa: E402
from hakai.solver import Solver  # noqa: E402

cases = {"C3": lambda: mesh.config_c3(v_end=5e5)}
if "c5" in sys.argv:
    cases["C5slab"] = lambda: mesh.config_c5(layers=200)
for name, mk in cases.items():
    m = mk()
    diag, _ = m.lumped_mass()
    with Solver(m, diag_M=diag) as sv:
        sv.set_tuning("graph", 0)
        sv.step(1, 2)
        st = {k: sv.stat(k) for k in ("own_steps", "own_slots", "own_rows", "own_entries", "own_superbatch")}
    print(json.dumps({"config": name, "elements": m.nElement, "nodes": m.nNode, **st}), flush=True)
