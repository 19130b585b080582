#!/usr/bin/env python3
"""Fused-kernel drift on the reference's own decks (GPU): the whole run in the default (fused)
element mode against the oracle fixtures (tests/golden/deck_*.npz), next to the decks' own 1-ulp
conditioning (profiles/r03_oracle_conditioning.jsonl, tools/oracle_conditioning.py). The numbers
behind the bounds of tests/test_gpu_decks.py. One JSON line per deck.

    python tools/deck_drift.py [deck-substring ...]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from deck_fixtures import model_from_arrays  # noqa: E402
from hakai.solver import Solver  # noqa: E402

DECKS = ["Charpy_test", "bullet_impact", "crash_tube_80_350_solid", "car_crash_N2k", "car_wall_N2k"]


def main():
    sel = sys.argv[1:]
    for name in DECKS:
        if sel and not any(s in name for s in sel):
            continue
        z = np.load(os.path.join(ROOT, "tests", "golden", f"deck_{name}.npz"))
        m = model_from_arrays(z, name)
        steps = int(z["steps"])
        t0 = time.time()
        with Solver(m) as sv:   # the test's call pattern: two calls
            sv.step(1, steps // 2)
            sv.step(1 + steps // 2, steps - steps // 2)
            g = sv.download()
            dels = [tuple(int(v) for v in x) for x in sv.deleted()]
        den = float(np.max(np.abs(z["disp"])))
        print(json.dumps({
            "deck": name, "steps": steps, "element_mode": "fused",
            "final_disp_rel_diff": float(np.max(np.abs(g.disp - z["disp"])) / den),
            "final_disp_pre_rel_diff": float(np.max(np.abs(g.disp_pre - z["disp_pre"])) / den),
            "same_deletions": dels == [tuple(int(v) for v in x) for x in z["deletions"]],
            "same_flags": bool(np.array_equal(g.element_flag, z["element_flag"])),
            "gpu_s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
