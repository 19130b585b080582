#!/usr/bin/env python3
"""How well-conditioned are the reference's own contact decks? The oracle (C restatement of HAKAI
v0.0.2) against ITSELF under a perturbation of one unit in the last place.

For each deck the committed golden fixture (tests/golden/deck_*.npz) holds the oracle's final
displacement from the deck as read. This tool runs the oracle again from the same deck with the
load perturbed by one ulp (np.nextafter towards +inf on every nonzero *Initial Conditions
velocity, or on every prescribed BC value of a deck without one), one node coordinate moved by one
ulp, or every coordinate moved by one ulp up or down (rounding-level noise everywhere, what a
re-associated element kernel injects), and reports the relative difference of the final
displacement, max|u_a - u_b| / max|u_b|, plus the deletion logs. A drift of the fused GPU element
kernel (rounding-level element differences) of the same size is then the decks' conditioning, not
a kernel error (VERDICT r2 "what's missing" 5). Output: one JSON line per (deck, perturbation).

    OMP_NUM_THREADS=4 python tools/oracle_conditioning.py [deck-substring ...]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as O  # noqa: E402
from deck_fixtures import model_from_arrays  # noqa: E402

DECKS = [("crash_tube_80_350_solid", False), ("car_crash_N2k", False), ("Charpy_test", False),
         ("bullet_impact", False), ("car_wall_N2k", True)]


def run(m, steps, indexed, threads):
    o = O.Oracle(m, nthreads=threads, contact_indexed=indexed)
    o.run(1, steps)
    return o.s["disp"].copy(), sorted(tuple(int(v) for v in x) for x in o.deletions)


def main():
    sel = sys.argv[1:]
    threads = int(os.environ.get("OMP_NUM_THREADS", "4"))
    for name, indexed in DECKS:
        if sel and not any(s in name for s in sel):
            continue
        z = np.load(os.path.join(ROOT, "tests", "golden", f"deck_{name}.npz"))
        steps = int(z["steps"])
        ref_disp = z["disp"]
        ref_del = sorted(tuple(int(v) for v in x) for x in z["deletions"])
        den = float(np.max(np.abs(ref_disp)))
        hows = os.environ.get("COND_PERTURB", "none,load,one_coord,all_coords").split(",")
        for how in hows:  # "none": the control, must reproduce the fixture
            m = model_from_arrays(z, name)
            npert = 0
            if how == "load":  # every nonzero *Initial Conditions velocity, or every BC value
                v = np.asarray(m.ic_values, np.float64).copy()
                nz = np.flatnonzero(v)
                if len(nz):
                    v[nz] = np.nextafter(v[nz], np.inf)
                    m.ic_values = v
                    npert = len(nz)
                else:
                    for g in m.bc:
                        g.entries = [(d, float(np.nextafter(val, np.inf)) if val != 0.0 else val)
                                     for d, val in g.entries]
                        npert += sum(1 for _, val in g.entries if val != 0.0)
            elif how == "one_coord":  # one coordinate of the middle node
                m.coordmat = m.coordmat.copy()
                j = m.nNode // 2
                m.coordmat[j, 0] = np.nextafter(m.coordmat[j, 0], np.inf)
                npert = 1
            elif how == "all_coords":  # every coordinate one ulp up or down (seeded): rounding noise
                rng = np.random.default_rng(0)
                c = m.coordmat.copy()
                up = rng.random(c.shape) < 0.5
                c = np.where(up, np.nextafter(c, np.inf), np.nextafter(c, -np.inf))
                m.coordmat = c
                npert = c.size
            t0 = time.time()
            d, dels = run(m, steps, indexed, threads)
            rel = float(np.max(np.abs(d - ref_disp)) / den)
            print(json.dumps({"deck": name, "steps": steps, "perturbation": how, "ulps": 0 if how == "none" else 1,
                              "perturbed_values": int(npert),
                              "final_disp_rel_diff": rel, "same_deletions": dels == ref_del,
                              "deletions": [len(dels), len(ref_del)], "oracle_s": round(time.time() - t0, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
