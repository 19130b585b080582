#!/usr/bin/env python3
"""Generate the committed oracle fixtures under tests/golden/ (run from the repo root).

  tensile5e_oracle.npz        Tensile5e.inp (C1): disp at the 100 output steps (every 200 steps),
                              final GP stress / eqps, deletion log.
  fast_deletion_bar_oracle.npz  2x2x8 bar pulled to fracture: final disp, deletion log.

The reference itself cannot run here (no Julia), so these pin the oracle against regressions; the
oracle is pinned against the reference by the KATs/NumPy restatement in tests/test_oracle.py.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as O  # noqa: E402
from hakai import mesh  # noqa: E402
from util import fast_deletion_bar  # noqa: E402


def main():
    out = os.path.join(ROOT, "tests", "golden")
    os.makedirs(out, exist_ok=True)
    m = mesh.tensile5e_model()
    o = O.Oracle(m)
    outs = []
    for k in range(100):
        o.run(1 + 200 * k, 200)
        outs.append(o.s["disp"].copy())
    np.savez_compressed(os.path.join(out, "tensile5e_oracle.npz"), disp_out=np.array(outs),
                        integ_stress=o.s["integ_stress"], integ_eq_plastic_strain=o.s["integ_eq_plastic_strain"],
                        deletions=np.array(o.deletions, np.int64).reshape(-1, 2))
    m = fast_deletion_bar()
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    np.savez_compressed(os.path.join(out, "fast_deletion_bar_oracle.npz"), disp=o.s["disp"],
                        deletions=np.array(o.deletions, np.int64).reshape(-1, 2))
    print("deletions tensile5e / bar:", len(outs), o.deletions[:5], len(o.deletions))


if __name__ == "__main__":
    main()
