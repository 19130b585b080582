"""Diagnostic: GPU vs oracle relative displacement error along a reference deck run
(tests/golden/deck_<name>.npz model), with the number of contact events per checkpoint."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("hakai-fem_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, d))
import oracle as O  # noqa: E402
from deck_fixtures import model_from_arrays  # noqa: E402
from hakai.solver import Solver  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "crash_tube_80_350_solid"
every = int(sys.argv[2]) if len(sys.argv) > 2 else 100
z = np.load(os.path.join(ROOT, "tests", "golden", f"deck_{name}.npz"))
m = model_from_arrays(z, name)
steps = int(z["steps"])
o = O.Oracle(m)
with Solver(m) as sv:
    for t0 in range(1, steps + 1, every):
        n = min(every, steps - t0 + 1)
        o.run(t0, n)
        sv.step(t0, n)
        g = sv.download(disp=True, element_flag=True)
        err = np.linalg.norm(g.disp - o.s["disp"]) / max(np.linalg.norm(o.s["disp"]), 1e-300)
        st = sv.contact_stats()
        print(f"step {t0 + n - 1:5d}  rel err {err:.3e}  events {st['events']}  flags equal "
              f"{np.array_equal(g.element_flag, o.s['element_flag'])}", flush=True)
