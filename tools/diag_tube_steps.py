"""Diagnostic: first steps of a deck on the GPU vs the oracle, pipelined vs simple element kernel."""
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
z = np.load(os.path.join(ROOT, "tests", "golden", f"deck_{name}.npz"))
m = model_from_arrays(z, name)
print("contact_flag", m.contact_flag, "materials", [(mt.plastic.shape[0], mt.ductile.shape[0]) for mt in m.materials])
for pipe in (512, 0):
    o = O.Oracle(m)
    with Solver(m) as sv:
        sv.set_tuning("elem_pipe_blocks", pipe)
        for t in range(1, 6):
            o.run(t, 1)
            sv.step(t, 1)
            g = sv.download()
            e_d = np.linalg.norm(g.disp - o.s["disp"]) / max(np.linalg.norm(o.s["disp"]), 1e-300)
            e_s = np.abs(g.integ_stress - o.s["integ_stress"]).max() / max(np.abs(o.s["integ_stress"]).max(), 1e-300)
            e_q = np.abs(g.Qe - o.s["Qe"]).max() / max(np.abs(o.s["Qe"]).max(), 1e-300)
            bad = np.nonzero(np.abs(g.Qe - o.s["Qe"]).max(axis=1) > 1e-9 * max(np.abs(o.s["Qe"]).max(), 1e-300))[0]
            print(f"pipe {pipe} step {t}: disp {e_d:.2e} stress {e_s:.2e} Qe {e_q:.2e} bad elems {bad[:8].tolist()}")
