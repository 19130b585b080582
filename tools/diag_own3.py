"""Diagnostic: the element-force row that differs between owner-computed and fe assembly after one
step: full-precision values of the element's 8 rows in both modes."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from hakai.solver import Solver  # noqa: E402
from util import fast_deletion_bar  # noqa: E402

m = fast_deletion_bar(4, 4, 400)
nE = m.nElement
out = {}
for own in (0, 1):
    for blocks in (16,):
        with Solver(m) as sv:
            sv.set_tuning("elem_pipe_min", 0)
            sv.set_tuning("elem_pipe_blocks", blocks)
            sv.set_tuning("graph", 0)
            sv.set_tuning("own_assembly", own)
            sv.step(1, 1)
            g = sv.download()
            out[own] = g.Qe.reshape(nE, 8, 3)
np.set_printoptions(precision=17)
for e in (6392, 6388, 6393, 6396):
    for k in range(8):
        a, b = out[0][e, k], out[1][e, k]
        flag = "  <-- differs" if not np.array_equal(a, b) else ""
        print(e, k, m.elementmat[e, k] - 1, a.tolist(), b.tolist(), flag)
d = np.nonzero(np.abs(out[0] - out[1]).max(axis=2))
print("all differing rows:", list(zip(*d)))
