"""Diagnostic: run-to-run consistency of the fe path and the owner-computed path (element forces
after one step, several grid sizes)."""
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
for G in (3, 16, 512):
    res = {}
    for own in (0, 0, 1, 1, 0):
        with Solver(m) as sv:
            sv.set_tuning("elem_pipe_min", 0)
            sv.set_tuning("elem_pipe_blocks", G)
            sv.set_tuning("graph", 0)
            sv.set_tuning("own_assembly", own)
            sv.step(1, 1)
            res.setdefault(own, []).append(sv.download().Qe.reshape(nE, 8, 3))
    for own, L in res.items():
        for i in range(1, len(L)):
            d = np.nonzero(np.abs(L[i] - L[0]).max(axis=2))
            print(f"G {G} own {own}: run {i} vs run 0: rows differing {len(d[0])} {list(zip(*d))[:4]}")
    d = np.nonzero(np.abs(res[1][0] - res[0][0]).max(axis=2))
    print(f"G {G} own vs fe: rows differing {len(d[0])} {list(zip(*d))[:4]}")
