"""Diagnostic: owner-computed assembly vs the fe path, step by step (stream mode); prints the first
differing nodes and how their incidences fall on the persistent blocks' batch ranges."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from hakai.solver import Solver  # noqa: E402
from util import fast_deletion_bar  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 3
m = fast_deletion_bar(4, 4, 400)
nE = m.nElement
nb = (nE + 31) // 32
bstart = [lb * nb // G for lb in range(G + 1)]
inc = [[] for _ in range(m.nNode)]
for e in range(nE):
    for k in range(8):
        inc[m.elementmat[e, k] - 1].append(e)
svs = []
for own in (0, 1):
    sv = Solver(m)
    sv.set_tuning("elem_pipe_min", 0)
    sv.set_tuning("elem_pipe_blocks", G)
    sv.set_tuning("graph", 0)
    sv.set_tuning("own_assembly", own)
    svs.append(sv)
t = 1
for n in (1, 1, 1, 1, 2, 4, 8, 16, 32, 64, 128):
    for sv in svs:
        sv.step(t, n)
    t += n
    a, b = svs[0].download(), svs[1].download()
    d = np.abs(a.disp - b.disp).reshape(-1, 3).max(axis=1)
    q = np.abs(a.Q - b.Q).reshape(-1, 3).max(axis=1)
    print(f"after step {t - 1}: disp nodes differing {np.count_nonzero(d)}, Q nodes differing {np.count_nonzero(q)}, "
          f"own_steps {svs[1].stat('own_steps')}")
    if np.count_nonzero(d) or np.count_nonzero(q):
        for node in np.nonzero(q if np.count_nonzero(q) else d)[0][:8]:
            blocks = sorted({next(lb for lb in range(G) if bstart[lb] <= e // 32 < bstart[lb + 1]) for e in inc[node]})
            print(f"  node {node}: incident elements {inc[node]} batches {[e // 32 for e in inc[node]]} blocks {blocks} "
                  f"Q fe {a.Q[3 * node:3 * node + 3]} own {b.Q[3 * node:3 * node + 3]}")
        qe = np.abs(a.Qe - b.Qe).reshape(nE, 8, 3).max(axis=2)
        for e, k in zip(*np.nonzero(qe)):
            print(f"  Qe differs: element {e} local node {k} (node {m.elementmat[e, k] - 1}) "
                  f"fe {a.Qe.reshape(nE, 8, 3)[e, k]} own {b.Qe.reshape(nE, 8, 3)[e, k]}")
        for k in ("integ_stress", "integ_strain", "integ_eq_plastic_strain", "integ_yield_stress"):
            x = np.abs(getattr(a, k) - getattr(b, k))
            print(f"  {k}: differing entries {np.count_nonzero(x)}")
        break
