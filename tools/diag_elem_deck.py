"""Diagnostic: drop-in cal_stress_hexa (GPU) vs the oracle on a reference deck's mesh, per element."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("hakai-fem_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, d))
import hakai  # noqa: E402
import oracle as O  # noqa: E402
from deck_fixtures import model_from_arrays  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "crash_tube_80_350_solid"
z = np.load(os.path.join(ROOT, "tests", "golden", f"deck_{name}.npz"))
m = model_from_arrays(z, name)
nE, nN = m.nElement, m.nNode
rng = np.random.default_rng(3)
from util import random_state  # noqa: E402
st, sn, eq, ys = random_state(rng, nE)
amp = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-4
pos = m.coordmat + rng.normal(0, 0.01, size=m.coordmat.shape)
dd = rng.normal(0, amp, size=3 * nN)
flag = np.ones(nE, np.int64)
o = O.Oracle(m)
Qo = np.zeros((nE, 24)); sto, sno, eqo, yso, vo = st.copy(), sn.copy(), eq.copy(), ys.copy(), np.zeros(nE)
O.cal_stress_hexa(o, Qo, sto, sno, yso, eqo, np.ascontiguousarray(pos), dd, flag, vo)
Qg = np.zeros((nE, 24)); stg, sng, eqg, ysg, vg = st.copy(), sn.copy(), eq.copy(), ys.copy(), np.zeros(nE)
hakai.cal_stress_hexa(Qg, stg, sng, ysg, eqg, pos, dd, m.elementmat, flag, 8, None, m.materials,
                      m.element_material, 1.0, vg)
de = np.abs(Qg - Qo).max(axis=1) / (np.abs(Qo).max() + 1e-300)
ds = np.abs(stg - sto).reshape(nE, 8, 6).max(axis=(1, 2)) / (np.abs(sto).max() + 1e-300)
bad = np.nonzero((de > 1e-9) | (ds > 1e-9))[0]
print("elements", nE, "bad", len(bad), "max Qe err", de.max(), "max stress err", ds.max())
for e in bad[:5]:
    X = pos[m.elementmat[e] - 1]
    print("elem", e + 1, "conn", m.elementmat[e].tolist(), "vol o/g", vo[e], vg[e])
    print("   coords", np.round(X, 3).tolist())
    print("   Qe o", np.round(Qo[e, :6], 5).tolist(), "g", np.round(Qg[e, :6], 5).tolist())
