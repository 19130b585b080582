import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("hakai-fem_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, d))
import oracle as O
from deck_fixtures import model_from_arrays
from hakai.solver import Solver, State
z = np.load(os.path.join(ROOT, "tests", "golden", "deck_crash_tube_80_350_solid.npz"))
m = model_from_arrays(z, "tube")
o = O.Oracle(m)
o.run(1, 3)
s = o.s
st = State(s["disp"].copy(), s["disp_pre"].copy(), s["velo"].copy(), s["Q"].copy(), s["integ_stress"].copy(),
           s["integ_strain"].copy(), s["integ_yield_stress"].copy(), s["integ_eq_plastic_strain"].copy(),
           s["integ_triax_stress"].copy(), s["element_flag"].copy(), s["Qe"].copy())
u3, up3 = s["disp"].copy(), s["disp_pre"].copy()
with Solver(m) as sv:
    sv.upload(st)
    f = sv.contact_force(4)
    fo, nev = o.contact_force()
    print("contact force step 4: equal", np.array_equal(f, fo), "max diff", np.abs(f - fo).max(), "events", nev)
    sv.step(4, 1)
    g = sv.download()
o.run(4, 1)
so, sg = o.s["integ_stress"].reshape(-1, 8, 6), g.integ_stress.reshape(-1, 8, 6)
d = np.abs(sg - so).max(axis=(1, 2))
print("disp rel err", np.linalg.norm(g.disp - o.s["disp"]) / np.linalg.norm(o.s["disp"]))
print("stress worst", d.max(), "elems", np.nonzero(d > 1e-6)[0][:10].tolist())
e = 344
n = m.elementmat[e] - 1
print("elem", e, "mat", m.element_material[e], "conn", m.elementmat[e].tolist())
print("eqps o", o.s["integ_eq_plastic_strain"][8*e:8*e+8].tolist())
print("eqps g", g.integ_eq_plastic_strain[8*e:8*e+8].tolist())
print("ys before", s["integ_yield_stress"][8*e:8*e+8].tolist())
print("mat plastic", m.materials[m.element_material[e]-1].plastic.tolist())
np.savez("gpurun_out/tube_e344.npz", X=m.coordmat[n], u3=u3.reshape(-1,3)[n], up3=up3.reshape(-1,3)[n],
         u4=o.s["disp"].reshape(-1,3)[n], sig3=s["integ_stress"][8*e:8*e+8], so=so[e], sg=sg[e])
