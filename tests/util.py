"""Test helpers: small synthetic models and comparison metrics."""
import numpy as np

from hakai import mesh
from hakai.model import BCGroup, Material, Model


def rel_err(a, b):
    a, b = np.asarray(a), np.asarray(b)
    den = max(np.max(np.abs(b)), 1e-300)
    return float(np.max(np.abs(a - b)) / den)


def small_bar(nx=3, ny=2, nz=6, v_end=2e5, perturb=0.02, seed=3, material=None, n_steps=400, d_time=1e-7):
    mat = material or mesh.steel_ductile()
    return mesh.bar_model(nx, ny, nz, mat, lambda z, L: v_end * z / L, perturb=perturb, seed=seed,
                          d_time=d_time, n_steps=n_steps, name="small_bar")


def fast_deletion_bar(nx=2, ny=2, nz=8, seed=5):
    """Bar pulled hard at the free end so plastic flow and ductile deletion happen in ~1-2 k steps."""
    m = mesh.bar_model(nx, ny, nz, mesh.steel_ductile(), 0.0, perturb=0.02, seed=seed, d_time=2e-8,
                       n_steps=3000, name="fast_deletion")
    top = mesh.plane_nodes(nx, ny, nz)
    m.bc.append(BCGroup([(top * 3, 4.0)], np.array([0.0, 3000 * 2e-8]), np.array([0.0, 1.0])))
    return m


def random_state(rng, nE, scale=300.0, yield_frac=0.5):
    """Random pre-stress (some GPs beyond yield after the increment), strain and eqps."""
    st = rng.normal(0, scale, size=(8 * nE, 6))
    sn = rng.normal(0, 1e-3, size=(8 * nE, 6))
    eq = np.abs(rng.normal(0, 0.05, size=8 * nE))
    eq[rng.random(8 * nE) < 0.3] = 0.0
    ys = 755.0 + 50 * eq
    return st, sn, eq, ys


# State arrays a bit-exact comparison covers (hakai.solver.State fields).
STATE = ("disp", "disp_pre", "integ_stress", "integ_strain", "integ_yield_stress", "integ_eq_plastic_strain",
         "element_flag", "Q", "Qe")


def bits(x):
    """The IEEE bit patterns of a float array (so -0.0 != +0.0), or the array itself for integers."""
    x = np.ascontiguousarray(x)
    return x.view(np.uint64) if x.dtype == np.float64 else x


def bitwise_equal(a, b):
    return np.shape(a) == np.shape(b) and np.array_equal(bits(a), bits(b))


def same_state(a, b, keys=STATE, triax=True):
    """Two downloaded states are identical bit for bit (signed zeros included)."""
    for k in keys:
        x, y = getattr(a, k), getattr(b, k)
        assert bitwise_equal(x, y), f"{k}: max rel diff {rel_err(x, y):.3e}"
    if triax:
        assert bitwise_equal(a.integ_triax_stress, b.integ_triax_stress)


def shuffled(m: Model, seed: int) -> Model:
    """The same model with randomly permuted element and node numbering."""
    rng = np.random.default_rng(seed)
    nN, nE = m.nNode, m.nElement
    pe = rng.permutation(nE)                 # new element i = old element pe[i]
    pn = rng.permutation(nN)                 # new node j = old node pn[j]
    newid = np.empty(nN, np.int64)
    newid[pn] = np.arange(nN)                # old node -> new (0-based)

    def dof(d):  # 1-based dof of an old node -> 1-based dof of its new number
        d = np.asarray(d, np.int64)
        n, c = (d - 1) // 3, (d - 1) % 3
        return 3 * newid[n] + c + 1

    bc = [BCGroup([(dof(d), v) for d, v in g.entries], g.amp_time, g.amp_value) for g in m.bc]
    return Model(m.coordmat[pn], newid[m.elementmat[pe] - 1] + 1, m.element_material[pe], m.materials, bc=bc,
                 ic_dofs=dof(m.ic_dofs), ic_values=np.asarray(m.ic_values), d_time=m.d_time,
                 end_time=m.end_time, mass_scaling=m.mass_scaling, name=m.name + "_shuffled")
