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
