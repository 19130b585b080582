"""Edge cases of the element / assembly path against the oracle, and loud failure on bad input.

* Ragged incidence: every element of a bar duplicated in place (two coincident elements share all
  8 nodes), so interior nodes have 16 incident elements. The padded [nN][8] gather cannot hold them
  and the library switches to the CSR gather; the element-order sum is still the reference's
  serial assembly (v2/HAKAI_j.jl:669-675).
* Inverted elements: every element with its two node faces swapped has det J < 0 at every Gauss
  point. The reference takes |det| in B-bar (`:1736-1742`, with a warning) but the signed det in
  Bfinal, the force weight and the lumped mass (`:1436-1443`, `:1335`, `:194`); the device must do
  the same and count the negative Jacobians. (A single inverted element in a right-handed mesh makes
  the reference blow up to NaN within a few steps, so the whole mesh is mirrored.)
* Out-of-range node or material indices: the reference raises BoundsError; the C ABI returns an
  error (no partial upload, no silent clamp).
"""
import numpy as np
import pytest

from hakai.model import Model
from hakai.solver import Solver
import oracle as O
from util import rel_err, small_bar

pytestmark = pytest.mark.gpu


def _clone(m, elementmat, element_material):
    return Model(m.coordmat.copy(), elementmat, element_material, m.materials, bc=m.bc, ic_dofs=m.ic_dofs,
                 ic_values=m.ic_values, d_time=m.d_time, end_time=m.end_time, name=m.name + "_edge")


def _run_both(m, n):
    o = O.Oracle(m)
    o.run(1, n)
    with Solver(m) as sv:
        sv.step(1, n)
        g = sv.download()
        dels = [tuple(int(v) for v in x) for x in sv.deleted()]
        nneg = sv.negative_jacobians()
    return o, g, dels, nneg


def test_duplicated_elements_ragged_incidence():
    base = small_bar(3, 2, 6, v_end=2e5, n_steps=400)
    em = np.repeat(base.elementmat, 2, axis=0)
    mm = np.repeat(base.element_material, 2)
    m = _clone(base, em, mm)
    counts = np.bincount(m.elementmat.ravel())
    assert counts.max() == 16
    o, g, dels, _ = _run_both(m, 400)
    assert dels == sorted(tuple(int(v) for v in d) for d in o.deletions)
    assert np.array_equal(g.element_flag, o.s["element_flag"])
    assert rel_err(g.disp, o.s["disp"]) < 1e-6
    assert rel_err(g.integ_stress, o.s["integ_stress"]) < 1e-6
    assert np.any(g.integ_eq_plastic_strain > 0)
    # coincident twins see identical nodes and state: their Gauss-point stresses are equal
    st = g.integ_stress.reshape(-1, 2, 8, 6)
    assert rel_err(st[:, 0], st[:, 1]) < 1e-12


def test_inverted_elements_parity():
    base = small_bar(3, 2, 6, v_end=2e5, n_steps=300)
    m = _clone(base, base.elementmat[:, [4, 5, 6, 7, 0, 1, 2, 3]].copy(), base.element_material.copy())
    o, g, dels, nneg = _run_both(m, 300)
    assert np.min(o.diag_M) < 0          # signed det in the lumped mass, as in the reference
    assert nneg > 0
    assert dels == sorted(tuple(int(v) for v in d) for d in o.deletions)
    assert rel_err(g.disp, o.s["disp"]) < 1e-6
    assert rel_err(g.integ_stress, o.s["integ_stress"]) < 1e-6
    # the two sign flips (mass and force weight) cancel: same motion as the right-handed mesh
    with Solver(base) as sv:
        sv.step(1, 300)
        g0 = sv.download(disp=True)
    assert rel_err(g.disp, g0.disp) < 1e-10


@pytest.mark.parametrize("what", ["node_zero", "node_past_end", "material"])
def test_bad_indices_fail_loudly(what):
    base = small_bar(2, 2, 3)
    em, mm = base.elementmat.copy(), base.element_material.copy()
    if what == "node_zero":
        em[1, 3] = 0
    elif what == "node_past_end":
        em[2, 6] = base.nNode + 1
    else:
        mm[0] = 2
    m = _clone(base, em, mm)
    with pytest.raises(Exception, match="out of"):
        Solver(m, diag_M=np.ones(3 * m.nNode))


@pytest.mark.parametrize("case", ["ragged", "inverted"])
def test_edge_meshes_exact_mode_bitexact(case):
    """The reference-order kernel (elem_exact) on the ragged (CSR gather) and the inverted mesh
    (negative det: |det| in BVbar, signed det in Bfinal and the force weight): bit-identical."""
    base = small_bar(3, 2, 6, v_end=2e5, n_steps=300)
    if case == "ragged":
        m = _clone(base, np.repeat(base.elementmat, 2, axis=0), np.repeat(base.element_material, 2))
    else:
        m = _clone(base, base.elementmat[:, [4, 5, 6, 7, 0, 1, 2, 3]].copy(), base.element_material.copy())
    o = O.Oracle(m)
    o.run(1, 300)
    with Solver(m) as sv:
        sv.set_tuning("elem_exact", 1)
        sv.step(1, 300)
        g = sv.download()
    for k in ("disp", "disp_pre", "integ_stress", "integ_strain", "integ_eq_plastic_strain", "Q"):
        assert np.array_equal(getattr(g, k), o.s[k]), k


def test_reupload_larger_model_without_bc():
    """hakai_upload_model drops the BC tables sized for the previous mesh (the fused-BC per-dof
    table would be read past its end): a larger model uploaded into a context that had BCs steps
    like a fresh context without BCs."""
    import ctypes
    from hakai._abi import check, ptr
    small = small_bar(2, 2, 3, n_steps=50)
    big = small_bar(3, 3, 12, n_steps=50)
    I64 = ctypes.c_int64
    diag, _ = big.lumped_mass()
    with Solver(small) as sv:
        sv.step(1, 5)
        mats, keep = big.c_materials()
        check(sv.L.hakai_upload_model(sv.ctx, big.nNode, ptr(big.coordmat), big.nElement, ptr(big.elementmat, I64),
                                      ptr(big.element_material, I64), len(big.materials), mats, ptr(diag)))
        del keep
        sv.model = big
        sv.reset()
        sv.step(1, 50)
        g = sv.download(disp=True)
    nobc = _clone(big, big.elementmat.copy(), big.element_material.copy())
    nobc.bc = []
    with Solver(nobc) as sv:
        sv.step(1, 50)
        r = sv.download(disp=True)
    assert np.array_equal(g.disp, r.disp)


def _exact_state_equal(g, s):
    from util import STATE, bitwise_equal
    for k in STATE:
        assert bitwise_equal(getattr(g, k), s[k]), k


@pytest.mark.parametrize("exact", [1, 0])
def test_single_element_bar(exact):
    """The smallest mesh: one hex (8 nodes, one batch slot of 64 lanes mostly empty), plastic flow
    under the stretch field. Reference order: bit-identical to the oracle; fused: within 1e-9."""
    m = small_bar(1, 1, 1, v_end=2e5, n_steps=300)
    assert m.nElement == 1 and m.nNode == 8
    o = O.Oracle(m)
    o.run(1, 300)
    with Solver(m) as sv:
        sv.set_tuning("elem_exact", exact)
        sv.step(1, 300)
        g = sv.download()
    assert np.any(o.s["integ_eq_plastic_strain"] > 0) and np.all(np.isfinite(o.s["disp"]))
    if exact:
        _exact_state_equal(g, o.s)
    else:
        assert rel_err(g.disp, o.s["disp"]) < 1e-9
        assert rel_err(g.integ_stress, o.s["integ_stress"]) < 1e-9


def test_zero_steps_is_a_no_op():
    """hakai_step with n_steps = 0 returns success and leaves every state array as it was; the
    run then continues bit-identically to one that never made the empty call."""
    m = small_bar(3, 2, 6, v_end=2e5, n_steps=200)
    with Solver(m) as sv:
        sv.set_tuning("elem_exact", 1)
        sv.step(1, 100)
        a = sv.download()
        sv.step(101, 0)
        b = sv.download()
        for k in ("disp", "disp_pre", "velo", "integ_stress", "integ_strain", "integ_eq_plastic_strain",
                  "integ_yield_stress", "element_flag"):
            assert np.array_equal(getattr(a, k), getattr(b, k)), k
        sv.step(101, 100)
        c = sv.download()
    o = O.Oracle(m)
    o.run(1, 200)
    _exact_state_equal(c, o.s)


def test_every_element_deleted():
    """A state whose elements are all deleted (element_flag 0 everywhere, uploaded mid-run): no
    element contributes force or changes its state, no deletion is logged again, and the nodes
    run on under their own momentum and the BCs -- bit-identical to the oracle."""
    m = small_bar(3, 2, 6, v_end=2e5, n_steps=200)
    o = O.Oracle(m)
    o.run(1, 100)
    with Solver(m) as sv:
        sv.set_tuning("elem_exact", 1)
        sv.step(1, 100)
        g = sv.download()
        g.element_flag[:] = 0
        sv.upload(g)
        sv.step(101, 100)
        r = sv.download()
        dels = sv.deleted()
    o.s["element_flag"][:] = 0
    o.run(101, 100)
    assert all(int(d[0]) <= 100 for d in dels) and all(d[0] <= 100 for d in o.deletions)
    _exact_state_equal(r, o.s)
    assert not np.array_equal(r.disp, g.disp)


def _many_materials_deck():
    """fast_deletion_bar with 11 materials cycled over the elements: ten scaled steel_Ductile
    variants and one with the largest tables the ABI takes (64 plastic rows, 32 ductile rows).
    11 > kMaxLdsMats (8), so the element kernel reads the material tables from global memory."""
    from hakai import mesh
    from hakai.model import Material
    from util import fast_deletion_bar
    base = fast_deletion_bar(3, 3, 10)
    mats = []
    for i in range(10):
        pl = mesh.STEEL_PLASTIC.copy()
        pl[:, 0] *= 1 + 0.03 * i
        du = mesh.STEEL_DUCTILE.copy()
        du[:, 0] *= 1 + 0.05 * i
        mats.append(Material(f"m{i}", 7.8e-9, 210000 * (1 + 0.05 * i), 0.3 - 0.01 * i, pl, du))
    eps = np.linspace(0, 4, 64)
    tri = np.linspace(-0.3, 2.0, 32)
    mats.append(Material("largest_tables", 7.8e-9, 200000., 0.29,
                         np.stack([700 + 400 * (1 - np.exp(-5 * eps)), eps], 1),
                         np.stack([1.0 - 0.35 * (tri + 0.3) / 2.3, tri, np.full(32, 30.)], 1)))
    em = (np.arange(base.nElement) % len(mats) + 1).astype(np.int64)
    m = Model(base.coordmat.copy(), base.elementmat.copy(), em, mats, bc=base.bc, ic_dofs=base.ic_dofs,
              ic_values=base.ic_values, d_time=base.d_time, end_time=base.end_time, name="many_materials")
    return m


@pytest.mark.parametrize("exact", [1, 0])
def test_many_materials_largest_tables(exact):
    """More materials than the LDS stages and the largest plastic / ductile tables, with
    deletions in several materials (the largest-table one included): reference order bit-identical
    to the oracle, fused within 1e-6 with the same deletions."""
    m = _many_materials_deck()
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    deleted_mats = {int(m.element_material[int(e) - 1]) for _, e in o.deletions}
    assert len(deleted_mats) >= 3 and len(m.materials) in deleted_mats
    with Solver(m) as sv:
        sv.set_tuning("elem_exact", exact)
        sv.step(1, m.n_steps)
        g = sv.download()
        dels = [tuple(int(v) for v in x) for x in sv.deleted()]
    assert dels == sorted(tuple(int(v) for v in d) for d in o.deletions)
    if exact:
        _exact_state_equal(g, o.s)
    else:
        assert rel_err(g.disp, o.s["disp"]) < 1e-6
        assert rel_err(g.integ_stress, o.s["integ_stress"]) < 1e-6
