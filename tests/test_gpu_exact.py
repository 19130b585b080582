"""Reference-order element kernel (tuning key "elem_exact", the mode hakai_run_inp uses): the
element update follows cal_stress_hexa's own arithmetic operation for operation
(v2/HAKAI_j.jl:1033-1371 with cal_BVbar_hexa :1705-1784 and cal_Bfinal :1415-1519), so -- with
the bit-exact nodal update, Q assembly and contact force -- the GPU trajectory equals the oracle's
BIT FOR BIT (IEEE bit patterns, signed zeros included: the kernel drops the reference's
structural-zero terms, which can only change the sign of a zero intermediate, never a stored value;
tests/test_exact_chains.py). Triaxiality is the one value computed differently (invariant form
instead of the reference's closed-form eigenvalues, equal to rounding); it enters only the
deletion test and the output, so it is compared to 1e-12 and the deletion logs must be identical.
The persistent kernel runs with owner-computed assembly (the default) and without it.
"""
import numpy as np
import pytest

import hakai
from hakai import mesh
from hakai.solver import Solver
import oracle as O
from util import STATE, bitwise_equal, fast_deletion_bar, random_state, rel_err, small_bar

pytestmark = pytest.mark.gpu


def _assert_state_bitexact(g, s):
    for k in STATE:
        a, b = getattr(g, k), s[k]
        assert bitwise_equal(a, b), f"{k}: max rel diff {rel_err(a, b):.3e}"
    assert rel_err(g.integ_triax_stress, s["integ_triax_stress"]) < 1e-12


@pytest.mark.parametrize("mat", ["ductile", "elastic"])
def test_exact_dropin_bitexact(mat, monkeypatch):
    """cal_stress_hexa drop-in in exact mode equals the oracle's element update bit for bit."""
    monkeypatch.setenv("HAKAI_ELEM_EXACT", "1")
    rng = np.random.default_rng(11)
    material = mesh.steel_ductile() if mat == "ductile" else mesh.steel_elastic()
    m = small_bar(4, 3, 5, material=material, perturb=0.05)
    nE, nN = m.nElement, m.nNode
    st, sn, eq, ys = random_state(rng, nE)
    pos = m.coordmat + rng.normal(0, 0.01, size=m.coordmat.shape)
    dd = rng.normal(0, 2e-3, size=3 * nN)
    flag = np.ones(nE, np.int64)
    flag[[2, 7]] = 0
    o = O.Oracle(m)
    Qo = np.zeros((nE, 24))
    sto, sno, eqo, yso, vo = st.copy(), sn.copy(), eq.copy(), ys.copy(), np.zeros(nE)
    O.cal_stress_hexa(o, Qo, sto, sno, yso, eqo, np.ascontiguousarray(pos), dd, flag, vo)
    Qg = np.zeros((nE, 24))
    stg, sng, eqg, ysg, vg = st.copy(), sn.copy(), eq.copy(), ys.copy(), np.zeros(nE)
    hakai.cal_stress_hexa(Qg, stg, sng, ysg, eqg, pos, dd, m.elementmat, flag, 8, None, m.materials,
                          m.element_material, 1.0, vg)
    for a, b, name in ((stg, sto, "stress"), (sng, sno, "strain"), (eqg, eqo, "eqps"), (ysg, yso, "yield"),
                       (Qg, Qo, "Qe"), (vg[flag == 1], vo[flag == 1], "volume")):
        assert bitwise_equal(a, b), f"{name}: max rel diff {rel_err(a, b):.3e}"
    if mat == "ductile":
        assert np.any(eqg != eq)


def test_exact_tensile5e_bitexact():
    """Tensile5e.inp (C1), all 20 000 steps, element 3 deleted at step 15153: bit-identical."""
    m = mesh.tensile5e_model()
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    with Solver(m) as sv:
        sv.set_tuning("elem_exact", 1)
        sv.step(1, m.n_steps)
        g = sv.download()
        dels = [tuple(x) for x in sv.deleted()]
    assert dels == o.deletions == [(15153, 3)]
    _assert_state_bitexact(g, o.s)


@pytest.mark.parametrize("pipe_min,own,blocks", [(0, 1, 512), (0, 1, 3), (0, 0, 512), (2, 1, 512)])
def test_exact_bar_with_deletion_bitexact(pipe_min, own, blocks):
    """Deletion bar: the persistent pipelined exact kernel (pipe_min 0) with owner-computed
    assembly (one or several batches per block) and with the fe gather, and the one-batch kernel."""
    m = fast_deletion_bar(3, 3, 10)
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    assert len(o.deletions) > 0
    with Solver(m) as sv:
        sv.set_tuning("elem_exact", 1)
        sv.set_tuning("elem_pipe_min", pipe_min)
        sv.set_tuning("elem_pipe_blocks", blocks)
        sv.set_tuning("own_assembly", own)
        sv.step(1, 1000)
        sv.step(1001, m.n_steps - 1000)
        g = sv.download()
        dels = [tuple(x) for x in sv.deleted()]
        own_steps = sv.stat("own_steps")
    assert (own_steps > 0) == (own == 1 and pipe_min == 0)
    assert dels == sorted(o.deletions)
    _assert_state_bitexact(g, o.s)


def test_exact_elastic_bar_bitexact():
    """Elastic material (no *Plastic): the any_plastic=false instantiation."""
    m = small_bar(3, 3, 12, material=mesh.steel_elastic(), v_end=1e4, n_steps=600)
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    with Solver(m) as sv:
        sv.set_tuning("elem_exact", 1)
        sv.set_tuning("elem_pipe_min", 0)
        sv.step(1, m.n_steps)
        g = sv.download()
    _assert_state_bitexact(g, o.s)
