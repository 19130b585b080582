"""Two-step chunked schedule (tuning key "tblock_mb", hakai_step on one GPU without contact).

Steps s and s+1 run interleaved chunk by chunk (element chunk of step s, then the nodes of step
s+1 whose incident elements are done, then the elements of step s+1 whose nodes are done), so step
s+1 finds its Gauss-point state, element forces and node rows in the Infinity Cache. It is a
reordering of the same computations (v2/HAKAI_j.jl:497-764, each node's Q still summed in element
order, :668-675), so every test demands BIT-identical state against the plain step loop, and the
Tensile5e case against the oracle as well. Meshes with shuffled element and node numbering check
that the schedule's hazard analysis holds for any numbering (it then degenerates, never breaks).
"""
import numpy as np
import pytest

from hakai import mesh
from hakai.model import BCGroup, Model
from hakai.solver import Solver
import oracle as O
from util import fast_deletion_bar, rel_err, small_bar

pytestmark = pytest.mark.gpu

STATE = ("disp", "disp_pre", "integ_stress", "integ_strain", "integ_yield_stress", "integ_eq_plastic_strain",
         "element_flag", "Q", "Qe")
K_ELEMENT = 0


def _same(a, b):
    for k in STATE:
        x, y = getattr(a, k), getattr(b, k)
        assert np.array_equal(x, y), f"{k}: max rel diff {rel_err(x, y):.3e}"
    assert np.array_equal(a.integ_triax_stress, b.integ_triax_stress)


def _run(m, calls, tune, tblock):
    """Run the model through the given (t_first, n) calls; returns (state, deletions, element launches)."""
    with Solver(m) as sv:
        for k, v in tune.items():
            sv.set_tuning(k, v)
        sv.set_tuning("tblock_mb", tblock)
        sv.profile(True, [K_ELEMENT])
        for t0, n in calls:
            sv.step(t0, n)
        g = sv.download()
        dels = [tuple(x) for x in sv.deleted()]
        _, launches = sv.profile_read(K_ELEMENT)
    return g, dels, launches


def _shuffled(m: Model, seed: int) -> Model:
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


@pytest.mark.parametrize("exact", [0, 1])
def test_tblock_deletion_bar_bitexact(exact):
    """Deleting bar (6 400 hex, amplitude BC on the pulled face), ~1 MB chunks: the pair schedule
    equals the plain loop bit for bit, incl. the deletion log; odd step counts and several calls."""
    m = fast_deletion_bar(4, 4, 400)
    calls = [(1, 301), (302, 1000), (1302, 1699)]
    tune = {"elem_exact": exact}
    g0, d0, n0 = _run(m, calls, tune, 0)
    g1, d1, n1 = _run(m, calls, tune, 1)
    assert n0 == 3000 and n1 > 3000, (n0, n1)  # the chunked schedule ran (several launches per pair)
    assert len(d0) > 0
    assert d1 == d0
    _same(g1, g0)


@pytest.mark.parametrize("pipe_min", [0, 2])
def test_tblock_elastoplastic_bar_chunks(pipe_min):
    """Plastic bar, persistent (pipe_min 0) and one-batch element kernels, several chunk sizes."""
    m = small_bar(6, 5, 300, n_steps=600, v_end=5e5)
    ref, _, _ = _run(m, [(1, 600)], {"elem_pipe_min": pipe_min}, 0)
    assert np.any(ref.integ_eq_plastic_strain > 0)
    for mb in (1, 3, 64):
        g, _, _ = _run(m, [(1, 600)], {"elem_pipe_min": pipe_min}, mb)
        _same(g, ref)


def test_tblock_shuffled_numbering_bitexact():
    """Random element and node numbering: ranges degenerate, results stay bit-identical."""
    m = _shuffled(fast_deletion_bar(3, 3, 200), seed=7)
    ref, d0, _ = _run(m, [(1, 3000)], {}, 0)
    g, d1, n1 = _run(m, [(1, 3000)], {}, 1)
    assert n1 >= 3000
    assert d1 == d0 and len(d0) > 0
    _same(g, ref)


def test_tblock_tensile5e_vs_oracle():
    """Tensile5e.inp (amplitude BCs, one chunk): bit-identical to the oracle in reference order."""
    m = mesh.tensile5e_model()
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    g, dels, _ = _run(m, [(1, m.n_steps)], {"elem_exact": 1}, 1)
    assert dels == o.deletions == [(15153, 3)]
    for k in STATE:
        assert np.array_equal(getattr(g, k), o.s[k]), k


def test_tblock_upload_mid_run():
    """A state uploaded between calls (Q from the uploaded buffer: that step runs unpaired, the
    rest in pairs) matches the plain loop."""
    m = fast_deletion_bar(3, 3, 120)
    with Solver(m) as sv:
        sv.step(1, 500)
        mid = sv.download()
    outs = []
    for mb in (0, 1):
        with Solver(m) as sv:
            sv.set_tuning("tblock_mb", mb)
            sv.upload(mid)
            sv.step(501, 800)
            outs.append(sv.download())
    _same(outs[1], outs[0])
