"""BASELINE configurations C2, C4 and C5 under GPU checks (C3 and C1: test_gpu_fullsize.py,
test_gpu_parity.py / test_gpu_exact.py).

* C2 (1 M-hex elastic bar, bench kernel k_element_pipe<ANY_PLASTIC=false>): the persistent elastic
  kernel on a small bar against the oracle; at full size, every element's nodal forces balance and a
  3-step window handed to the oracle agrees (fused kernel <= 1e-9; reference-order kernel bit for bit).
* C4 (4 M-hex two-body impact with contact, frictionless): a mid-size two-body model whose hash grid
  has more than 32 768 buckets (the device-wide hipcub scan, not the one-block scan) against the
  literal oracle over a whole run with contact; at full size, the GPU runs into the impact (events
  and element deletions every step), hands its state to the oracle (indexed contact mode -- the
  literal O(F^2) setup cannot run at 24 M faces) and both run a window: same contact force at the
  hand-off, same deletions, displacement within 1e-6 (fused) and bit for bit (reference order);
  incremental live lists bit-identical to a full rebuild at that size.
* C5 (16 M hex over 8 ranks): the 8-rank in-process group (same partition, pack / fix kernels and
  exchange protocol as the RCCL path) at 100x100x1600 is bit-identical to one 16 M context.
Reference: v2/HAKAI_j.jl:487-764 (step body), :2248-2706 (contact).
"""
import os

import numpy as np
import pytest

from hakai import dist, mesh
from hakai.solver import Solver, State, step_group
from util import rel_err, small_bar

pytestmark = pytest.mark.gpu

STATE_KEYS = ("disp", "disp_pre", "velo", "Q", "Qe", "integ_stress", "integ_strain", "integ_yield_stress",
              "integ_eq_plastic_strain", "integ_triax_stress", "element_flag")


def _threads():
    return int(os.environ.get("OMP_NUM_THREADS", "8"))


def _to_oracle(o, g, m):
    s = o.s
    for k in STATE_KEYS:
        s[k][...] = getattr(g, k)
    s["position"][...] = m.coordmat + g.disp.reshape(-1, 3)


def _window(m, g, t0, n, o_kwargs=None, probe=False):
    """Oracle from GPU state g (after step t0-1); runs steps t0..t0+n-1. Returns the oracle (and
    its contact force at the hand-off if probe)."""
    import oracle as O
    o = O.Oracle(m, nthreads=_threads(), **(o_kwargs or {}))
    _to_oracle(o, g, m)
    f = o.contact_force() if probe else None
    o.run(t0, n)
    return o, f


def _assert_bitexact(g, s, keys=("disp", "disp_pre", "integ_stress", "integ_strain", "integ_eq_plastic_strain",
                                 "integ_yield_stress", "element_flag", "Q")):
    for k in keys:
        a, b = getattr(g, k), s[k]
        assert np.array_equal(a, b), f"{k}: max rel diff {rel_err(a, b):.3e}"


# ---- C2 ----------------------------------------------------------------------------------------
def test_c2_persistent_elastic_kernel_vs_oracle():
    """The bench's C2 kernel (persistent, pipelined, ANY_PLASTIC=false) on a 640-hex elastic bar."""
    import oracle as O
    m = small_bar(4, 4, 40, material=mesh.steel_elastic(), v_end=1e4, n_steps=400)
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    with Solver(m) as sv:
        sv.set_tuning("elem_pipe_min", 0)   # persistent kernel even on this small mesh (20 batches)
        sv.step(1, 200)
        sv.step(201, m.n_steps - 200)
        g = sv.download()
    assert rel_err(g.disp, o.s["disp"]) < 1e-9
    assert rel_err(g.integ_stress, o.s["integ_stress"]) < 1e-8
    assert not np.any(g.integ_eq_plastic_strain)


@pytest.mark.timeout(600)
def test_c2_fullsize_window_vs_oracle():
    m = mesh.config_c2()
    t0, n = 51, 3
    with Solver(m) as sv:
        sv.step(1, t0 - 1)
        g = sv.download()
        o, _ = _window(m, g, t0, n)
        # fused kernel (the bench's)
        sv.step(t0, n)
        gf = sv.download()
        assert rel_err(gf.disp, o.s["disp"]) < 1e-9
        assert rel_err(gf.integ_stress, o.s["integ_stress"]) < 1e-9
        # every element's nodal forces balance (sum_i dN_i/dx = 0)
        fe = gf.Qe.reshape(m.nElement, 8, 3)
        scale = np.max(np.abs(fe), axis=(1, 2))
        assert np.all(scale > 0)
        assert np.max(np.abs(fe.sum(axis=1)).max(axis=1) / scale) < 1e-11
        del fe, gf
        # reference-order kernel from the same hand-off state: the oracle's bits
        sv.upload(g)
        sv.set_tuning("elem_exact", 1)
        sv.step(t0, n)
        ge = sv.download()
    _assert_bitexact(ge, o.s)


# ---- C4 ----------------------------------------------------------------------------------------
def test_c4_midsize_device_wide_scan_vs_oracle():
    """Two-body impact whose plate-side hash grid alone has 32 768 buckets: the contact step takes
    the device-wide hipcub scan. Whole run against the literal oracle: reference-order kernel bit for
    bit; fused kernel <= 1e-6 (nodes perturbed 2 %: an aligned mesh puts impactor nodes exactly on
    plate triangle edges, where contact decisions follow the last bit, as on the crash-tube deck)."""
    import oracle as O
    m = mesh.two_body_model(plate=(64, 64, 2), impactor=(8, 8, 6), v=-1e5, myu=0.0, perturb=0.02, seed=3,
                            n_steps=150)
    o = O.Oracle(m, nthreads=_threads())
    o.run(1, m.n_steps)
    runs = {}
    for exact in (1, 0):
        with Solver(m) as sv:
            sv.set_tuning("elem_exact", exact)
            sv.step(1, 60)
            st = sv.contact_stats()
            sv.step(61, m.n_steps - 60)
            runs[exact] = (sv.download(), st)
    assert runs[1][1]["hash_buckets"] > 32768
    assert runs[1][1]["events"] > 0
    _assert_bitexact(runs[1][0], o.s)
    g = runs[0][0]
    assert rel_err(g.disp, o.s["disp"]) < 1e-6
    assert rel_err(g.integ_stress, o.s["integ_stress"]) < 1e-6


@pytest.fixture(scope="module")
def c4_handoff():
    """C4 at full size, run into the impact: the first step D with an element deletion is found,
    the run is repeated from the start to step D-3 and that state is the hand-off (window D-2..D+1
    holds contact events and deletions)."""
    m = mesh.config_c4()
    sv = Solver(m)
    t = 1
    while not len(sv.deleted()) and t < 400:
        sv.step(t, 10)
        t += 10
    dels = sv.deleted()
    assert len(dels), "C4 must delete elements within 400 steps"
    D = int(dels[0][0])
    sv.reset()
    sv.step(1, D - 3)
    g = sv.download()
    yield m, sv, g, D - 2
    sv.close()


@pytest.mark.timeout(900)
def test_c4_fullsize_contact_window_vs_oracle(c4_handoff):
    m, sv, g, t0 = c4_handoff
    n = 4
    o, (fo, nev) = _window(m, g, t0, n, dict(contact_indexed=True), probe=True)
    assert nev > 0, "the hand-off state must be in contact"
    odels = sorted(tuple(int(v) for v in d) for d in o.deletions)
    assert len(odels) > 0, "the window must hold element deletions"
    # contact force at the hand-off state: bit for bit
    sv.upload(g)
    assert np.array_equal(sv.contact_force(t0), fo)
    # reference-order kernel window: the oracle's bits (the GPU log of an uploaded state holds the
    # window's deletions only)
    sv.upload(g)
    sv.set_tuning("elem_exact", 1)
    sv.step(t0, n)
    assert [tuple(int(v) for v in x) for x in sv.deleted()] == odels
    ge = sv.download()
    sv.set_tuning("elem_exact", 0)
    _assert_bitexact(ge, o.s)
    del ge
    # fused kernel window (the bench's kernel): rounding-level element differences
    sv.upload(g)
    sv.step(t0, n)
    gf = sv.download()
    assert [tuple(int(v) for v in x) for x in sv.deleted()] == odels
    assert np.array_equal(gf.element_flag, o.s["element_flag"])
    assert rel_err(gf.disp, o.s["disp"]) < 1e-6
    assert rel_err(gf.integ_stress, o.s["integ_stress"]) < 1e-6


@pytest.mark.timeout(600)
def test_c4_fullsize_incremental_lists_equal_full_rebuild(c4_handoff):
    m, sv, g, t0 = c4_handoff
    out = []
    for full in (0, 1):
        sv.upload(g)
        sv.set_tuning("contact_full_rebuild", full)
        sv.step(t0, 8)
        st = sv.contact_stats()
        out.append((sv.download(disp=True, integ_stress=True, element_flag=True), st))
    sv.set_tuning("contact_full_rebuild", 0)
    (a, sa), (b, sb) = out
    assert np.array_equal(a.disp, b.disp) and np.array_equal(a.integ_stress, b.integ_stress)
    assert np.array_equal(a.element_flag, b.element_flag)
    for k in ("events", "live_triangles", "live_nodes_i", "live_nodes_j", "hash_buckets"):
        assert sa[k] == sb[k], k
    assert sa["hash_buckets"] > 32768


# ---- C5 ----------------------------------------------------------------------------------------
@pytest.mark.timeout(900)
def test_c5_eight_ranks_fullsize_bitexact():
    """C5 at its BASELINE shape: 100x100x1600 (16 M hex) in 8 z-slabs of 2 M, as an in-process
    group, against one 16 M context, 30 steps (the impact front has entered every slab's
    neighbourhood of the clamped face only near rank 0; every rank exchanges interface forces)."""
    world, layers, n_steps = 8, 1600, 30
    glob = mesh.config_c5(layers=layers)
    with Solver(glob) as sv:
        sv.step(1, n_steps)
        g = sv.download(disp=True, disp_pre=True, element_flag=True, integ_eq_plastic_strain=True)
    assert np.any(g.disp != 0) and np.any(g.integ_eq_plastic_strain > 0)
    svs, parts = [], []
    try:
        for r in range(world):
            loc, diag, iface = dist.slab_partition(glob, r, world, nx=100, ny=100)
            sv = Solver(loc, diag_M=diag)
            sv.set_element_offset(loc.global_element_offset)
            sv.comm_init_local(r, world, 8161)
            sv.set_interface(*iface)
            svs.append(sv)
            parts.append(loc)
        step_group(svs, 1, n_steps)
        for sv, loc in zip(svs, parts):
            st = sv.download(disp=True, disp_pre=True, element_flag=True, integ_eq_plastic_strain=True)
            n0, nl = loc.global_node_offset, loc.nNode
            e0, el = loc.global_element_offset, loc.nElement
            assert np.array_equal(st.disp, g.disp[3 * n0:3 * (n0 + nl)])
            assert np.array_equal(st.disp_pre, g.disp_pre[3 * n0:3 * (n0 + nl)])
            assert np.array_equal(st.element_flag, g.element_flag[e0:e0 + el])
            assert np.array_equal(st.integ_eq_plastic_strain, g.integ_eq_plastic_strain[8 * e0:8 * (e0 + el)])
    finally:
        for sv in svs:
            sv.close()
