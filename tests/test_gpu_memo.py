"""Prefilter memo (hakai_contact.hip TriMemo, tuning contact_filter_memo): the triangle prefilter
skips a triangle it rejected before while the contact nodes' accumulated motion (the box array's
motion word, summed into a per-step clock) cannot have carried it to its pair's range box. The
skip only drops triangles the full test would reject, so the candidates of every step, and the
whole run, must equal the memo-off run bit for bit -- with deletions (new triangles and dead
elements), self-contact, graphs, the fused small-deck path and state uploads that move the nodes
without the clock (they void every record). The memo must also actually skip (stat
tested_triangles)."""
import numpy as np
import pytest

from hakai import mesh
from hakai.solver import Solver

pytestmark = pytest.mark.gpu

KEYS = ("disp", "disp_pre", "velo", "integ_stress", "integ_eq_plastic_strain", "element_flag")


def _deck(flag=1):
    return mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400,
                               contact_flag=flag)


def _stepwise(m, memo):
    with Solver(m) as sv:
        sv.set_tuning("graph", 0)
        sv.set_tuning("contact_filter_memo", memo)
        per = []
        for t in range(1, m.n_steps + 1):
            sv.step(t, 1)
            st = sv.contact_stats()
            per.append((st["candidate_triangles"], st["events"], st["live_triangles"], st["tested_triangles"]))
        return sv.download(), [tuple(int(v) for v in x) for x in sv.deleted()], per


@pytest.mark.parametrize("flag", [1, 2])
def test_memo_same_candidates_every_step(flag):
    m = _deck(flag)
    a, da, pa = _stepwise(m, 0)
    b, db, pb = _stepwise(m, 1)
    assert da == db and len(da) > 0
    assert [p[:3] for p in pa] == [p[:3] for p in pb]  # candidates, events, live triangles
    assert all(q[3] <= p[3] <= p[2] for p, q in zip(pa, pb))  # (off: all with a non-empty range)
    tested_off, tested_on = sum(p[3] for p in pa), sum(p[3] for p in pb)
    assert tested_on < 0.7 * tested_off, (tested_on, tested_off)
    for k in KEYS:
        assert np.array_equal(getattr(a, k), getattr(b, k)), k


@pytest.mark.parametrize("graph,fuse", [(16, 1), (16, 0), (0, 1)])
def test_memo_graphs_and_fused_path_bitexact(graph, fuse):
    m = _deck(2)
    out = []
    for memo in (0, 1):
        with Solver(m) as sv:
            sv.set_tuning("graph", graph)
            sv.set_tuning("contact_fuse_small", fuse)
            sv.set_tuning("contact_filter_memo", memo)
            sv.step(1, 250)
            sv.step(251, m.n_steps - 250)
            out.append((sv.download(), [tuple(int(v) for v in x) for x in sv.deleted()], sv.contact_stats()))
    (a, da, sa), (b, db, sb) = out
    assert da == db and len(da) > 0
    assert sa["max_events"] == sb["max_events"] and sa["candidate_triangles"] == sb["candidate_triangles"]
    for k in KEYS:
        assert np.array_equal(getattr(a, k), getattr(b, k)), k


def test_memo_upload_voids_records():
    """A state upload moves the nodes outside the clock: the records made before it must not be
    used after it."""
    m = _deck(1)
    out = []
    for memo in (0, 1):
        with Solver(m) as sv:
            sv.set_tuning("graph", 0)
            sv.set_tuning("contact_filter_memo", memo)
            sv.step(1, 150)
            st = sv.download()
            # the impactor (its 3x3x4 nodes come last) moved rigidly by a third of the plate in x
            # and y: records made before the upload would now be wrong by that much
            x = m.coordmat
            imp = np.arange(x.shape[0] - 36, x.shape[0])
            assert x[imp, 2].min() > x[:-36, 2].max()
            w = x[:-36, 0].max() - x[:-36, 0].min()
            sh = np.zeros_like(x)
            sh[imp, 0] = sh[imp, 1] = w / 3
            st.disp = st.disp + sh.reshape(-1)
            st.disp_pre = st.disp_pre + sh.reshape(-1)
            sv.upload(st)
            sv.step(151, m.n_steps - 150)
            out.append((sv.download(), [tuple(int(v) for v in x) for x in sv.deleted()]))
    (a, da), (b, db) = out
    assert da == db
    for k in KEYS:
        assert np.array_equal(getattr(a, k), getattr(b, k)), k


def test_memo_tuning_is_validated():
    from hakai._abi import HakaiError
    with Solver(_deck(1)) as sv:
        with pytest.raises(HakaiError):
            sv.set_tuning("contact_filter_memo", 2)


@pytest.mark.parametrize("fuse_small", [0, 1])
def test_binfilter_fusion_bitexact(fuse_small):
    """The binning and the prefilter in one launch (tuning contact_fuse_binfilter, default on) or in
    two: the same run bit for bit (large decks take this path; here the small-deck fusion is off)."""
    m = _deck(2)
    out = []
    for bf in (0, 1):
        with Solver(m) as sv:
            sv.set_tuning("contact_fuse_small", fuse_small)
            sv.set_tuning("contact_fuse_binfilter", bf)
            sv.step(1, m.n_steps)
            out.append((sv.download(), [tuple(int(v) for v in x) for x in sv.deleted()], sv.contact_stats()))
    (a, da, sa), (b, db, sb) = out
    assert da == db and len(da) > 0
    assert sa["candidate_triangles"] == sb["candidate_triangles"] and sa["events"] == sb["events"]
    for k in KEYS:
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
