"""Graph mode of hakai_step (an even number of steps per captured hipGraph, step number from a device counter):
bit-identical to stream mode on decks with BC amplitudes, deletion and contact, across call
boundaries, parity changes, a d_time change and state uploads, and actually used."""
import numpy as np
import pytest

from hakai import mesh
from hakai.solver import Solver
from util import fast_deletion_bar

pytestmark = pytest.mark.gpu

KEYS = ("disp", "disp_pre", "integ_stress", "integ_strain", "integ_eq_plastic_strain", "integ_yield_stress",
        "integ_triax_stress", "element_flag", "Q")


def run(m, chunks, graph, dts=None, upload_at=None):
    with Solver(m, device=0) as sv:
        sv.set_tuning("graph", graph)
        t = 1
        for i, n in enumerate(chunks):
            if upload_at is not None and i == upload_at:
                sv.upload(sv.download())  # a state upload invalidates captured graphs
            sv.step(t, n, None if dts is None else dts[i])
            t += n
        st = sv.download()
        return st, sv.deleted(), sv.graph_steps()


def same(a, b):
    for k in KEYS:
        x, y = getattr(a[0], k), getattr(b[0], k)
        if x is None and y is None:
            continue
        assert np.array_equal(x, y), k
    assert np.array_equal(a[1], b[1])


@pytest.mark.parametrize("per", [2, 16])
def test_graph_tensile5e_bitexact(per):
    """Tensile5e: amplitude BC, plasticity, the element-3 deletion at step 15 153."""
    m = mesh.tensile5e_model()
    chunks = [1, 2, 3, 7, 100, 5000, 10037, m.n_steps - 15150]
    g = run(m, chunks, per)
    s = run(m, chunks, 0)
    same(g, s)
    assert s[2] == 0 and g[2] > 0.9 * m.n_steps
    assert g[1].shape[0] >= 1  # the deletion happened inside a graph-mode chunk


@pytest.mark.parametrize("per", [2, 16])
def test_graph_deletion_bar_dt_change_and_upload(per):
    m = fast_deletion_bar()
    chunks = [5, 300, 1, 1400, 1294]
    dts = [m.dt, m.dt, m.dt * 0.5, m.dt * 0.5, m.dt]
    g = run(m, chunks, per, dts=dts, upload_at=3)
    s = run(m, chunks, 0, dts=dts, upload_at=3)
    same(g, s)
    assert g[2] > 2500 and s[2] == 0


@pytest.mark.parametrize("flag,per", [(1, 16), (2, 2)])
def test_graph_contact_with_deletion_bitexact(flag, per):
    """Two bodies with contact (and self-contact) and deletions: incremental surface updates run
    inside graphs; a non-consecutive t forces a stream-mode rebuild step."""
    m = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400,
                            contact_flag=flag)
    chunks = [3, 150, 2, 245]
    g = run(m, chunks, per)
    s = run(m, chunks, 0)
    same(g, s)
    assert g[2] > 300 and len(s[1]) > 0
    # non-consecutive restart: the rebuild step runs in stream mode, the rest from graphs
    with Solver(m, device=0) as sv1, Solver(m, device=0) as sv2:
        sv1.set_tuning("graph", per)
        sv2.set_tuning("graph", 0)
        for sv in (sv1, sv2):
            sv.step(1, 100)
            sv.step(150, 100)
        a, b = sv1.download(), sv2.download()
        for k in ("disp", "integ_stress", "element_flag"):
            assert np.array_equal(getattr(a, k), getattr(b, k)), k
        assert sv1.graph_steps() > 150


def test_graph_settings(monkeypatch):
    """Odd step counts are refused; HAKAI_GRAPH sets the default of new contexts; profiling events
    keep the loop in stream mode."""
    import hakai
    m = mesh.tensile5e_model()
    with Solver(m, device=0) as sv:
        with pytest.raises(hakai.HakaiError):
            sv.set_tuning("graph", 3)
        sv.step(1, 100)
        assert sv.graph_steps() > 0  # default on
        n0 = sv.graph_steps()
        sv.profile(True)
        sv.step(101, 100)
        sv.profile(False)
        assert sv.graph_steps() == n0
    monkeypatch.setenv("HAKAI_GRAPH", "0")
    with Solver(m, device=0) as sv:
        sv.step(1, 100)
        assert sv.graph_steps() == 0
    monkeypatch.setenv("HAKAI_GRAPH", "4")
    with Solver(m, device=0) as sv:
        sv.step(1, 100)
        # 24 graphs of 4 steps, one 2-step tail graph, then the call's last 2 steps in stream mode
        assert sv.graph_steps() == 98
