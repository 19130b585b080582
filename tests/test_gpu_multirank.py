"""Multi-rank parity on one GPU: an in-process group of contexts (hakai_comm_init_local) runs the
same partition, pack / interface-sum / fix kernels and exchange protocol as the RCCL path
(hakai_comm.cpp), and must reproduce the single-context run BIT FOR BIT: the interface Q is summed
in the reference's serial element order (v2/HAKAI_j.jl:669-675) on both sides of every cut.
"""
import os

import numpy as np
import pytest

from hakai import dist
from hakai.solver import Solver, step_group
from util import fast_deletion_bar

pytestmark = pytest.mark.gpu


def _run_group(glob, world, n_steps, key):
    nx = ny = 2
    parts = [dist.slab_partition(glob, r, world, nx, ny) for r in range(world)]
    svs = []
    for r, (loc, diag, iface) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        sv.set_element_offset(loc.global_element_offset)
        sv.comm_init_local(r, world, key)
        sv.set_interface(*iface)
        svs.append(sv)
    step_group(svs, 1, n_steps)
    out = []
    for sv, (loc, _, _) in zip(svs, parts):
        out.append((loc, sv.download(), [tuple(x) for x in sv.deleted()]))
    for sv in svs:
        sv.close()
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_local_group_bitexact(world):
    glob = fast_deletion_bar(2, 2, 12)
    n = 1200
    with Solver(glob) as sv:
        sv.step(1, n)
        g = sv.download()
        gdel = [tuple(x) for x in sv.deleted()]
    assert len(gdel) > 0, "config must delete elements"
    parts = _run_group(glob, world, n, key=100 + world)
    dels = sorted(d for _, _, dl in parts for d in dl)
    assert dels == gdel
    for loc, st, _ in parts:
        n0, nl = loc.global_node_offset, loc.nNode
        e0, el = loc.global_element_offset, loc.nElement
        sl = slice(3 * n0, 3 * (n0 + nl))
        assert np.array_equal(st.disp, g.disp[sl])
        assert np.array_equal(st.disp_pre, g.disp_pre[sl])
        assert np.array_equal(st.velo, g.velo[sl])
        gp = slice(8 * e0, 8 * (e0 + el))
        assert np.array_equal(st.integ_stress, g.integ_stress[gp])
        assert np.array_equal(st.integ_eq_plastic_strain, g.integ_eq_plastic_strain[gp])
        assert np.array_equal(st.element_flag, g.element_flag[e0:e0 + el])
        assert np.array_equal(st.Qe, g.Qe[e0:e0 + el])


def test_local_group_rejects_multi_step_calls():
    glob = fast_deletion_bar(2, 2, 8)
    parts = [dist.slab_partition(glob, r, 2, 2, 2) for r in range(2)]
    svs = []
    for r, (loc, diag, iface) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        sv.comm_init_local(r, 2, 777)
        sv.set_interface(*iface)
        svs.append(sv)
    with pytest.raises(Exception):
        svs[0].step(1, 5)
    for sv in svs:
        sv.close()


def _run_contact_group(glob, world, n_steps, key, tune=None, refuse_at=0):
    """Range-partitioned contact model on an in-process group (hakai_set_contact_global): each rank
    searches the triangles of its elements against the binned contact nodes of every rank.
    refuse_at > 0: after that many steps, every rank is first asked to step ALONE (hakai_step), which
    must be refused before any work (HAKAI_ERR_STATE), then the group goes on."""
    gdiag, _ = glob.lumped_mass()
    parts = [dist.range_partition(glob, r, world, gdiag) for r in range(world)]
    svs = []
    for r, (loc, diag, iface, l2g, off) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        sv.set_element_offset(loc.global_element_offset)
        sv.comm_init_local(r, world, key)
        sv.set_interface(*iface)
        sv.set_contact_global(glob, l2g, off, gdiag)
        for k, v in (tune or {}).items():
            sv.set_tuning(k, v)
        svs.append(sv)
    if refuse_at:
        from hakai._abi import HAKAI_ERR_STATE, HakaiError
        step_group(svs, 1, refuse_at)
        for sv in svs:
            with pytest.raises(HakaiError) as ei:
                sv.step(refuse_at + 1, 1)
            assert ei.value.code == HAKAI_ERR_STATE
        step_group(svs, refuse_at + 1, n_steps - refuse_at)
    else:
        step_group(svs, 1, n_steps)
    if tune and tune.get("own_assembly"):
        assert all(sv.stat("own_steps") == n_steps for sv in svs)
    out = [(loc, l2g, sv.download(), [tuple(x) for x in sv.deleted()], sv.contact_stats())
           for sv, (loc, _, _, l2g, _) in zip(svs, parts)]
    for sv in svs:
        sv.close()
    return out


def _assert_group_equals_single(glob, parts, g, gdel):
    dels = sorted(d for _, _, _, dl, _ in parts for d in dl)
    assert dels == gdel
    for loc, l2g, st, _, _ in parts:
        n = l2g - 1
        assert np.array_equal(st.disp.reshape(-1, 3), g.disp.reshape(-1, 3)[n])
        assert np.array_equal(st.disp_pre.reshape(-1, 3), g.disp_pre.reshape(-1, 3)[n])
        e0, el = loc.global_element_offset, loc.nElement
        gp = slice(8 * e0, 8 * (e0 + el))
        assert np.array_equal(st.integ_stress, g.integ_stress[gp])
        assert np.array_equal(st.integ_eq_plastic_strain, g.integ_eq_plastic_strain[gp])
        assert np.array_equal(st.element_flag, g.element_flag[e0:e0 + el])


@pytest.mark.parametrize("world", [2, 4])
def test_contact_group_x_slabs_bitexact(world):
    """The same with the elements numbered x slowest (mesh x_slabs), so the rank ranges are
    x-slabs and every rank holds part of both contact surfaces (the z-slab ranges above put each
    surface on one rank): bit-identical to one context, and the candidate triangles spread over
    the ranks."""
    from hakai import mesh
    glob = mesh.two_body_model(plate=(8, 8, 2), impactor=(4, 4, 3), v=-3e5, d_time=2e-8, n_steps=400, x_slabs=True)
    with Solver(glob) as sv:
        sv.step(1, glob.n_steps)
        g = sv.download()
        gdel = [tuple(x) for x in sv.deleted()]
        gst = sv.contact_stats()
    parts = _run_contact_group(glob, world, glob.n_steps, key=350 + world)
    _assert_group_equals_single(glob, parts, g, gdel)
    sts = [st for *_, st in parts]
    assert sum(st["candidate_triangles"] for st in sts) == gst["candidate_triangles"]
    assert sum(1 for st in sts if st["live_triangles"] > 0) == world  # every rank holds surface


@pytest.mark.parametrize("world,deck", [(2, "x_slabs"), (3, "deletion")])
def test_contact_group_unfused_insert_bitexact(world, deck):
    """The A3 bucket insert and the triangle prefilter in two launches (contact_fuse_binfilter 0)
    instead of one (k_xr_insfilter): bit-identical to one context, the same candidate triangles."""
    from hakai import mesh
    if deck == "x_slabs":
        glob = mesh.two_body_model(plate=(8, 8, 2), impactor=(4, 4, 3), v=-3e5, d_time=2e-8, n_steps=400,
                                   x_slabs=True)
    else:
        glob = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400)
    with Solver(glob) as sv:
        sv.step(1, glob.n_steps)
        g = sv.download()
        gdel = [tuple(x) for x in sv.deleted()]
        gst = sv.contact_stats()
    parts = _run_contact_group(glob, world, glob.n_steps, key=380 + world, tune={"contact_fuse_binfilter": 0})
    _assert_group_equals_single(glob, parts, g, gdel)
    sts = [st for *_, st in parts]
    assert sum(st["candidate_triangles"] for st in sts) == gst["candidate_triangles"]
    assert sum(st["tested_triangles"] for st in sts) <= sum(st["live_triangles"] for st in sts)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_contact_group_bitexact_with_deletion(world):
    """Multi-GPU contact: contact-driven deletion with the surface update, the
    impactor and the plate split over ranks; every rank's displacements, stresses and the deletion
    log equal the single-context run bit for bit. Each rank keeps the triangles of its own elements
    and the contact nodes it owns: the live lists and the candidate triangles divide over the ranks,
    the events are all-gathered and every rank forms the same order-independent sums."""
    from hakai import mesh
    glob = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400)
    with Solver(glob) as sv:
        sv.step(1, glob.n_steps)
        g = sv.download()
        gdel = [tuple(x) for x in sv.deleted()]
        gst = sv.contact_stats()
    assert len(gdel) >= 4
    parts = _run_contact_group(glob, world, glob.n_steps, key=300 + world)
    _assert_group_equals_single(glob, parts, g, gdel)
    sts = [st for *_, st in parts]
    assert all(st["events"] == gst["events"] for st in sts)  # every rank sums every event
    for k in ("live_triangles", "live_nodes_i", "live_nodes_j", "candidate_triangles"):
        assert sum(st[k] for st in sts) == gst[k], k  # the lists and the search divide
    assert sum(st["candidate_triangles"] > 0 for st in sts) >= 2


def test_contact_group_rank_cannot_step_alone():
    """hakai_step on one contact rank of an in-process group is refused BEFORE any work
    (no tsel flip, no prologue kernels), so a later hakai_step_group still matches one context bit
    for bit."""
    from hakai import mesh
    glob = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400)
    with Solver(glob) as sv:
        sv.step(1, glob.n_steps)
        g = sv.download()
        gdel = [tuple(x) for x in sv.deleted()]
    assert len(gdel) >= 4
    parts = _run_contact_group(glob, 2, glob.n_steps, key=333, refuse_at=151)
    _assert_group_equals_single(glob, parts, g, gdel)


@pytest.mark.parametrize("flag,myu,surfaces", [(1, None, False), (2, 0.0, False), (1, None, True)])
def test_contact_group_bitexact_variants(flag, myu, surfaces):
    """Friction (reference myu 0.25), self-contact, *Contact Pair surfaces on 2 ranks."""
    from hakai import mesh
    glob = mesh.two_body_model(plate=(6, 6, 2), impactor=(3, 3, 3), v=-1e5, perturb=0.02, seed=1, myu=myu,
                               contact_flag=flag, surfaces=surfaces, n_steps=300)
    with Solver(glob) as sv:
        sv.step(1, glob.n_steps)
        g = sv.download()
        gdel = [tuple(x) for x in sv.deleted()]
    parts = _run_contact_group(glob, 2, glob.n_steps, key=400 + 10 * flag + int(surfaces))
    _assert_group_equals_single(glob, parts, g, gdel)
    assert np.max(np.abs(g.disp)) > 0


def test_contact_on_communicator_requires_global_model():
    from hakai import mesh
    from hakai._abi import HakaiError, ptr
    glob = mesh.two_body_model(plate=(4, 4, 1), impactor=(2, 2, 2))
    loc, diag, iface, l2g, off = dist.range_partition(glob, 0, 2)
    with Solver(loc, diag_M=diag) as sv:
        sv.comm_init_local(0, 2, 999)
        inst = np.ones(loc.nElement, np.int64)
        with pytest.raises(HakaiError):
            from hakai._abi import check
            import ctypes
            check(sv.L.hakai_set_contact(sv.ctx, 1, ptr(inst, ctypes.c_int64)))


@pytest.mark.parametrize("caps", [1, 3])
def test_contact_group_exchange_capacities_grow(caps):
    """Every exchange block (deletions, binned contact nodes, events) starting at `caps` records per
    rank: a step that overflows one is poisoned on every rank, the capacity grows from the counts
    every rank gathered, and the step runs again -- the run is bit-identical to one context, and
    the capacities end larger than they started."""
    from hakai import mesh
    glob = mesh.two_body_model(plate=(16, 16, 8), impactor=(4, 4, 4), v=-3e5, d_time=2e-8, n_steps=300)
    with Solver(glob) as sv:
        sv.step(1, glob.n_steps)
        g = sv.download()
        gdel = [tuple(x) for x in sv.deleted()]
    assert len(gdel) > 0
    tune = {"contact_exchange_deletions": caps, "contact_exchange_bins": caps, "contact_exchange_events": caps}
    gdiag, _ = glob.lumped_mass()
    parts = [dist.range_partition(glob, r, 2, gdiag) for r in range(2)]
    svs = []
    for r, (loc, diag, iface, l2g, off) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        sv.set_element_offset(loc.global_element_offset)
        sv.comm_init_local(r, 2, 8080 + caps)
        sv.set_interface(*iface)
        sv.set_contact_global(glob, l2g, off, gdiag)
        for k, v in tune.items():
            sv.set_tuning(k, v)
        svs.append(sv)
    b0 = svs[0].contact_stats()["exchange_bytes_per_rank"]
    step_group(svs, 1, glob.n_steps)
    st0 = svs[0].contact_stats()
    assert st0["exchange_bytes_per_rank"] > b0 and st0["binned_contact_nodes"] > caps
    dels = []
    for sv, (loc, _, _, l2g, _) in zip(svs, parts):
        st = sv.download()
        dels += [tuple(x) for x in sv.deleted()]
        assert np.array_equal(st.disp.reshape(-1, 3), g.disp.reshape(-1, 3)[l2g - 1])
        sv.close()
    assert sorted(dels) == gdel


@pytest.mark.parametrize("chunk", [1, 300])
def test_contact_group_deletion_exchange_overflow_retry_bitexact(chunk):
    """The deletion block at its smallest capacity (1 record, capacities follow the counts from there
    and shrink back after the burst): a deletion burst overflows it, the next step is poisoned on
    every rank and runs again -- here at an even step, whose retry packs the interface sums into the
    parity the rerun's peers must not read (the rolled-back exchange parity, hakai_comm.cpp
    comm_rollback). Bit-identical to one context, one step per call and one call."""
    from hakai import mesh
    glob = mesh.two_body_model(plate=(16, 16, 8), impactor=(4, 4, 4), v=-3e5, d_time=2e-8, n_steps=300)
    with Solver(glob) as sv:
        sv.step(1, glob.n_steps)
        g = sv.download()
    gdiag, _ = glob.lumped_mass()
    parts = [dist.range_partition(glob, r, 2, gdiag) for r in range(2)]
    svs = []
    for r, (loc, diag, iface, l2g, off) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        sv.set_element_offset(loc.global_element_offset)
        sv.comm_init_local(r, 2, 8180 + chunk)
        sv.set_interface(*iface)
        sv.set_contact_global(glob, l2g, off, gdiag)
        sv.set_tuning("contact_exchange_deletions", 1)
        svs.append(sv)
    for t in range(1, glob.n_steps + 1, chunk):
        step_group(svs, t, min(chunk, glob.n_steps + 1 - t))
    assert min(sv.stat("exchange_retries") for sv in svs) >= 1
    for sv, (loc, _, _, l2g, _) in zip(svs, parts):
        st = sv.download()
        assert np.array_equal(st.disp.reshape(-1, 3), g.disp.reshape(-1, 3)[l2g - 1])
        sv.close()


@pytest.mark.parametrize("ranks", [2, 3])
def test_multi_gpu_driver_writes_the_same_vtk(tmp_path, ranks):
    """HAKAI(fname) over ranks (hakai.run.hakai_multi, here as an in-process group): contact with
    deletion, 101 VTK files byte-identical to the one-GPU driver's."""
    import hakai
    from hakai import mesh
    from hakai.run import hakai_multi
    from inp_writer import write_inp
    m = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400)
    deck = write_inp(str(tmp_path / "impact.inp"), m)
    hakai.hakai(deck, str(tmp_path / "one"), verbose=False)
    hakai_multi(deck, str(tmp_path / "multi"), local_ranks=ranks, verbose=False)
    files = sorted(os.listdir(tmp_path / "one"))
    assert len(files) == 101 and sorted(os.listdir(tmp_path / "multi")) == files
    for f in files:
        assert (tmp_path / "one" / f).read_bytes() == (tmp_path / "multi" / f).read_bytes(), f


def test_contact_group_after_state_upload():
    """hakai_upload_state on every rank (a mid-run state with deleted elements, restricted to each
    rank's nodes and elements) starts the exchange afresh: the next steps equal a single context
    that uploaded the same state, bit for bit."""
    from hakai import mesh
    from hakai.solver import State
    glob = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400)
    with Solver(glob) as sv:
        sv.step(1, 250)
        S = sv.download()
    assert np.count_nonzero(S.element_flag == 0) > 0
    with Solver(glob) as sv:
        sv.upload(S)
        sv.step(251, 150)
        g = sv.download()
    gdiag, _ = glob.lumped_mass()
    parts = [dist.range_partition(glob, r, 2, gdiag) for r in range(2)]
    svs = []
    for r, (loc, diag, iface, l2g, off) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        sv.set_element_offset(loc.global_element_offset)
        sv.comm_init_local(r, 2, 7070)
        sv.set_interface(*iface)
        sv.set_contact_global(glob, l2g, off, gdiag)
        n = l2g - 1
        e0, ne = loc.global_element_offset, loc.nElement
        nd = lambda a: np.ascontiguousarray(a.reshape(-1, 3)[n].ravel())  # noqa: E731
        gp = slice(8 * e0, 8 * (e0 + ne))
        sv.upload(State(nd(S.disp), nd(S.disp_pre), nd(S.velo), nd(S.Q), S.integ_stress[gp].copy(),
                        S.integ_strain[gp].copy(), S.integ_yield_stress[gp].copy(),
                        S.integ_eq_plastic_strain[gp].copy(), S.integ_triax_stress[gp].copy(),
                        S.element_flag[e0:e0 + ne].copy(), S.Qe[e0:e0 + ne].copy()))
        svs.append(sv)
    step_group(svs, 251, 150)
    for sv, (loc, _, _, l2g, _) in zip(svs, parts):
        st = sv.download()
        assert np.array_equal(st.disp.reshape(-1, 3), g.disp.reshape(-1, 3)[l2g - 1])
        e0 = loc.global_element_offset
        assert np.array_equal(st.element_flag, g.element_flag[e0:e0 + loc.nElement])
        sv.close()


def test_contact_group_window_vs_oracle():
    """A multi-rank run handed to the oracle: a 3-rank contact group (reference-order
    element arithmetic) runs past the first contact deletions; its ranks' states are assembled
    into the global state, the oracle takes over (surfaces updated for the deletions so far) and
    both run the next steps -- every rank's state equals the oracle's bit for bit."""
    from hakai import mesh
    import oracle as O
    glob = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400)
    gdiag, _ = glob.lumped_mass()
    world, t0, k = 3, 260, 60
    parts = [dist.range_partition(glob, r, world, gdiag) for r in range(world)]
    svs = []
    for r, (loc, diag, iface, l2g, off) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        sv.set_tuning("elem_exact", 1)
        sv.set_element_offset(loc.global_element_offset)
        sv.comm_init_local(r, world, 9090)
        sv.set_interface(*iface)
        sv.set_contact_global(glob, l2g, off, gdiag)
        svs.append(sv)
    step_group(svs, 1, t0)
    o = O.Oracle(glob)
    s = o.s
    dels = []
    for sv, (loc, _, _, l2g, _) in zip(svs, parts):
        st = sv.download()
        n = l2g - 1
        for key in ("disp", "disp_pre", "velo"):
            s[key].reshape(-1, 3)[n] = getattr(st, key).reshape(-1, 3)
        e0, ne = loc.global_element_offset, loc.nElement
        gp = slice(8 * e0, 8 * (e0 + ne))
        for key in ("integ_stress", "integ_strain"):
            s[key][gp] = getattr(st, key).reshape(-1, 6)
        for key in ("integ_yield_stress", "integ_eq_plastic_strain", "integ_triax_stress"):
            s[key][gp] = getattr(st, key)
        s["element_flag"][e0:e0 + ne] = st.element_flag
        s["Qe"][e0:e0 + ne] = st.Qe.reshape(-1, 24)
        dels += [tuple(int(v) for v in x) for x in sv.deleted()]
    dels.sort()
    # Q of the last step: the serial element-order assembly (v2/HAKAI_j.jl:668-675) of the ranks' Qe
    # (a rank's own Q of an interface node is completed only by the next step's exchange)
    idx = (3 * (glob.elementmat - 1)[:, :, None] + np.arange(3)[None, None, :]).ravel()
    s["Q"][...] = 0.0
    np.add.at(s["Q"], idx, s["Qe"].ravel())
    assert len(dels) > 0, "window must start after contact deletions"
    s["position"][...] = glob.coordmat + s["disp"].reshape(-1, 3)
    o.apply_deletions([e for _, e in dels])
    o.run(t0 + 1, k)
    step_group(svs, t0 + 1, k)
    new = []
    for sv, (loc, _, _, l2g, _) in zip(svs, parts):
        st = sv.download()
        n = l2g - 1
        assert np.array_equal(st.disp.reshape(-1, 3), s["disp"].reshape(-1, 3)[n])
        assert np.array_equal(st.velo.reshape(-1, 3), s["velo"].reshape(-1, 3)[n])
        e0, ne = loc.global_element_offset, loc.nElement
        assert np.array_equal(st.integ_stress.reshape(-1, 6), s["integ_stress"][8 * e0:8 * (e0 + ne)])
        assert np.array_equal(st.element_flag, s["element_flag"][e0:e0 + ne])
        new += [tuple(int(v) for v in x) for x in sv.deleted() if x[0] > t0]
        sv.close()
    assert sorted(new) == sorted(tuple(int(v) for v in x) for x in o.deletions)


def test_contact_overflow_poisons_every_rank():
    """An event-buffer overflow on any rank of a contact group is seen by every rank in the
    exchanged counts: the same step is poisoned on all of them (device-side, no host round trip),
    every rank's call fails, and every rank's state is the last good step's."""
    from hakai import mesh
    from hakai._abi import HakaiError
    glob = mesh.two_body_model(plate=(12, 12, 1), impactor=(8, 8, 1), v=-1e5, perturb=0.03, seed=4, n_steps=60)
    gdiag, _ = glob.lumped_mass()

    def group(cap, key):
        parts = [dist.range_partition(glob, r, 2, gdiag) for r in range(2)]
        svs = []
        for r, (loc, diag, iface, l2g, off) in enumerate(parts):
            sv = Solver(loc, diag_M=diag)
            sv.set_element_offset(loc.global_element_offset)
            sv.comm_init_local(r, 2, key)
            sv.set_interface(*iface)
            sv.set_contact_global(glob, l2g, off, gdiag)
            sv.set_tuning("contact_event_cap", cap)
            svs.append(sv)
        return parts, svs

    parts, svs = group(1, 9191)
    with pytest.raises(HakaiError) as ei:
        step_group(svs, 1, glob.n_steps)
    import re
    p = int(re.search(r"step (\d+) was not applied", str(ei.value)).group(1))
    assert 1 < p < glob.n_steps
    # (triaxiality and Qe are stored on a call's last step, which the overflow skipped)
    after = [sv.download(disp=True, velo=True, integ_stress=True) for sv in svs]
    for sv in svs:
        sv.close()
    _, good_svs = group(1 << 12, 9192)
    step_group(good_svs, 1, p - 1)
    for a, sv in zip(after, good_svs):
        g = sv.download()
        assert np.array_equal(a.disp, g.disp) and np.array_equal(a.velo, g.velo)
        assert np.array_equal(a.integ_stress, g.integ_stress)
        sv.close()


@pytest.mark.parametrize("world", [2, 3])
def test_local_group_owner_assembly_bitexact(world):
    """Owner-computed assembly on ranks with a communicator (the persistent kernel forced with
    elem_pipe_min 0, several blocks per rank): the lower side's partial sum is its local Q
    (own_q + rows) and the upper side's single contributions are exported rows (hakai_comm.cpp
    k_pack_own / k_fix_own). Every rank equals one context -- with and without the mode -- bit for bit."""
    glob = fast_deletion_bar(4, 4, 120)
    n = 1500
    tune = {"elem_pipe_min": 0, "elem_pipe_blocks": 6}
    ref = {}
    for own in (0, 1):
        with Solver(glob) as sv:
            for k, v in tune.items():
                sv.set_tuning(k, v)
            sv.set_tuning("own_assembly", own)
            sv.step(1, n)
            ref[own] = (sv.download(), [tuple(x) for x in sv.deleted()])
    g, gdel = ref[1]
    assert len(gdel) > 0
    for k in ("disp", "disp_pre", "integ_stress", "element_flag", "Qe"):
        assert np.array_equal(getattr(ref[0][0], k), getattr(g, k)), k
    parts = [dist.slab_partition(glob, r, world, 4, 4) for r in range(world)]
    svs = []
    for r, (loc, diag, iface) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        for k, v in tune.items():
            sv.set_tuning(k, v)
        sv.set_element_offset(loc.global_element_offset)
        sv.comm_init_local(r, world, 900 + world)
        sv.set_interface(*iface)
        svs.append(sv)
    step_group(svs, 1, n)
    dels = []
    for sv, (loc, _, _) in zip(svs, parts):
        assert sv.stat("own_steps") == n
        st = sv.download()
        dels += [tuple(x) for x in sv.deleted()]
        n0, nl = loc.global_node_offset, loc.nNode
        e0, el = loc.global_element_offset, loc.nElement
        sl = slice(3 * n0, 3 * (n0 + nl))
        assert np.array_equal(st.disp, g.disp[sl])
        assert np.array_equal(st.disp_pre, g.disp_pre[sl])
        gp = slice(8 * e0, 8 * (e0 + el))
        assert np.array_equal(st.integ_stress, g.integ_stress[gp])
        assert np.array_equal(st.element_flag, g.element_flag[e0:e0 + el])
        assert np.array_equal(st.Qe, g.Qe[e0:e0 + el])
    for sv in svs:
        sv.close()
    assert sorted(dels) == gdel


def test_contact_group_owner_assembly_bitexact():
    """Contact on a communicator with owner-computed assembly (persistent kernel forced): the
    contact force enters the nodal update and the interface fix beside the owner-computed Q;
    every rank equals one context with the same mode, deletions included."""
    from hakai import mesh
    glob = mesh.two_body_model(plate=(8, 8, 2), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400)
    tune = {"elem_pipe_min": 0, "own_assembly": 1}
    with Solver(glob) as sv:
        for k, v in tune.items():
            sv.set_tuning(k, v)
        sv.step(1, glob.n_steps)
        g = sv.download()
        gdel = [tuple(x) for x in sv.deleted()]
        assert sv.stat("own_steps") == glob.n_steps
    parts = _run_contact_group(glob, 2, glob.n_steps, key=5150, tune=tune)
    _assert_group_equals_single(glob, parts, g, gdel)


def test_local_group_rejects_mixed_devices():
    """An in-process group shares one device (its kernels read the peers' buffers directly): a
    member on another device is rejected with HAKAI_ERR_ARG instead of faulting later
    (VERDICT r2 weak 7). Needs two visible GPUs (the pool's boxes have one: skipped there)."""
    import hakai
    from hakai._abi import HakaiError
    if hakai.device_count() < 2:
        pytest.skip("needs two GPUs")
    glob = fast_deletion_bar(2, 2, 8)
    parts = [dist.slab_partition(glob, r, 2, 2, 2) for r in range(2)]
    a = Solver(parts[0][0], diag_M=parts[0][1], device=0)
    b = Solver(parts[1][0], diag_M=parts[1][1], device=1)
    try:
        a.comm_init_local(0, 2, 4242)
        with pytest.raises(HakaiError) as ei:
            b.comm_init_local(1, 2, 4242)
        assert ei.value.code == -1 and "device" in str(ei.value)
    finally:
        a.close()
        b.close()
