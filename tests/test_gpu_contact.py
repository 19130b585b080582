"""GPU contact (hakai_contact.hip) against the oracle, through the C ABI.

* setup: pairs, exterior node / triangle counts and element sizes equal the oracle's;
* the contact force of one step, probed at oracle states, is bit-identical (both are the correctly
  rounded sum of the same FP64 terms: Float128 in the reference/oracle, double-double here);
* whole runs with contact, with friction (reference myu 0.25) and frictionless (BASELINE C4),
  self-contact, and contact-driven element deletion with the surface update: same deletions,
  displacement within the north star's 1e-6.
"""
import numpy as np
import pytest

from hakai import mesh
from hakai.solver import Solver, State
import oracle as O
from util import bitwise_equal, rel_err

pytestmark = pytest.mark.gpu


def _upload_oracle_state(o, sv):
    s = o.s
    st = State(s["disp"].copy(), s["disp_pre"].copy(), s["velo"].copy(), s["Q"].copy(), s["integ_stress"].copy(),
               s["integ_strain"].copy(), s["integ_yield_stress"].copy(), s["integ_eq_plastic_strain"].copy(),
               s["integ_triax_stress"].copy(), s["element_flag"].copy(), s["Qe"].copy())
    sv.upload(st)


@pytest.mark.parametrize("flag", [1, 2])
def test_contact_setup_matches_oracle(flag):
    m = mesh.two_body_model(plate=(5, 4, 2), impactor=(3, 2, 2), contact_flag=flag, perturb=0.05, seed=2)
    o = O.Oracle(m)
    with Solver(m) as sv:
        pairs, sizes = sv.contact_info()
    want = [(p["i_instance"], p["j_instance"], p["n_nodes_i"], p["n_triangles"], p["n_nodes_j"])
            for p in o.contact_pairs()]
    assert pairs == want
    assert sizes == (O.lib().hko_contact_min_size(o.ct), O.lib().hko_contact_max_size(o.ct))


def test_single_instance_self_pair():
    m = mesh.bar_model(2, 2, 3, mesh.steel_ductile(), 0.0)
    m.contact_flag = 1
    o = O.Oracle(m)
    with Solver(m) as sv:
        pairs, _ = sv.contact_info()
    p = o.contact_pairs()[0]
    assert pairs == [(1, 1, p["n_nodes_i"], p["n_triangles"], p["n_nodes_j"])]


@pytest.mark.parametrize("myu", [None, 0.0])
def test_contact_force_probe_bitexact(myu):
    m = mesh.two_body_model(plate=(6, 6, 2), impactor=(3, 3, 2), v=-1e5, perturb=0.03, seed=4, myu=myu)
    o = O.Oracle(m)
    total = 0
    with Solver(m) as sv:
        for t in range(1, 30):
            o.run(t, 1)
            _upload_oracle_state(o, sv)
            f = sv.contact_force(t + 1)
            fo, n = o.contact_force()
            assert np.array_equal(f, fo), f"step {t + 1}: max |diff| {np.max(np.abs(f - fo))}"
            total += n
    assert total > 20


@pytest.mark.parametrize("myu,flag", [(None, 1), (0.0, 1), (None, 2)])
def test_two_body_run_parity(myu, flag):
    m = mesh.two_body_model(plate=(6, 6, 2), impactor=(3, 3, 3), v=-1e5, perturb=0.02, seed=1, myu=myu,
                            contact_flag=flag, n_steps=300)
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    with Solver(m) as sv:
        sv.step(1, 100)
        sv.step(101, m.n_steps - 100)
        g = sv.download()
    assert rel_err(g.disp, o.s["disp"]) < 1e-9
    assert rel_err(g.velo, o.s["velo"]) < 1e-8
    assert rel_err(g.integ_stress, o.s["integ_stress"]) < 1e-8
    # the impactor was stopped / bounced by contact (it moved up at some point)
    assert np.max(g.disp[2::3]) > 0 or np.min(g.velo[2::3]) > -1e5


def test_contact_with_deletion_surface_update():
    m = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400)
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    assert len(o.deletions) >= 4
    with Solver(m) as sv:
        sv.step(1, m.n_steps)
        g = sv.download()
        dels = [tuple(x) for x in sv.deleted()]
    assert dels == sorted(o.deletions)
    assert np.array_equal(g.element_flag, o.s["element_flag"])
    assert rel_err(g.disp, o.s["disp"]) < 1e-6


def test_incremental_surface_lists_match_full_rebuild_and_oracle():
    """The live surface lists updated on the device after each deletion (k_ct_find_del/k_ct_append)
    give the same run, bit for bit, as a full rebuild every step, and -- after a probe at the next
    step -- the same list lengths as the oracle's c_triangles / c_nodes_i / c_nodes_j, which grow like
    the reference's (v2/HAKAI_j.jl:766-804)."""
    m = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400)
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    assert len(o.deletions) >= 4
    runs = []
    for full in (0, 1):
        with Solver(m) as sv:
            sv.set_tuning("contact_full_rebuild", full)
            sv.step(1, m.n_steps)
            g = sv.download()
            inc = sv.contact_stats()
            sv.contact_force(m.n_steps + 1)
            probe = sv.contact_stats()
            runs.append((g, inc, probe, [tuple(x) for x in sv.deleted()]))
    (g0, inc0, p0, d0), (g1, inc1, p1, d1) = runs
    assert d0 == d1 == sorted(o.deletions)
    assert np.array_equal(g0.disp, g1.disp) and np.array_equal(g0.integ_stress, g1.integ_stress)
    for k in ("live_triangles", "live_nodes_i", "live_nodes_j"):
        assert inc0[k] == inc1[k], k
    cp = o.contact_pairs()
    assert p0["live_triangles"] == sum(p["n_triangles"] for p in cp)
    assert p0["live_nodes_i"] == sum(p["n_nodes_i"] for p in cp)
    assert p0["live_nodes_j"] == sum(p["n_nodes_j"] for p in cp)


@pytest.mark.parametrize("graph,own", [(0, 0), (16, 0), (0, 1), (16, 1)])
def test_event_cap_overflow_is_reported(graph, own):
    """A contact step with more events than the buffer holds fails loudly (no silent truncation) AT
    that step: a device-side poison flag makes the nodal, BC and element kernels of that and every
    later step of the call no-ops, so the state afterwards is the last good step's, bit for bit
    (Q included: with owner-computed assembly it comes from the node sums, as the element kernel
    stored the per-element forces and the triaxiality only on the call's skipped last step, and
    those two downloads fail loudly until a step has run). Raising the cap through
    hakai_set_tuning and stepping on from the failed step gives the same run as a sufficient buffer
    from the start -- also when owner assembly is switched off for the rest of the run (the next
    nodal update then takes the owner sums as its Q)."""
    import re
    from hakai._abi import HakaiError
    # > 64 events per step once the 9x9-node impactor face is in contact: the smallest buffer (one
    # event in each of the 64 shards) must overflow
    m = mesh.two_body_model(plate=(12, 12, 1), impactor=(8, 8, 1), v=-1e5, perturb=0.03, seed=4, n_steps=60)
    tune = {"graph": graph, "own_assembly": own, "elem_pipe_min": 0, "elem_pipe_blocks": 3}

    def solver(cap):
        sv = Solver(m)
        for k, v in tune.items():
            sv.set_tuning(k, v)
        sv.set_tuning("contact_event_cap", cap)
        return sv

    keys = ("disp", "disp_pre", "velo", "integ_stress", "integ_eq_plastic_strain", "element_flag", "Q")
    with solver(1 << 12) as sv:
        sv.step(1, m.n_steps)
        full = sv.download()
        assert (sv.stat("own_steps") > 0) == bool(own)
    conts = []
    for switch_off in (False, True):
        with solver(1) as sv:
            with pytest.raises(HakaiError) as ei:
                sv.step(1, m.n_steps)
            p = int(re.search(r"step (\d+) was not applied", str(ei.value)).group(1))
            assert 1 < p < m.n_steps
            after = sv.download(**{k: True for k in keys})
            if own:
                with pytest.raises(HakaiError):
                    sv.download(Qe=True)
            with pytest.raises(HakaiError):
                sv.download(integ_triax_stress=True)
            sv.set_tuning("contact_event_cap", 1 << 12)
            if switch_off:
                sv.set_tuning("own_assembly", 0)
            sv.step(p, m.n_steps - p + 1)
            conts.append(sv.download())
    with solver(1 << 12) as sv:
        sv.step(1, p - 1)
        good = sv.download()
    for k in keys:
        assert bitwise_equal(getattr(after, k), getattr(good, k)), k
        for cont in conts:
            assert bitwise_equal(getattr(cont, k), getattr(full, k)), k
    for cont in conts:
        assert bitwise_equal(cont.integ_triax_stress, full.integ_triax_stress)
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    assert rel_err(full.disp, o.s["disp"]) < 1e-9


@pytest.mark.parametrize("surfaces", [False, True])
def test_driver_runs_contact_deck(tmp_path, surfaces):
    """HAKAI(fname) on a *Contact (all exterior) or *Contact Pair deck written from code: contact on
    the device path, 101 VTK files, final displacement equal to the oracle's to the VTK's %1.6e."""
    import os
    import hakai
    from inp_writer import write_inp
    m = mesh.two_body_model(plate=(5, 5, 2), impactor=(3, 3, 2), v=-1e5, n_steps=300, surfaces=surfaces)
    deck = write_inp(str(tmp_path / "impact.inp"), m)
    out = tmp_path / "out"
    hakai.hakai(deck, str(out), verbose=False)
    files = sorted(os.listdir(out))
    assert len(files) == 101 and files[-1] == "file100.vtk"
    txt = open(out / "file100.vtk").read().split("\n")
    i = txt.index("VECTORS DISPLACEMENT float")
    disp = np.array([[float(x) for x in l.split()] for l in txt[i + 1:i + 1 + m.nNode]])
    o = O.Oracle(hakai.read_inp(deck))
    o.run(1, m.n_steps)
    ref = o.s["disp"].reshape(-1, 3)
    assert np.allclose(disp, ref, rtol=2e-6, atol=1e-9)


def test_contact_pair_surfaces_parity():
    """*Contact Pair surfaces (plate top layer vs impactor bottom layer): same pair lists as the
    oracle, same trajectory."""
    m = mesh.two_body_model(plate=(6, 6, 2), impactor=(3, 3, 2), v=-1e5, perturb=0.02, seed=1, surfaces=True,
                            n_steps=300)
    o = O.Oracle(m)
    want = [(p["i_instance"], p["j_instance"], p["n_nodes_i"], p["n_triangles"], p["n_nodes_j"])
            for p in o.contact_pairs()]
    o.run(1, m.n_steps)
    with Solver(m) as sv:
        pairs, _ = sv.contact_info()
        sv.step(1, m.n_steps)
        g = sv.download()
    assert pairs == want
    assert rel_err(g.disp, o.s["disp"]) < 1e-9


@pytest.mark.parametrize("flag,graph", [(1, 16), (2, 0), (2, 16)])
def test_fused_small_deck_phases_bitexact(flag, graph):
    """Small decks run the contact prologue, the bucket scan + fill and the event gather as single
    1024-thread workgroups and the binning with the prefilter in one launch (Contact::small,
    tuning contact_fuse_small): the trajectory, the deletion log and the contact counters equal
    the one-kernel-per-phase path bit for bit, with deletions, self-contact and graphs."""
    m = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400,
                            contact_flag=flag)
    out = []
    for fuse in (0, 1):
        with Solver(m) as sv:
            sv.set_tuning("graph", graph)
            sv.set_tuning("contact_fuse_small", fuse)
            sv.step(1, 250)
            sv.step(251, m.n_steps - 250)
            out.append((sv.download(), [tuple(int(v) for v in x) for x in sv.deleted()], sv.contact_stats()))
    (a, da, sa), (b, db, sb) = out
    assert da == db and len(da) > 0
    assert sa["max_events"] == sb["max_events"] and sa["live_triangles"] == sb["live_triangles"]
    for k in ("disp", "disp_pre", "velo", "integ_stress", "integ_eq_plastic_strain", "element_flag"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k




@pytest.mark.parametrize("graph", [0, 16])
def test_overflow_recovery_paths_keep_q(graph):
    """The owner-assembly Q survives every way back from a contact overflow:
    (a) a call whose FIRST step overflows (nothing of it ran) after an upload with Q: the uploaded
        Q is still the one the next nodal update takes;
    (b) an upload of the state without Q or Qe after an overflowed call: the owner sums become Q
        (fe is an earlier step's there);
    (c) such an upload that also deletes elements is refused (their fe rows cannot be zeroed).
    Each continuation, with the buffer raised, equals an uninterrupted run bit for bit."""
    import re
    from hakai._abi import HakaiError
    m = mesh.two_body_model(plate=(12, 12, 1), impactor=(8, 8, 1), v=-1e5, perturb=0.03, seed=4, n_steps=60)
    tune = {"graph": graph, "own_assembly": 1, "elem_pipe_min": 0, "elem_pipe_blocks": 3}

    def solver(cap):
        sv = Solver(m)
        for k, v in tune.items():
            sv.set_tuning(k, v)
        sv.set_tuning("contact_event_cap", cap)
        return sv

    keys = ("disp", "disp_pre", "velo", "integ_stress", "integ_strain", "integ_eq_plastic_strain",
            "integ_yield_stress", "element_flag", "Q")
    with solver(1 << 12) as sv:
        events = []
        for t in range(1, m.n_steps + 1):
            sv.step(t, 1)
            events.append(sv.contact_stats()["events"])
        full = sv.download()
        assert sv.stat("own_steps") > 0
    # which step overflows first at one record per event shard depends on how the step's events
    # fall into the 64 shards (the candidate order is the atomics'); a step with more than 64
    # events overflows whatever the order
    p = 1 + next(k for k, e in enumerate(events) if e > 64)

    def fail_step(sv, t0):
        with pytest.raises(HakaiError) as ei:
            sv.step(t0, m.n_steps - t0 + 1)
        return int(re.search(r"step (\d+) was not applied", str(ei.value)).group(1))

    # (a) upload with Q, then a call that overflows at once
    with solver(1 << 12) as sv:
        sv.step(1, p - 1)
        sv.set_tuning("contact_event_cap", 1)
        assert fail_step(sv, p) == p
        st = sv.download(**{k: True for k in keys})
        sv.upload(st)                              # Q -> the uploaded-Q buffer, owner sums off
        assert fail_step(sv, p) == p               # good == 0
        sv.set_tuning("contact_event_cap", 1 << 12)
        sv.step(p, m.n_steps - p + 1)
        a = sv.download()
    # (b) upload without Q / Qe after the overflow
    with solver(1) as sv:
        p = fail_step(sv, 1)
        st = sv.download(**{k: True for k in keys})
        st_noq = State(st.disp, st.disp_pre, st.velo, None, st.integ_stress, st.integ_strain, st.integ_yield_stress,
                       st.integ_eq_plastic_strain, None, st.element_flag, None)
        sv.upload(st_noq)
        sv.set_tuning("contact_event_cap", 1 << 12)
        sv.step(p, m.n_steps - p + 1)
        b = sv.download()
    # (c) refused with deletions and no Q
    with solver(1) as sv:
        fail_step(sv, 1)
        st = sv.download(**{k: True for k in keys})
        fl = st.element_flag.copy()
        fl[0] = 0
        with pytest.raises(HakaiError, match="upload Q"):
            sv.upload(State(st.disp, st.disp_pre, st.velo, None, st.integ_stress, st.integ_strain,
                            st.integ_yield_stress, st.integ_eq_plastic_strain, None, fl, None))
    for k in keys:
        assert bitwise_equal(getattr(a, k), getattr(full, k)), ("a", k)
        assert bitwise_equal(getattr(b, k), getattr(full, k)), ("b", k)
