"""Owner-computed assembly (tuning key "own_assembly"): the persistent element kernel sums node
forces in LDS, in element order, and hands the nodal update each node's Q -- or its prefix partial
plus the later blocks' contributions as individual rows -- instead of the 24-B-per-element-node fe
array. The additions are the nodal gather's own, in the same order
(v2/HAKAI_j.jl:668-675 serial sum), so every run here must be BIT-identical to the fe path: the same
tuning with own_assembly 0. Block ranges are forced small so node sums straddle 2-3 blocks (prefix
partial + exported rows), and meshes that need more LDS sums than a block holds fall back.
"""
import numpy as np
import pytest

from hakai import mesh
from hakai.solver import Solver
from util import same_state as _same, shuffled as _shuffled
from util import fast_deletion_bar, small_bar

pytestmark = pytest.mark.gpu


def _run(m, calls, tune, own, graph=None):
    with Solver(m) as sv:
        for k, v in tune.items():
            sv.set_tuning(k, v)
        sv.set_tuning("own_assembly", own)
        if graph is not None:
            sv.set_tuning("graph", graph)
        for t0, n in calls:
            sv.step(t0, n)
        g = sv.download()
        dels = [tuple(x) for x in sv.deleted()]
        st = {k: sv.stat(k) for k in ("own_steps", "own_rows", "own_entries", "graph_steps")}
    return g, dels, st


PIPE = {"elem_pipe_min": 0}


@pytest.mark.parametrize("blocks", [3, 16, 200])
def test_own_deletion_bar_bitexact(blocks):
    """Deleting bar, 6 400 hex = 200 batches over 3 / 16 / 200 persistent blocks (200: one batch per
    block, most nodes straddle blocks); odd step counts, several calls, graphs on."""
    m = fast_deletion_bar(4, 4, 400)
    calls = [(1, 301), (302, 1000), (1302, 1699)]
    tune = {**PIPE, "elem_pipe_blocks": blocks}
    g0, d0, s0 = _run(m, calls, tune, 0)
    g1, d1, s1 = _run(m, calls, tune, 1)
    assert s0["own_steps"] == 0 and s1["own_steps"] == 3000, (s0, s1)
    assert s1["own_rows"] > 0 and s1["graph_steps"] > 0
    assert len(d0) > 0 and d1 == d0
    _same(g1, g0)


def test_own_stream_mode_and_toggle():
    """Stream mode (graph 0), and own_assembly switched off and on between calls."""
    m = small_bar(6, 5, 300, n_steps=600, v_end=5e5)
    tune = {**PIPE, "elem_pipe_blocks": 32}
    g0, _, _ = _run(m, [(1, 600)], tune, 0, graph=0)
    with Solver(m) as sv:
        for k, v in tune.items():
            sv.set_tuning(k, v)
        sv.set_tuning("graph", 0)
        for t0, n, own in ((1, 150, 1), (151, 151, 0), (302, 99, 1), (401, 200, 1)):
            sv.set_tuning("own_assembly", own)
            sv.step(t0, n)
        g1 = sv.download()
        assert sv.stat("own_steps") == 449
    assert np.any(g0.integ_eq_plastic_strain > 0)
    _same(g1, g0)


def test_own_shuffled_numbering_bitexact():
    """Random element and node numbering (long-lived LDS sums, many rows) or a fallback: bit-identical."""
    m = _shuffled(fast_deletion_bar(3, 3, 200), seed=11)
    tune = {**PIPE, "elem_pipe_blocks": 8}
    g0, d0, _ = _run(m, [(1, 3000)], tune, 0)
    g1, d1, s1 = _run(m, [(1, 3000)], tune, 1)
    assert d1 == d0 and len(d0) > 0
    _same(g1, g0)
    # the sums of a shuffled mesh stay open for most of a block's range: more than a block's LDS slots
    assert s1["own_steps"] in (0, 3000)


def test_own_wide_section_finer_grid_or_fallback():
    """A 40x40 cross-section on 1 block: too many open sums, so the lists are built for 8 blocks
    (blocks then run in waves) -- or the fe path; either way bit-identical. A shuffled wide mesh
    fits in one block's slots or takes the fe path."""
    m = small_bar(40, 40, 6, n_steps=200, v_end=5e5)
    tune = {**PIPE, "elem_pipe_blocks": 1}
    g0, _, _ = _run(m, [(1, 200)], tune, 0)
    g1, _, s1 = _run(m, [(1, 200)], tune, 1)
    assert s1["own_steps"] == 200, s1
    _same(g1, g0)
    ms = _shuffled(m, seed=3)
    g0, _, _ = _run(ms, [(1, 60)], tune, 0)
    g1, _, s1 = _run(ms, [(1, 60)], tune, 1)
    # (since round 3 a block holds up to 2048 sums, what its LDS allows, so this mesh may fit)
    assert s1["own_steps"] == 60 or (s1["own_steps"] == 0 and s1["own_rows"] == -1), s1
    _same(g1, g0)


@pytest.mark.parametrize("layers", [12])
def test_own_wide_section_two_entry_passes(layers):
    """100x100 cross-section (C5's): some 64-element super-batches need more than 256 entries, so
    those passes take a second entry per thread; bit-identical to the fe path."""
    m = small_bar(100, 100, layers, n_steps=100, v_end=5e5)
    g0, _, _ = _run(m, [(1, 100)], {}, 0)
    with Solver(m) as sv:
        sv.set_tuning("own_assembly", 1)
        sv.step(1, 100)
        g1 = sv.download()
        assert sv.stat("own_steps") == 100
        assert sv.stat("own_superbatch") == 2
    _same(g1, g0)


def test_own_contact_two_bodies_bitexact():
    """External (contact) force beside the owner-computed Q: impactor on a plate, with deletions."""
    m = mesh.two_body_model(plate=(12, 12, 3), impactor=(4, 4, 6), gap=0.05, v=-2e5)
    n = 1500
    tune = {**PIPE, "elem_pipe_blocks": 2}
    g0, d0, _ = _run(m, [(1, 701), (702, n - 701)], tune, 0)
    g1, d1, s1 = _run(m, [(1, 701), (702, n - 701)], tune, 1)
    assert s1["own_steps"] == n
    assert d1 == d0
    assert np.max(np.abs(g0.disp)) > 0
    _same(g1, g0)


def test_own_upload_state_mid_run():
    """An uploaded state (Q from the upload, then fe gathers on the first owner step) matches."""
    m = fast_deletion_bar(3, 3, 120)
    with Solver(m) as sv:
        sv.step(1, 500)
        mid = sv.download()
    outs = []
    for own in (0, 1):
        with Solver(m) as sv:
            for k, v in {**PIPE, "elem_pipe_blocks": 5}.items():
                sv.set_tuning(k, v)
            sv.set_tuning("own_assembly", own)
            sv.upload(mid)
            sv.step(501, 800)
            outs.append(sv.download())
    _same(outs[1], outs[0])


def test_own_tensile5e_padded_batch_vs_oracle():
    """Tensile5e.inp (5 hex: one batch, 27 padding elements; amplitude BCs; element 3 deleted at
    step 15 153) on the persistent kernel with owner assembly: the fused kernel's oracle parity
    (1e-6) and bit-identity with the fe path."""
    import oracle as O
    m = mesh.tensile5e_model()
    o = O.Oracle(m)
    o.run(1, m.n_steps)
    g0, d0, _ = _run(m, [(1, m.n_steps)], PIPE, 0)
    g1, d1, s1 = _run(m, [(1, m.n_steps)], PIPE, 1)
    assert s1["own_steps"] == m.n_steps
    assert d1 == d0 == o.deletions == [(15153, 3)]
    _same(g1, g0)
    assert np.max(np.abs(g1.disp - o.s["disp"])) / np.max(np.abs(o.s["disp"])) < 1e-6


def test_own_isolated_node_and_ragged_batch():
    """63 hex (last batch ragged) plus a node no element uses (Q = 0, its own sum never written)."""
    from hakai.model import Model
    base = small_bar(3, 3, 7, n_steps=300, v_end=5e5)
    coord = np.vstack([base.coordmat, [[50.0, 50.0, 50.0]]])
    extra = coord.shape[0]
    m = Model(coord, base.elementmat, base.element_material, base.materials, bc=base.bc,
              ic_dofs=np.concatenate([base.ic_dofs, [3 * extra]]),
              ic_values=np.concatenate([np.asarray(base.ic_values), [1e3]]), d_time=base.d_time,
              end_time=base.end_time, name="ragged_isolated")
    g0, _, _ = _run(m, [(1, 151), (152, 149)], PIPE, 0)
    g1, _, s1 = _run(m, [(1, 151), (152, 149)], PIPE, 1)
    assert s1["own_steps"] == 300
    # the isolated node has no mass (the reference's update divides by it): compare NaN as equal
    from util import STATE
    for k in STATE:
        assert np.array_equal(getattr(g1, k), getattr(g0, k), equal_nan=True), k
    assert np.all(g1.Q[3 * extra - 3:] == 0.0)
    assert np.all(np.isfinite(g1.disp[:3 * extra - 3]))


def test_own_grid_change_between_calls_rebuilds():
    """elem_pipe_blocks changed between calls: the owner lists are rebuilt for the new grid (the
    call boundary leaves fe valid for the first step), results unchanged."""
    m = small_bar(6, 5, 300, n_steps=600, v_end=5e5)
    g0, _, _ = _run(m, [(1, 600)], PIPE, 0)
    with Solver(m) as sv:
        sv.set_tuning("elem_pipe_min", 0)
        seen = []
        for t0, n, blocks in ((1, 201, 32), (202, 200, 12), (402, 199, 40)):
            sv.set_tuning("elem_pipe_blocks", blocks)
            sv.step(t0, n)
            seen.append(sv.stat("own_entries"))
        g1 = sv.download()
        assert sv.stat("own_steps") == 600
    assert len(set(seen)) == 3  # three partitions, three list sets
    _same(g1, g0)


@pytest.mark.parametrize("shape", [(100, 100, 16), (200, 200, 5)])
def test_own_banded_wide_sections_bitexact(shape):
    """Wide cross-sections (C5's 100x100, C4's plate 200x200): the planner picks the row-band
    schedule (each block walks one band of element rows over a run of layers; it exports fewer rows
    than contiguous batch ranges, tests/test_own_plan.py) and the result is bit-identical to the fe
    path."""
    nx, ny, nz = shape
    m = small_bar(nx, ny, nz, n_steps=120, v_end=5e5)
    tune = {"elem_pipe_blocks": 128}  # (the 200-wide section's 67 row bands need a block each)
    calls = [(1, 61), (62, 59)]
    g0, _, _ = _run(m, calls, tune, 0)
    g1, _, st = _run(m, calls, tune, 1)
    _same(g1, g0)
    assert st["own_steps"] == 120, st
    with Solver(m) as sv:
        for k, v in tune.items():
            sv.set_tuning(k, v)
        sv.step(1, 1)
        assert sv.stat("own_banded") == 1


def test_own_banded_two_bodies_contact_bitexact():
    """C4's shape at small size: a 120x120 plate and an impactor (two structured regions with
    different strides), contact on, row bands in each region: bit-identical to the fe path."""
    m = mesh.two_body_model(plate=(120, 120, 3), impactor=(30, 30, 12), gap=0.05, v=-2e4)
    n = 300
    tune = {"elem_pipe_blocks": 48}
    g0, d0, _ = _run(m, [(1, 151), (152, n - 151)], tune, 0)
    with Solver(m) as sv:
        for k, v in tune.items():
            sv.set_tuning(k, v)
        sv.set_tuning("own_assembly", 1)
        sv.step(1, 151)
        sv.step(152, n - 151)
        g1 = sv.download()
        d1 = [tuple(x) for x in sv.deleted()]
        assert sv.stat("own_steps") == n and sv.stat("own_banded") == 1
    assert d1 == d0
    assert np.all(np.isfinite(g0.disp)) and np.max(np.abs(g0.disp)) > 0
    assert np.max(np.abs(g0.Q)) > 0
    _same(g1, g0)


@pytest.mark.parametrize("shape", [(100, 100, 12), (20, 20, 60)])
def test_own_reference_order_mode_bitexact(shape):
    """The reference-order kernel with owner sums forced on (own_assembly 2), on a wide section
    whose lists need second-entry passes (where the default, own_assembly 1, takes the fe path) and
    on a slender one: bit-identical to the fe path."""
    m = small_bar(*shape, n_steps=80, v_end=5e5)
    tune = {"elem_pipe_blocks": 64, "elem_exact": 1}
    calls = [(1, 41), (42, 39)]
    g0, _, _ = _run(m, calls, tune, 0)
    stats = {}
    for own in (1, 2):
        g1, _, st = _run(m, calls, tune, own)
        _same(g1, g0)
        stats[own] = st
    assert stats[2]["own_steps"] == 80, stats


def test_own_elem_exact_switch_mid_run_replans():
    """Switching the element kernel between calls re-plans the owner lists for the new kernel's LDS
    budget: on a wide section over 8 blocks the fused kernel's row bands need ~1670 slots,
    more than the reference-order kernel has (~920), so keeping that plan failed the launch. Fused ->
    reference order -> fused with owner sums forced on (own_assembly 2) must equal the same switches
    on the fe path, bit for bit."""
    m = small_bar(100, 100, 12, n_steps=90, v_end=5e5)
    res = {}
    for own in (0, 2):
        with Solver(m) as sv:
            sv.set_tuning("elem_pipe_blocks", 8)
            sv.set_tuning("own_assembly", own)
            sv.step(1, 30)
            slots_fused = sv.stat("own_slots")
            sv.set_tuning("elem_exact", 1)
            sv.step(31, 30)
            slots_exact = sv.stat("own_slots")
            sv.set_tuning("elem_exact", 0)
            sv.step(61, 30)
            res[own] = (sv.download(), sv.stat("own_steps"), slots_fused, slots_exact)
    g2, steps2, sf, se = res[2]
    assert steps2 == 90, res[2][1:]
    assert sf > 923 >= se, (sf, se)  # the two kernels really needed different plans
    _same(g2, res[0][0])


def test_own_band_rows_change_between_calls_replans():
    """own_band_rows forces the row-band height (2, 3, then the planned 4 again); each change
    re-plans the lists at the next step, handing the previous step's sums to the nodal update through
    the uploaded-Q path: bit-identical to the fe path, and each height gives its own list set."""
    m = small_bar(100, 100, 16, n_steps=90, v_end=5e5)
    tune = {"elem_pipe_blocks": 128}
    g0, _, _ = _run(m, [(1, 31), (32, 30), (62, 29)], tune, 0)
    with Solver(m) as sv:
        for k, v in tune.items():
            sv.set_tuning(k, v)
        sv.set_tuning("own_assembly", 1)
        rows = []
        for (t0, n), r in zip(((1, 31), (32, 30), (62, 29)), (2, 3, 0)):
            sv.set_tuning("own_band_rows", r)
            sv.step(t0, n)
            assert sv.stat("own_banded") == 1
            rows.append(sv.stat("own_rows"))
        g1 = sv.download()
        assert sv.stat("own_steps") == 90
        with pytest.raises(Exception):
            sv.set_tuning("own_band_rows", -1)
    assert rows[0] > rows[1] > rows[2], rows  # lower bands export more rows (CPU replay: 543 k, 412 k, 402 k)
    _same(g1, g0)


def test_own_pass_batches_forced_one_bitexact():
    """own_pass_batches 1: one batch per summing pass where the planner would take two (a 100-wide
    section, whose two-batch passes need second entry rounds): re-planned between calls, bit-identical
    to the fe path, no second rounds."""
    m = small_bar(100, 100, 16, n_steps=60, v_end=5e5)
    tune = {"elem_pipe_blocks": 128}
    g0, _, _ = _run(m, [(1, 31), (32, 29)], tune, 0)
    with Solver(m) as sv:
        for k, v in tune.items():
            sv.set_tuning(k, v)
        sv.set_tuning("own_assembly", 1)
        sv.step(1, 31)
        assert sv.stat("own_superbatch") == 2
        sv.set_tuning("own_pass_batches", 1)
        sv.step(32, 29)
        assert sv.stat("own_superbatch") == 1 and sv.stat("own_round2") == 0
        assert sv.stat("own_steps") == 60
        g1 = sv.download()
        with pytest.raises(Exception):
            sv.set_tuning("own_pass_batches", 3)
    _same(g1, g0)
