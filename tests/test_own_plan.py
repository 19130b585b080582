"""Owner-computed assembly plans, replayed on the CPU (tools/own_plan_check.cpp, no GPU).

The planner (hakai_capi.cpp own_choose / own_plan: block schedules, contiguous batch ranges or row
bands) decides which element-kernel block sums
which node contributions in which order. The replay executes each plan as k_element_pipe and k_nodal
do and checks that every node's Q equals the reference's serial assembly in ascending element order
(v2/HAKAI_j.jl:668-675) BIT FOR BIT, for random contributions spanning 60 binades -- for slender and
wide sections, two bodies with different lattice strides (C4's shape), shuffled numbering, the
finer fallback grid and tiny grids. The GPU tests (tests/test_gpu_own.py) then check that the
kernels execute the same plans.
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "_build", "own_plan_check")

CASES = [
    ("20 20 300", {}),                                              # C3's section
    ("20 20 300 --exact 1", {}),
    ("100 100 40 --G 32", {"banded": 1, "epb": 32}),              # C5's section: row bands
    ("100 100 40 --G 32 --exact 1", {"banded": 1}),
    ("200 200 5 --G 128 --schedule 2", {"banded": 1}),             # C4 plate's section
    ("30 30 12 --plate 120 120 3 --G 48 --schedule 2", {"banded": 1}),  # two lattices (C4's shape)
    ("40 30 8 --plate 60 50 4 --exact 1", {}),
    ("3 3 200 --G 8 --shuffle 11", {"banded": 0}),                  # shuffled numbering
    ("60 60 6 --G 1", {"grid": 8}),                                 # too many open sums: 8x finer grid
    ("4 4 40 --G 3", {"grid": 3}),
    ("5 1 1 --G 1", {}),                                            # Tensile5e-sized: one batch
    ("100 100 16 --G 128 --band-rows 2 --schedule 2", {"banded": 1}),  # forced band heights (own_band_rows)
    ("100 100 16 --G 128 --band-rows 3 --schedule 2 --exact 1", {"banded": 1}),
]


@pytest.mark.parametrize("args,expect", CASES)
def test_owner_plan_replay_bitexact(args, expect):
    if not os.path.exists(EXE):
        pytest.skip("tools/_build/own_plan_check not built (__graft_entry__.build())")
    out = subprocess.run([EXE] + args.split(), capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["ok"] and r["planned"], r
    assert r["mismatch"] == 0 and r["double_fin"] == 0, r
    assert r["slots"] <= r["slot_cap"], r
    for k, v in expect.items():
        assert r[k] == v, (k, r)


def test_owner_plan_wide_sections_export_fewer_rows():
    """Row bands cut the exported rows of a 100x100 section against contiguous ranges."""
    if not os.path.exists(EXE):
        pytest.skip("tools/_build/own_plan_check not built")
    res = {}
    for sched in (1, 2):
        out = subprocess.run([EXE, "100", "100", "40", "--G", "64", "--schedule", str(sched)], capture_output=True,
                             text=True, timeout=120)
        res[sched] = json.loads(out.stdout.strip().splitlines()[-1])
    assert res[2]["planned"] and res[2]["banded"] == 1
    if res[1]["planned"]:
        assert res[2]["rows"] < res[1]["rows"], res
