"""The reference's own input decks on the GPU path, against the oracle (tests/golden/deck_*.npz,
made by tools/make_deck_golden.py from HAKAI-v0.0.0/v0.0.1 decks parsed by the v0.0.2 reader):

* Charpy-test.inp: *Contact between the striker and a notched specimen, ductile deletion;
* crash-tube-80-350-solid.inp: HAKAIoption=self-contact (contact_flag 2), a buckling tube;
* bullet-impact.inp: projectile into a plate with deletion.

Same deletion log and element flags, displacement within the north star's 1e-6 relative; and the
Charpy deck on a 2-rank in-process group (multi-GPU contact) bit-identical to one context.
"""
import os

import numpy as np
import pytest

from deck_fixtures import model_from_arrays
from hakai import dist
from hakai.solver import Solver, step_group
from util import rel_err

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _deck(name):
    z = np.load(os.path.join(GOLDEN, f"deck_{name}.npz"))
    return z, model_from_arrays(z, name)


@pytest.mark.parametrize("name", ["Charpy_test", "crash_tube_80_350_solid", "bullet_impact"])
def test_reference_deck_parity(name):
    z, m = _deck(name)
    steps = int(z["steps"])
    with Solver(m) as sv:
        sv.step(1, steps // 2)
        sv.step(1 + steps // 2, steps - steps // 2)
        g = sv.download()
        dels = [tuple(int(v) for v in x) for x in sv.deleted()]
    assert dels == [tuple(int(v) for v in x) for x in z["deletions"]]
    assert np.array_equal(g.element_flag, z["element_flag"])
    assert rel_err(g.disp, z["disp"]) < 1e-6
    assert rel_err(g.disp_pre, z["disp_pre"]) < 1e-6


def test_charpy_deck_two_ranks_bitexact():
    z, glob = _deck("Charpy_test")
    steps = int(z["steps"])
    with Solver(glob) as sv:
        sv.step(1, steps)
        g = sv.download()
        gdel = [tuple(x) for x in sv.deleted()]
    gdiag, _ = glob.lumped_mass()
    parts = [dist.range_partition(glob, r, 2, gdiag) for r in range(2)]
    svs = []
    for r, (loc, diag, iface, l2g, off) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        sv.set_element_offset(loc.global_element_offset)
        sv.comm_init_local(r, 2, 5150)
        sv.set_interface(*iface)
        sv.set_contact_global(glob, l2g, off, gdiag)
        svs.append(sv)
    step_group(svs, 1, steps)
    dels = []
    for sv, (loc, _, _, l2g, _) in zip(svs, parts):
        st = sv.download()
        dels += [tuple(x) for x in sv.deleted()]
        assert np.array_equal(st.disp.reshape(-1, 3), g.disp.reshape(-1, 3)[l2g - 1])
        e0 = loc.global_element_offset
        assert np.array_equal(st.element_flag, g.element_flag[e0:e0 + loc.nElement])
        sv.close()
    assert sorted(dels) == gdel and len(gdel) > 0
