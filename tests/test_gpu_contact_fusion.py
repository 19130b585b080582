"""Contact launch fusions (hakai_contact.hip): the binning and the triangle prefilter as one launch
(k_ct_binfilter; tuning contact_fuse_binfilter) give the same run as two launches, bit for bit,
with deletions, self-contact and graphs (the multi-GPU insert + prefilter fusion, k_xr_insfilter,
is checked in test_gpu_multirank.py)."""
import numpy as np
import pytest

from hakai import mesh
from hakai.solver import Solver

pytestmark = pytest.mark.gpu

KEYS = ("disp", "disp_pre", "velo", "integ_stress", "integ_eq_plastic_strain", "element_flag")


def _deck(flag=1):
    return mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400,
                               contact_flag=flag)


@pytest.mark.parametrize("graph", [0, 16])
def test_binfilter_fusion_bitexact(graph):
    """The binning and the prefilter in one launch (tuning contact_fuse_binfilter, default on) or in
    two: the same run bit for bit (large decks take this path; contact_fuse_small 0 runs it here)."""
    m = _deck(2)
    out = []
    for bf in (0, 1):
        with Solver(m) as sv:
            sv.set_tuning("graph", graph)
            sv.set_tuning("contact_fuse_small", 0)
            sv.set_tuning("contact_fuse_binfilter", bf)
            sv.step(1, m.n_steps)
            out.append((sv.download(), [tuple(int(v) for v in x) for x in sv.deleted()], sv.contact_stats()))
    (a, da, sa), (b, db, sb) = out
    assert da == db and len(da) > 0
    assert sa["candidate_triangles"] == sb["candidate_triangles"] and sa["events"] == sb["events"]
    for k in KEYS:
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
