"""Multi-rank parity on one GPU: an in-process group of contexts (hakai_comm_init_local) runs the
same partition, pack / interface-sum / fix kernels and exchange protocol as the RCCL path
(hakai_comm.cpp), and must reproduce the single-context run BIT FOR BIT: the interface Q is summed
in the reference's serial element order (v2/HAKAI_j.jl:669-675) on both sides of every cut.
"""
import numpy as np
import pytest

from hakai import dist
from hakai.solver import Solver, step_group
from util import fast_deletion_bar

pytestmark = pytest.mark.gpu


def _run_group(glob, world, n_steps, key, fe_layout=0):
    nx = ny = 2
    parts = [dist.slab_partition(glob, r, world, nx, ny) for r in range(world)]
    svs = []
    for r, (loc, diag, iface) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        sv.set_tuning("fe_layout", fe_layout)
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


@pytest.mark.parametrize("world,fe_layout", [(2, 0), (3, 0), (2, 1)])
def test_local_group_bitexact(world, fe_layout):
    glob = fast_deletion_bar(2, 2, 12)
    n = 1200
    with Solver(glob) as sv:
        sv.step(1, n)
        g = sv.download()
        gdel = [tuple(x) for x in sv.deleted()]
    assert len(gdel) > 0, "config must delete elements"
    parts = _run_group(glob, world, n, key=100 + 10 * fe_layout + world, fe_layout=fe_layout)
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
