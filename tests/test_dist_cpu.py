"""Multi-rank path on CPU: the slab partition (hakai.dist) and the interface-exchange protocol of
hakai_comm.cpp, run over torch.distributed `gloo` with world_size 2 and 3.

The protocol claim: at a node shared by ranks r < r+1, rank r sends P = its own contributions summed
in element order, rank r+1 sends its contributions one by one (zero padded to nslot), and both form
((P + c1) + c2) + ... -- bit-identical to the reference's serial element-order assembly
(v2/HAKAI_j.jl:669-675) over the whole mesh. Element forces here are seeded random vectors: the
claim is about summation order only.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

from hakai import dist
from util import fast_deletion_bar

NX = NY = 2

def _serial_Q(nN, elementmat, Qe):
    Q = np.zeros(3 * nN)
    for e in range(elementmat.shape[0]):
        for i in range(8):
            n = elementmat[e, i] - 1
            for c in range(3):
                Q[3 * n + c] += Qe[e, 3 * i + c]
    return Q

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p

def _worker(rank, world, port, nz, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        glob = fast_deletion_bar(NX, NY, nz)
        loc, diag, (ln, lo, hi) = dist.slab_partition(glob, rank, world, NX, NY)
        rng = np.random.default_rng(1234)
        Qe_glob = rng.normal(0, 1.0, size=(glob.nElement, 24))
        e0 = loc.global_element_offset
        Qe = Qe_glob[e0:e0 + loc.nElement]
        # own contributions per local node, in element order (the device CSR incidence order)
        contrib = [[] for _ in range(loc.nNode)]
        for e in range(loc.nElement):
            for i in range(8):
                contrib[loc.elementmat[e, i] - 1].append(Qe[e, 3 * i:3 * i + 3])
        Q = np.zeros(3 * loc.nNode)
        for n in range(loc.nNode):
            for f in contrib[n]:
                Q[3 * n:3 * n + 3] += f
        up = ln[lo == rank]
        dn = ln[hi == rank]
        nslot = torch.tensor([max([len(contrib[n]) for n in dn], default=0)])
        tdist.all_reduce(nslot, op=tdist.ReduceOp.MAX)
        nslot = int(nslot)
        P = np.array([Q[3 * n:3 * n + 3] for n in up]).reshape(-1, 3)
        C = np.zeros((len(dn), nslot, 3))
        for j, n in enumerate(dn):
            for s, f in enumerate(contrib[n]):
                C[j, s] = f
        ops, recvC, recvP = [], None, None
        if len(up):
            recvC = torch.zeros(len(up), nslot, 3, dtype=torch.float64)
            ops += [tdist.P2POp(tdist.isend, torch.from_numpy(P.copy()), rank + 1),
                    tdist.P2POp(tdist.irecv, recvC, rank + 1)]
        if len(dn):
            recvP = torch.zeros(len(dn), 3, dtype=torch.float64)
            ops += [tdist.P2POp(tdist.isend, torch.from_numpy(C.copy()), rank - 1),
                    tdist.P2POp(tdist.irecv, recvP, rank - 1)]
        for r in tdist.batch_isend_irecv(ops):
            r.wait()
        for j, n in enumerate(up):
            q = P[j].copy()
            for s in range(nslot):
                q = q + recvC[j, s].numpy()
            Q[3 * n:3 * n + 3] = q
        for j, n in enumerate(dn):
            q = recvP[j].numpy().copy()
            for s in range(nslot):
                q = q + C[j, s]
            Q[3 * n:3 * n + 3] = q
        Qref = _serial_Q(glob.nNode, glob.elementmat, Qe_glob)
        n0 = loc.global_node_offset
        gdiag, _ = glob.lumped_mass()
        ok_q = np.array_equal(Q, Qref[3 * n0:3 * (n0 + loc.nNode)])
        ok_m = np.array_equal(diag, gdiag[3 * n0:3 * (n0 + loc.nNode)])
        ok_x = np.array_equal(loc.coordmat, glob.coordmat[n0:n0 + loc.nNode])
        ok_e = np.array_equal(loc.elementmat + n0, glob.elementmat[e0:e0 + loc.nElement])
        ret[rank] = (ok_q, ok_m, ok_x, ok_e, len(up), len(dn))
    finally:
        tdist.destroy_process_group()

@pytest.mark.parametrize("world", [2, 3])
def test_gloo_interface_protocol_bitexact(world):
    ctx = mp.get_context("spawn")
    ret = ctx.Manager().dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 12, ret))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    for r in range(world):
        ok_q, ok_m, ok_x, ok_e, nu, nd = ret[r]
        assert ok_q, f"rank {r}: interface Q differs from the serial assembly"
        assert ok_m, f"rank {r}: halo lumped mass differs from the global mass"
        assert ok_x and ok_e
        assert nu == (NX + 1) * (NY + 1) * (r < world - 1)
        assert nd == (NX + 1) * (NY + 1) * (r > 0)

def test_partition_covers_mesh_and_bcs():
    glob = fast_deletion_bar(NX, NY, 12)
    for world in (1, 2, 3, 4):
        parts = [dist.slab_partition(glob, r, world, NX, NY) for r in range(world)]
        assert sum(p[0].nElement for p in parts) == glob.nElement
        # every constrained global dof appears in the local BCs of each rank holding that node
        for loc, _, _ in parts:
            n0 = loc.global_node_offset
            gd = {int(d) for g in glob.bc for d, _ in g.entries for d in d
                  if n0 <= (d - 1) // 3 < n0 + loc.nNode}
            ld = {int(d) + 3 * n0 for g in loc.bc for d, _ in g.entries for d in d}
            assert gd == ld

def _same_model(a, b):
    assert np.array_equal(a.coordmat, b.coordmat) and a.coordmat.dtype == b.coordmat.dtype
    assert np.array_equal(a.elementmat, b.elementmat)
    assert np.array_equal(a.element_material, b.element_material)
    assert np.array_equal(a.ic_dofs, b.ic_dofs) and np.array_equal(a.ic_values, b.ic_values)
    assert (a.d_time, a.end_time, a.mass_scaling, a.name) == (b.d_time, b.end_time, b.mass_scaling, b.name)
    assert len(a.bc) == len(b.bc)
    for ga, gb in zip(a.bc, b.bc):
        assert len(ga.entries) == len(gb.entries)
        for (da, va), (db, vb) in zip(ga.entries, gb.entries):
            assert np.array_equal(da, db) and va == vb
    assert getattr(a, "global_node_offset", 0) == getattr(b, "global_node_offset", 0)
    assert getattr(a, "global_element_offset", 0) == getattr(b, "global_element_offset", 0)


@pytest.mark.parametrize("shape,v_z", [((3, 2, 12), lambda z, L: 5e5 * z / 4), ((2, 2, 9), -1e5)])
def test_bar_slab_equals_global_partition(shape, v_z):
    """bench.py's ranks build their slab directly (dist.bar_slab), never the whole bar: the same model,
    lumped mass and interface bit for bit as slab_partition of the global bar_model (and, with one rank,
    as the global model itself)."""
    from hakai import mesh
    nx, ny, nz = shape
    glob = mesh.bar_model(nx, ny, nz, mesh.steel_ductile(), v_z, name="B")
    gdiag, _ = glob.lumped_mass()
    one, d1, i1 = dist.bar_slab(nx, ny, nz, 0, 1, mesh.steel_ductile(), v_z, name="B")
    _same_model(one, glob)
    assert np.array_equal(d1, gdiag) and all(len(x) == 0 for x in i1)
    for world in (2, 3, 4):
        for r in range(world):
            ref = dist.slab_partition(glob, r, world, nx, ny)
            got = dist.bar_slab(nx, ny, nz, r, world, mesh.steel_ductile(), v_z, name="B")
            _same_model(got[0], ref[0])
            assert np.array_equal(got[1], ref[1])
            for x, y in zip(got[2], ref[2]):
                assert np.array_equal(x, y) and x.dtype == y.dtype


def test_partition_ranges():
    assert dist.partition_ranges(10, 3) == [(0, 4), (4, 7), (7, 10)]
    with pytest.raises(ValueError):
        dist.slab_partition(fast_deletion_bar(NX, NY, 4), 1, 3, NX, NY)


def test_range_partition_two_body():
    """General-mesh partition (contact models): contiguous element ranges, nodes renumbered in
    global order, the global lumped mass restricted, IC/BC dofs mapped, adjacent-rank sharing."""
    from hakai import mesh
    glob = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3))
    gdiag, _ = glob.lumped_mass()
    for world in (1, 2, 3):
        parts = [dist.range_partition(glob, r, world, gdiag) for r in range(world)]
        assert sum(p[0].nElement for p in parts) == glob.nElement
        ups, dns = {}, {}
        for r, (loc, diag, (ln, lo, hi), l2g, off) in enumerate(parts):
            assert off[0] == 0 and off[-1] == glob.nElement and loc.global_element_offset == off[r]
            assert np.array_equal(l2g[loc.elementmat - 1], glob.elementmat[off[r]:off[r + 1]])
            assert np.array_equal(loc.coordmat, glob.coordmat[l2g - 1])
            assert np.array_equal(diag, gdiag.reshape(-1, 3)[l2g - 1].ravel())
            assert np.all(hi == lo + 1) and np.all((lo == r) | (hi == r))
            assert np.all(np.diff(l2g[ln]) > 0)
            ups[r], dns[r] = l2g[ln[lo == r]], l2g[ln[hi == r]]
            held = set(l2g.tolist())
            gic = {(int(d), float(v)) for d, v in zip(glob.ic_dofs, glob.ic_values) if (d - 1) // 3 + 1 in held}
            lic = {(int(3 * (l2g[(d - 1) // 3] - 1) + (d - 1) % 3 + 1), float(v))
                   for d, v in zip(loc.ic_dofs, loc.ic_values)}
            assert gic == lic
            gbc = {int(d) for g in glob.bc for dd, _ in g.entries for d in dd if (d - 1) // 3 + 1 in held}
            lbc = {int(3 * (l2g[(d - 1) // 3] - 1) + (d - 1) % 3 + 1) for g in loc.bc for dd, _ in g.entries
                   for d in dd}
            assert gbc == lbc
        for r in range(world - 1):  # the two sides of a cut list the same nodes in the same order
            assert np.array_equal(ups[r], dns[r + 1])
    with pytest.raises(ValueError):  # a cut that makes ranks 0 and 2 share nodes
        dist.range_partition(mesh.two_body_model(plate=(6, 6, 2), impactor=(3, 3, 3)), 0, 3)


def test_rank_device_shares_scarce_gpus(monkeypatch):
    """One GPU per local rank when there are enough (nothing set); fewer visible GPUs than local
    ranks wrap the ranks around the devices, and only HAKAI_RCCL_SHARED_GPU=1 (a one-GPU
    rehearsal) gives each rank its own RCCL host id, so RCCL's duplicate-GPU check lets them share."""
    for k in ("NCCL_HOSTID", "NCCL_SOCKET_IFNAME", "NCCL_IB_DISABLE", "HAKAI_RCCL_SHARED_GPU"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert dist.rank_device(5, 8) == 5
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert dist.rank_device(3, 8) == 0  # e.g. per-rank HIP_VISIBLE_DEVICES: each rank's device 0
    assert "NCCL_HOSTID" not in os.environ
    monkeypatch.setenv("HAKAI_RCCL_SHARED_GPU", "1")
    assert dist.rank_device(3, 4) == 0
    h3 = os.environ["NCCL_HOSTID"]
    assert dist.rank_device(2, 4) == 0
    assert os.environ["NCCL_HOSTID"] != h3 and h3.endswith("rank3")
    assert os.environ["NCCL_SOCKET_IFNAME"] == "lo"
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    assert [dist.rank_device(r, 4) for r in range(4)] == [0, 1, 0, 1]
