"""Element partitioning for multi-GPU runs (one process per GPU).

Ranks own contiguous global element-id ranges, so the reference's serial element-order force
assembly (v2/HAKAI_j.jl:669-675) visits, at a node shared by ranks r and r+1, all of rank r's
contributions before rank r+1's. The library's interface exchange (hakai_comm.cpp) uses that to keep
the N-rank result bit-identical to one rank. Lumped mass at shared nodes is computed from the rank's
elements plus one halo layer, in global element order, so it is bit-identical to the global mass.
"""
from __future__ import annotations

import numpy as np

from . import mesh as _mesh
from .model import Model


def partition_ranges(n: int, world: int) -> list[tuple[int, int]]:
    """Split n items into `world` contiguous ranges (first ranks take the remainder)."""
    q, r = divmod(n, world)
    out, s = [], 0
    for i in range(world):
        e = s + q + (1 if i < r else 0)
        out.append((s, e))
        s = e
    return out


def range_partition(glob: Model, rank: int, world: int, glob_diag: np.ndarray | None = None):
    """Contiguous global element ranges of a general mesh (e.g. a multi-instance contact model).

    Rank r holds elements [off[r], off[r+1]) (partition_ranges) and the nodes they touch, numbered
    in ascending global id. A node may be shared by two ADJACENT ranks only (the interface protocol
    of hakai_comm.cpp); other cuts raise ValueError. The lumped mass is the global one restricted,
    so it is bit-identical to the single-GPU mass.

    Returns (local Model, local diag_M (3 nN_local), (local_node, rank_lo, rank_hi),
    local_node_global (1-based, nN_local), rank_elem_off (world+1))."""
    rng = partition_ranges(glob.nElement, world)
    off = np.array([r[0] for r in rng] + [glob.nElement], np.int64)
    e0, e1 = rng[rank]
    E = glob.elementmat - 1
    elem_rank = np.repeat(np.arange(world, dtype=np.int64), np.diff(off))
    lo = np.full(glob.nNode, world, np.int64)
    hi = np.full(glob.nNode, -1, np.int64)
    np.minimum.at(lo, E.ravel(), np.repeat(elem_rank, 8))
    np.maximum.at(hi, E.ravel(), np.repeat(elem_rank, 8))
    if np.any(hi - lo > 1):
        bad = int(np.argmax(hi - lo > 1))
        raise ValueError(f"node {bad + 1} is shared by ranks {lo[bad]} and {hi[bad]}: only adjacent ranks may "
                         "share nodes (use fewer ranks or renumber the elements)")
    mine = np.unique(E[e0:e1].ravel())
    g2l = np.full(glob.nNode, -1, np.int64)
    g2l[mine] = np.arange(mine.shape[0])
    if glob_diag is None:
        glob_diag, _ = glob.lumped_mass()
    diag = np.ascontiguousarray(np.asarray(glob_diag).reshape(-1, 3)[mine].ravel())

    def to_local_dofs(d):
        d = np.asarray(d, np.int64)
        ln = g2l[(d - 1) // 3]
        keep = ln >= 0
        return 3 * ln[keep] + (d[keep] - 1) % 3 + 1

    bc = []
    for g in glob.bc:
        ents = [(to_local_dofs(d), v) for d, v in g.entries]
        ents = [(d, v) for d, v in ents if len(d)]
        if ents:
            bc.append(type(g)(ents, g.amp_time, g.amp_value))
    ic_l = g2l[(glob.ic_dofs - 1) // 3]
    keep = ic_l >= 0
    local = Model(np.ascontiguousarray(glob.coordmat[mine]), g2l[E[e0:e1]] + 1,
                  glob.element_material[e0:e1].copy(), glob.materials, bc,
                  3 * ic_l[keep] + (glob.ic_dofs[keep] - 1) % 3 + 1, glob.ic_values[keep], glob.d_time,
                  glob.end_time, glob.mass_scaling, name=f"{glob.name}[rank {rank}/{world}]")
    shared = mine[lo[mine] != hi[mine]]
    iface = (g2l[shared], lo[shared].astype(np.int32), hi[shared].astype(np.int32))
    local.global_element_offset = int(e0)
    return local, diag, iface, (mine + 1).astype(np.int64), off


def _bar_layers(nx, ny, k0, k1, coord_global):
    """Nodes of layers k0..k1 (inclusive) and elements of layers k0..k1-1 of a structured bar,
    renumbered locally (1-based). coord_global: (nN_global, 3)."""
    npl = (nx + 1) * (ny + 1)
    coord = coord_global[k0 * npl:(k1 + 1) * npl].copy()
    nzl = k1 - k0
    iz, iy, ix = np.meshgrid(np.arange(nzl), np.arange(ny), np.arange(nx), indexing="ij")
    ix, iy, iz = ix.ravel(), iy.ravel(), iz.ravel()
    n = lambda a, b, c: _mesh.node_id(ix + a, iy + b, iz + c, nx, ny)  # noqa: E731
    elem = np.stack([n(0, 0, 0), n(1, 0, 0), n(1, 1, 0), n(0, 1, 0),
                     n(0, 0, 1), n(1, 0, 1), n(1, 1, 1), n(0, 1, 1)], axis=1).astype(np.int64)
    return np.ascontiguousarray(coord), np.ascontiguousarray(elem)


def slab_partition(glob: Model, rank: int, world: int, nx: int, ny: int):
    """Split a structured nx x ny x nz bar model (from hakai.mesh.bar_model) into z-slabs.

    Returns (local Model, local diag_M (3 nN_local), (local_node, rank_lo, rank_hi))."""
    npl = (nx + 1) * (ny + 1)
    nz = glob.nElement // (nx * ny)
    assert nz * nx * ny == glob.nElement and (nz + 1) * npl == glob.nNode, "not a structured bar"
    k0, k1 = partition_ranges(nz, world)[rank]
    if k1 - k0 < 2 and world > 1:
        raise ValueError("each slab needs >= 2 element layers (a node may be shared by two ranks only)")
    coord, elem = _bar_layers(nx, ny, k0, k1, glob.coordmat)
    # lumped mass with one halo layer each side, elements in global order
    h0, h1 = max(0, k0 - 1), min(nz, k1 + 1)
    hc, he = _bar_layers(nx, ny, h0, h1, glob.coordmat)
    mat = glob.element_material[h0 * nx * ny:h1 * nx * ny].copy()
    halo = Model(hc, he, mat, glob.materials, mass_scaling=glob.mass_scaling)
    hdiag, _ = halo.lumped_mass()
    off = (k0 - h0) * npl
    diag = np.ascontiguousarray(hdiag[3 * off:3 * (off + coord.shape[0])])
    # boundary conditions / initial velocity restricted to the local node range
    g0 = k0 * npl                      # global 0-based id of local node 0
    nloc = coord.shape[0]

    def to_local_dofs(d):
        d = np.asarray(d, np.int64)
        n0 = (d - 1) // 3
        keep = (n0 >= g0) & (n0 < g0 + nloc)
        return d[keep] - 3 * g0

    bc = []
    for g in glob.bc:
        ents = [(to_local_dofs(d), v) for d, v in g.entries]
        ents = [(d, v) for d, v in ents if len(d)]
        if ents:
            bc.append(type(g)(ents, g.amp_time, g.amp_value))
    icn = (glob.ic_dofs - 1) // 3
    keep = (icn >= g0) & (icn < g0 + nloc)
    local = Model(coord, elem, glob.element_material[k0 * nx * ny:k1 * nx * ny].copy(), glob.materials, bc,
                  glob.ic_dofs[keep] - 3 * g0, glob.ic_values[keep], glob.d_time, glob.end_time, glob.mass_scaling,
                  name=f"{glob.name}[rank {rank}/{world}]")
    # interface: bottom layer shared with rank-1, top layer with rank+1 (ascending global id)
    ln, lo, hi = [], [], []
    if rank > 0:
        ln.append(np.arange(0, npl))
        lo.append(np.full(npl, rank - 1))
        hi.append(np.full(npl, rank))
    if rank < world - 1:
        ln.append(np.arange(nloc - npl, nloc))
        lo.append(np.full(npl, rank))
        hi.append(np.full(npl, rank + 1))
    iface = (np.concatenate(ln).astype(np.int64) if ln else np.zeros(0, np.int64),
             np.concatenate(lo).astype(np.int32) if lo else np.zeros(0, np.int32),
             np.concatenate(hi).astype(np.int32) if hi else np.zeros(0, np.int32))
    local.global_node_offset = g0
    local.global_element_offset = k0 * nx * ny
    return local, diag, iface


def bar_slab(nx: int, ny: int, nz: int, rank: int, world: int, material, v_z, perturb: float = 0.01, seed: int = 0,
             d_time: float = 1e-7, n_steps: int = 1000, name: str = "bar"):
    """slab_partition(mesh.bar_model(nx, ny, nz, material, v_z, ...), rank, world, nx, ny) built
    directly: only the rank's layers (plus one halo layer each side for the lumped mass) are ever
    materialised, so a rank of a 16 M-hex bar holds 2 M hex of host arrays instead of the whole bar.
    Bit-identical to the global construction (tests/test_dist_cpu.py); world = 1 gives the whole bar.

    Returns (local Model, local diag_M (3 nN_local), (local_node, rank_lo, rank_hi))."""
    npl = (nx + 1) * (ny + 1)
    k0, k1 = partition_ranges(nz, world)[rank]
    if k1 - k0 < 2 and world > 1:
        raise ValueError("each slab needs >= 2 element layers (a node may be shared by two ranks only)")
    h0, h1 = max(0, k0 - 1), min(nz, k1 + 1)
    hc = _mesh.bar_layer_coords(nx, ny, h0, h1, perturb=perturb, seed=seed)
    _, he = _bar_layers(nx, ny, 0, h1 - h0, hc)
    mats = [material]
    halo = Model(hc, he, np.ones(he.shape[0], np.int64), mats)
    hdiag, _ = halo.lumped_mass()
    off = (k0 - h0) * npl
    nloc = (k1 - k0 + 1) * npl
    coord = np.ascontiguousarray(hc[off:off + nloc])
    _, elem = _bar_layers(nx, ny, 0, k1 - k0, coord)
    diag = np.ascontiguousarray(hdiag[3 * off:3 * (off + nloc)])
    L = float(nz)
    vz = v_z(coord[:, 2], L) if callable(v_z) else np.full(nloc, float(v_z))
    bc = [_mesh.encastre(_mesh.plane_nodes(nx, ny, 0))] if k0 == 0 else []
    local = Model(coord, elem, np.ones(elem.shape[0], np.int64), mats, bc,
                  np.arange(1, nloc + 1, dtype=np.int64) * 3, np.ascontiguousarray(vz, dtype=np.float64), d_time,
                  d_time * n_steps, name=f"{name}[rank {rank}/{world}]" if world > 1 else name)
    ln, lo, hi = [], [], []
    if rank > 0:
        ln.append(np.arange(0, npl))
        lo.append(np.full(npl, rank - 1))
        hi.append(np.full(npl, rank))
    if rank < world - 1:
        ln.append(np.arange(nloc - npl, nloc))
        lo.append(np.full(npl, rank))
        hi.append(np.full(npl, rank + 1))
    iface = (np.concatenate(ln).astype(np.int64) if ln else np.zeros(0, np.int64),
             np.concatenate(lo).astype(np.int32) if lo else np.zeros(0, np.int32),
             np.concatenate(hi).astype(np.int32) if hi else np.zeros(0, np.int32))
    local.global_node_offset = k0 * npl
    local.global_element_offset = k0 * nx * ny
    return local, diag, iface


def rank_device(local_rank: int, local_world: int) -> int:
    """The HIP device of a local rank: device = local rank on a node with a GPU per rank; with fewer
    visible GPUs than local ranks, local rank mod the visible count (e.g. one visible GPU per process
    under per-rank HIP_VISIBLE_DEVICES: device 0 of each).

    HAKAI_RCCL_SHARED_GPU=1 (tests and rehearsals only) declares that the ranks really share GPUs,
    as on the one-GPU test box: RCCL's duplicate-GPU check would refuse such a communicator, so each
    rank gets its own NCCL_HOSTID, RCCL sees separate hosts and connects them with its socket
    transport over loopback. The RCCL calls, their order, sizes and buffers are the ones an N-GPU
    node runs; only the transport and the timings differ. Never set on a production node: it would
    take xGMI out of the path. Must run before the first RCCL call of the process."""
    import os
    import socket
    import torch
    n = max(torch.cuda.device_count(), 1)  # counts devices without initialising the GPU
    if n >= local_world:
        return local_rank
    if os.environ.get("HAKAI_RCCL_SHARED_GPU") == "1":
        os.environ["NCCL_HOSTID"] = f"{socket.gethostname()}-rank{local_rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    return local_rank % n
