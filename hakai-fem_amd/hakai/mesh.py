"""Synthetic structured hex8 meshes and the benchmark configurations of BASELINE.md (C2, C3, C5).

Meshes use the reference's conventions: node ids and element connectivity are 1-based, element
node order is the C3D8 one (bottom face counter-clockwise, then top face) giving positive
Jacobians, nodes are numbered x fastest, then y, then z, and elements likewise, so a z-slab of
layers is a contiguous range of element ids and of node ids.
"""
from __future__ import annotations

import numpy as np

from .model import BCGroup, Material, Model

# Tensile5e.inp materials (HAKAI-v0.0.0/input/Tensile5e.inp), units N, mm, s, t.
STEEL_PLASTIC = np.array([[755., 0.], [809., 0.01], [829., 0.02], [842., 0.1], [895., 0.15], [922., 0.4],
                          [953., 1.], [1100., 4.]])
STEEL_DUCTILE = np.array([[1.0, 0., 30.], [0.3, 0.3, 30.]])


def steel_elastic() -> Material:
    return Material("steel_Elastic", 7.8e-09, 210000., 0.3)


def steel_ductile() -> Material:
    return Material("steel_Ductile", 7.8e-09, 210000., 0.3, STEEL_PLASTIC.copy(), STEEL_DUCTILE.copy())


def node_id(ix, iy, iz, nx, ny):
    return 1 + ix + (nx + 1) * (iy + (ny + 1) * iz)


def hex_bar(nx: int, ny: int, nz: int, h: float = 1.0, perturb: float = 0.0, seed: int = 0,
            z0: float = 0.0, x_slabs: bool = False) -> tuple[np.ndarray, np.ndarray]:
    """Structured bar of nx*ny*nz unit hexes. Returns coordmat (nN,3), elementmat (nE,8) 1-based.

    perturb: uniform random node displacement amplitude as a fraction of h (all three axes).
    x_slabs: elements numbered z fastest and x slowest (nodes keep their numbering), so contiguous
    element ranges are x-slabs instead of z-slabs."""
    xs = np.arange(nx + 1, dtype=np.float64) * h
    ys = np.arange(ny + 1, dtype=np.float64) * h
    zs = z0 + np.arange(nz + 1, dtype=np.float64) * h
    Z, Y, X = np.meshgrid(zs, ys, xs, indexing="ij")
    coord = np.stack([X.ravel(), Y.ravel(), Z.ravel()], axis=1)
    if perturb > 0:
        rng = np.random.default_rng(seed)
        coord += rng.uniform(-perturb * h, perturb * h, size=coord.shape)
    if x_slabs:
        ix, iy, iz = np.meshgrid(np.arange(nx), np.arange(ny), np.arange(nz), indexing="ij")
    else:
        iz, iy, ix = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    ix, iy, iz = ix.ravel(), iy.ravel(), iz.ravel()
    n = lambda a, b, c: node_id(ix + a, iy + b, iz + c, nx, ny)  # noqa: E731
    elem = np.stack([n(0, 0, 0), n(1, 0, 0), n(1, 1, 0), n(0, 1, 0),
                     n(0, 0, 1), n(1, 0, 1), n(1, 1, 1), n(0, 1, 1)], axis=1).astype(np.int64)
    return np.ascontiguousarray(coord), np.ascontiguousarray(elem)


def bar_layer_coords(nx: int, ny: int, k0: int, k1: int, h: float = 1.0, perturb: float = 0.0,
                     seed: int = 0) -> np.ndarray:
    """Node coordinates of layers k0..k1 (inclusive) of hex_bar(nx, ny, nz, h, perturb, seed), for any
    nz > k1, without building the whole bar: the same values bit for bit. The perturbation of node g
    is draws 3g..3g+2 of the bar's PCG64 stream (Generator.uniform takes one 64-bit output per
    double), so the stream is advanced to the first node of layer k0."""
    npl = (nx + 1) * (ny + 1)
    xs = np.arange(nx + 1, dtype=np.float64) * h
    ys = np.arange(ny + 1, dtype=np.float64) * h
    zs = np.arange(k0, k1 + 1, dtype=np.float64) * h  # hex_bar's z0 + k * h with z0 = 0, k = k0..k1
    Z, Y, X = np.meshgrid(zs, ys, xs, indexing="ij")
    coord = np.stack([X.ravel(), Y.ravel(), Z.ravel()], axis=1)
    if perturb > 0:
        bg = np.random.PCG64(seed)  # = default_rng(seed)'s bit generator
        bg.advance(3 * k0 * npl)
        coord += np.random.Generator(bg).uniform(-perturb * h, perturb * h, size=coord.shape)
    return np.ascontiguousarray(coord)


def plane_nodes(nx, ny, iz) -> np.ndarray:
    """1-based ids of the nodes of layer iz."""
    iy, ix = np.meshgrid(np.arange(ny + 1), np.arange(nx + 1), indexing="ij")
    return node_id(ix.ravel(), iy.ravel(), iz, nx, ny).astype(np.int64)


def encastre(nodes: np.ndarray) -> BCGroup:
    """*Boundary  Set, ENCASTRE (v2/readInpFile_j.jl:923-929): x dofs, then y, then z."""
    d = np.concatenate([nodes * 3 - 2, nodes * 3 - 1, nodes * 3]).astype(np.int64)
    return BCGroup([(d, 0.0)])


def bar_model(nx, ny, nz, material: Material, v_z, perturb=0.01, seed=0, d_time=1e-7, n_steps=1000,
              name="bar") -> Model:
    """Bar clamped (ENCASTRE) at z=0 with an initial z-velocity field v_z(z) (callable or constant)."""
    coord, elem = hex_bar(nx, ny, nz, perturb=perturb, seed=seed)
    L = float(nz)
    nodes_all = np.arange(1, coord.shape[0] + 1, dtype=np.int64)
    vz = v_z(coord[:, 2], L) if callable(v_z) else np.full(coord.shape[0], float(v_z))
    m = Model(coord, elem, np.ones(elem.shape[0], np.int64), [material],
              bc=[encastre(plane_nodes(nx, ny, 0))], ic_dofs=nodes_all * 3, ic_values=vz,
              d_time=d_time, end_time=d_time * n_steps, name=name)
    return m


# ---- BASELINE configurations -------------------------------------------------------------------
def config_c2(scale: int = 1) -> Model:
    """C2: 20x20x2500 elastic bar (1 M hex), v_z = 1e4 (z/L) mm/s, dt 1e-7, perturbation 1 %, seed 0."""
    return bar_model(20, 20, 2500 // scale, steel_elastic(), lambda z, L: 1e4 * z / L, name="C2")


def config_c3(scale: int = 1, v_end: float = 5e4) -> Model:
    """C3: 20x20x5000 elastoplastic (Tensile5e steel_Ductile) bar (2 M hex), v_z = 5e4 (z/L)."""
    return bar_model(20, 20, 5000 // scale, steel_ductile(), lambda z, L: v_end * z / L, name="C3")


def config_c5(layers: int = 1600, n: int = 100) -> Model:
    """C5 family: n x n x layers elastoplastic bar, uniform v_z = -1e5 mm/s into the clamped z=0 face
    (rigid-wall impact). layers = 200 per GPU gives 2 M hex per rank; 1600 layers = 16 M."""
    return bar_model(n, n, layers, steel_ductile(), -1e5, name=f"C5-{n}x{n}x{layers}")


def two_body_model(plate=(8, 8, 2), impactor=(4, 4, 4), gap=0.1, v=-1e5, material: Material | None = None,
                   perturb=0.0, seed=0, d_time=1e-7, n_steps=1000, contact_flag=1, myu=None, surfaces=False,
                   name="two_body", x_slabs=False) -> Model:
    """Two instances: a plate (instance 1) clamped on its bottom face and an impactor block
    (instance 2) above it, centred in x/y, `gap` mm away, with initial velocity v along z.
    All-exterior contact (*Contact, no *Contact Pair). myu overrides the reference's friction 0.25
    (BASELINE C4 runs frictionless: myu=0). x_slabs: elements of each body numbered x slowest, so
    range partitions cut both bodies into x-slabs and spread the contact zone over the ranks."""
    mat = material or steel_ductile()
    px, py, pz = plate
    ix, iy, iz = impactor
    if surfaces and x_slabs:
        raise ValueError("two_body_model: surfaces assume the z-slab element numbering")
    c1, e1 = hex_bar(px, py, pz, perturb=perturb, seed=seed, x_slabs=x_slabs)
    c2, e2 = hex_bar(ix, iy, iz, perturb=perturb, seed=seed + 1, z0=pz + gap, x_slabs=x_slabs)
    c2[:, 0] += (px - ix) / 2.0
    c2[:, 1] += (py - iy) / 2.0
    n1 = c1.shape[0]
    coord = np.concatenate([c1, c2])
    elem = np.concatenate([e1, e2 + n1])
    inst = np.concatenate([np.ones(e1.shape[0], np.int64), np.full(e2.shape[0], 2, np.int64)])
    imp_nodes = np.arange(n1 + 1, coord.shape[0] + 1, dtype=np.int64)
    params = None if myu is None else (float(myu), 1.0, 1.0, 0.0, 0.0)
    cps = None
    if surfaces:  # *Contact Pair: plate top element layer vs impactor bottom element layer
        top = np.arange((pz - 1) * px * py + 1, pz * px * py + 1, dtype=np.int64)
        bottom = np.arange(1, ix * iy + 1, dtype=np.int64)
        cps = [((1, top), (2, bottom))]
    return Model(coord, elem, np.ones(elem.shape[0], np.int64), [mat], bc=[encastre(plane_nodes(px, py, 0))],
                 ic_dofs=imp_nodes * 3, ic_values=np.full(imp_nodes.shape[0], float(v)), d_time=d_time,
                 end_time=d_time * n_steps, contact_flag=contact_flag, element_instance=inst, name=name,
                 contact_params=params, contact_pairs=cps)


def config_c4(scale: int = 1, x_slabs: bool = False) -> Model:
    """C4: plate 200x200x50 + impactor 100x100x200 (2 M hex each), gap 0.1 mm, impactor
    v = -1e5 mm/s, elastoplastic steel, all-exterior contact, frictionless (myu = 0).
    scale > 1 divides every edge count (tests). x_slabs: the same model with its elements numbered
    x slowest (range partitions then cut x-slabs, each holding part of the contact zone)."""
    return two_body_model((200 // scale, 200 // scale, 50 // scale), (100 // scale, 100 // scale, 200 // scale),
                          gap=0.1, v=-1e5, myu=0.0, name="C4" + (" (x-slab numbering)" if x_slabs else ""),
                          x_slabs=x_slabs)


def tensile5e_model() -> Model:
    """The Tensile5e.inp deck (HAKAI-v0.0.0/input/Tensile5e.inp) rebuilt in code: 5 hex, 24 nodes,
    ENCASTRE on Set-2, y-displacement 10*amp on Set-3. Used when the .inp file is not at hand
    (the GPU box has no /root/reference); tests check it equals read_inp() of the real deck."""
    pts = []
    for x in (-5., 5.):
        for z in (5., 0.):
            for y in (-25., -15., -5., 5., 15., 25.):
                pts.append((x, y, z))
    coord = np.array(pts)
    elem = np.array([[13, 14, 20, 19, 1, 2, 8, 7], [14, 15, 21, 20, 2, 3, 9, 8], [15, 16, 22, 21, 3, 4, 10, 9],
                     [16, 17, 23, 22, 4, 5, 11, 10], [17, 18, 24, 23, 5, 6, 12, 11]], np.int64)
    set2 = np.arange(1, 20, 6, dtype=np.int64)
    set3 = np.arange(6, 25, 6, dtype=np.int64)
    bc = [encastre(set2),
          BCGroup([(set3 * 3 - 2, 0.0), (set3 * 3 - 1, 10.0), (set3 * 3, 0.0)],
                  np.array([0., 0.01]), np.array([0., 1.]))]
    mats = [steel_elastic(),
            Material("steel_Elastoplast", 7.8e-09, 210000., 0.3, STEEL_PLASTIC.copy()),
            steel_ductile()]
    return Model(coord, elem, np.full(5, 3, np.int64), mats, bc, d_time=5.0e-07, end_time=0.01,
                 name="Tensile5e")
