"""HAKAI model container in the reference's own layout (ModelType, v2/readInpFile_j.jl:129-150).

All index arrays are int64 and 1-based, exactly like the Julia arrays:
  coordmat (nNode, 3) C-order  == Julia 3 x nNode column-major
  elementmat (nElement, 8)     == Julia 8 x nElement column-major
Boundary conditions keep the BCType structure (groups of (dof list, value) with an optional
amplitude); the initial velocity is flattened to (dofs, values) in IC order.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _abi
from ._abi import BCT, MaterialT, check, lib, ptr


@dataclass
class Material:
    """MaterialType (v2/readInpFile_j.jl:84-96): density, elastic, *Plastic table, DUCTILE table."""
    name: str
    density: float
    young: float
    poisson: float
    plastic: np.ndarray = field(default_factory=lambda: np.zeros((0, 2)))   # (yield stress, eq. plastic strain)
    ductile: np.ndarray = field(default_factory=lambda: np.zeros((0, 3)))   # (fracture strain, triax, rate)


@dataclass
class BCGroup:
    """One *Boundary block (BCType, v2/readInpFile_j.jl:98-104)."""
    entries: list  # [(dofs int64 1-based, value float)]
    amp_time: np.ndarray | None = None
    amp_value: np.ndarray | None = None


@dataclass
class Model:
    coordmat: np.ndarray
    elementmat: np.ndarray
    element_material: np.ndarray
    materials: list
    bc: list = field(default_factory=list)
    ic_dofs: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    ic_values: np.ndarray = field(default_factory=lambda: np.zeros(0))
    d_time: float = 1e-7          # *Dynamic, Explicit increment (before mass scaling)
    end_time: float = 1e-4
    mass_scaling: float = 1.0
    contact_flag: int = 0
    element_instance: np.ndarray | None = None
    name: str = "model"
    # cal_contact_force constants (myu, kc_o, kc_s, Cr_o, Cr_s); None = the reference's
    # hard-coded (0.25, 1, 1, 0, 0) (v2/HAKAI_j.jl:2255-2259)
    contact_params: tuple | None = None
    # *Contact Pair surfaces: [((instance, elements), (instance, elements)), ...] with 1-based
    # instances and instance-local 1-based element ids; None = all-exterior contact
    contact_pairs: list | None = None

    def c_contact_pairs(self):
        """(n_cp, cp_instance int32[2n], cp_elem_off int64[2n+1], cp_elems int64[]) for the C ABI."""
        cps = self.contact_pairs or []
        inst = np.array([s[0] for cp in cps for s in cp], np.int32)
        lists = [np.asarray(s[1], np.int64) for cp in cps for s in cp]
        off = np.concatenate([[0], np.cumsum([len(x) for x in lists])]).astype(np.int64)
        els = np.concatenate(lists).astype(np.int64) if lists else np.zeros(0, np.int64)
        return len(cps), np.ascontiguousarray(inst), np.ascontiguousarray(off), np.ascontiguousarray(els)

    def __post_init__(self):
        self.coordmat = np.ascontiguousarray(self.coordmat, dtype=np.float64)
        self.elementmat = np.ascontiguousarray(self.elementmat, dtype=np.int64)
        self.element_material = np.ascontiguousarray(self.element_material, dtype=np.int64)
        self.ic_dofs = np.ascontiguousarray(self.ic_dofs, dtype=np.int64)
        self.ic_values = np.ascontiguousarray(self.ic_values, dtype=np.float64)

    @property
    def nNode(self) -> int:
        return self.coordmat.shape[0]

    @property
    def nElement(self) -> int:
        return self.elementmat.shape[0]

    @property
    def dt(self) -> float:
        """Step after mass scaling (v2/HAKAI_j.jl:114)."""
        return self.d_time * np.sqrt(self.mass_scaling)

    @property
    def time_num(self) -> float:
        return self.end_time / self.dt

    @property
    def n_steps(self) -> int:
        """Iterations of `for t = 1:time_num` (Float64 range)."""
        tn = self.time_num
        return int(np.floor(tn)) if tn >= 1 else 0

    # ---- ctypes views (keep the returned holder alive while the C side uses it) ----
    def c_materials(self):
        keep = []
        arr = (MaterialT * len(self.materials))()
        for i, m in enumerate(self.materials):
            pl = np.ascontiguousarray(m.plastic, dtype=np.float64).reshape(-1, 2)
            du = np.ascontiguousarray(m.ductile, dtype=np.float64).reshape(-1, 3)
            keep += [pl, du]
            arr[i].density, arr[i].young, arr[i].poisson = m.density, m.young, m.poisson
            arr[i].n_plastic, arr[i].plastic = pl.shape[0], ptr(pl)
            arr[i].n_ductile, arr[i].ductile = du.shape[0], ptr(du)
        return arr, keep

    def bc_arrays(self):
        amp_n, amp_off, amp_t, amp_v, entry_off, entry_val, dof_off, dofs = [], [], [], [], [], [], [], []
        for g in self.bc:
            amp_off.append(len(amp_t))
            if g.amp_time is None:
                amp_n.append(0)
            else:
                amp_n.append(len(g.amp_time))
                amp_t += list(np.asarray(g.amp_time, dtype=np.float64))
                amp_v += list(np.asarray(g.amp_value, dtype=np.float64))
            entry_off.append(len(entry_val))
            for d, v in g.entries:
                dof_off.append(len(dofs))
                entry_val.append(float(v))
                dofs += list(np.asarray(d, dtype=np.int64))
        entry_off.append(len(entry_val))
        dof_off.append(len(dofs))
        return dict(amp_n=np.array(amp_n, np.int32), amp_off=np.array(amp_off, np.int64),
                    amp_time=np.array(amp_t + [0.0], np.float64), amp_value=np.array(amp_v + [0.0], np.float64),
                    entry_off=np.array(entry_off, np.int64), entry_value=np.array(entry_val + [0.0], np.float64),
                    dof_off=np.array(dof_off, np.int64), dofs=np.array(dofs + [0], np.int64))

    def c_bc(self):
        a = self.bc_arrays()
        s = BCT()
        s.n_groups = len(self.bc)
        s.amp_n = ptr(a["amp_n"], ctypes.c_int32)
        s.amp_off = ptr(a["amp_off"], ctypes.c_int64)
        s.amp_time = ptr(a["amp_time"])
        s.amp_value = ptr(a["amp_value"])
        s.entry_off = ptr(a["entry_off"], ctypes.c_int64)
        s.entry_value = ptr(a["entry_value"])
        s.dof_off = ptr(a["dof_off"], ctypes.c_int64)
        s.dofs = ptr(a["dofs"], ctypes.c_int64)
        return s, a

    def lumped_mass(self) -> tuple[np.ndarray, np.ndarray]:
        """diag_M (3nN, per dof) and elementVolume via the library's host code (v2/HAKAI_j.jl:183-218)."""
        mats, keep = self.c_materials()
        diag = np.zeros(3 * self.nNode)
        vol = np.zeros(self.nElement)
        check(lib().hakai_lumped_mass(self.nNode, ptr(self.coordmat), self.nElement,
                                      ptr(self.elementmat, ctypes.c_int64), ptr(self.element_material, ctypes.c_int64),
                                      len(self.materials), mats, self.mass_scaling, ptr(diag), ptr(vol)))
        del keep
        return diag, vol


def _arr(p, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dtype, copy=True)


def read_inp(path: str) -> Model:
    """readInpFile (v2/readInpFile_j.jl:152) through the library's C++ reader."""
    L = lib()
    out = ctypes.POINTER(_abi.InpModelT)()
    check(L.hakai_inp_read(str(path).encode(), ctypes.byref(out)))
    try:
        m = out.contents
        nN, nE = m.nNode, m.nElement
        coord = _arr(m.coordmat, 3 * nN, np.float64).reshape(nN, 3)
        elem = _arr(m.elementmat, 8 * nE, np.int64).reshape(nE, 8)
        emat = _arr(m.element_material, nE, np.int64)
        einst = _arr(m.element_instance, nE, np.int64)
        mats = []
        for i in range(m.nMat):
            mt = m.materials[i]
            pl = _arr(mt.plastic, 2 * mt.n_plastic, np.float64).reshape(-1, 2)
            du = _arr(mt.ductile, 3 * mt.n_ductile, np.float64).reshape(-1, 3)
            mats.append(Material(f"mat{i + 1}", mt.density, mt.young, mt.poisson, pl, du))
        bc = []
        b = m.bc
        G = b.n_groups
        if G:
            entry_off = _arr(b.entry_off, G + 1, np.int64)
            n_ent = int(entry_off[-1])
            dof_off = _arr(b.dof_off, n_ent + 1, np.int64)
            dofs = _arr(b.dofs, int(dof_off[-1]), np.int64)
            vals = _arr(b.entry_value, n_ent, np.float64)
            amp_n = _arr(b.amp_n, G, np.int32)
            amp_off = _arr(b.amp_off, G, np.int64)
            n_amp = int(max([amp_off[g] + amp_n[g] for g in range(G)] + [0]))
            at = _arr(b.amp_time, n_amp, np.float64)
            av = _arr(b.amp_value, n_amp, np.float64)
            for g in range(G):
                ents = [(dofs[dof_off[j]:dof_off[j + 1]].copy(), float(vals[j]))
                        for j in range(entry_off[g], entry_off[g + 1])]
                if amp_n[g] > 0:
                    sl = slice(amp_off[g], amp_off[g] + amp_n[g])
                    bc.append(BCGroup(ents, at[sl].copy(), av[sl].copy()))
                else:
                    bc.append(BCGroup(ents))
        ic_d = _arr(m.ic_dofs, m.n_ic_dofs, np.int64)
        ic_v = _arr(m.ic_values, m.n_ic_dofs, np.float64)
        cps = None
        if m.n_cp > 0:
            inst = _arr(m.cp_instance, 2 * m.n_cp, np.int64)
            off = _arr(m.cp_elem_off, 2 * m.n_cp + 1, np.int64)
            els = _arr(m.cp_elems, int(off[-1]), np.int64)
            cps = [tuple((int(inst[2 * k + s]), els[off[2 * k + s]:off[2 * k + s + 1]].copy()) for s in range(2))
                   for k in range(m.n_cp)]
        return Model(coord, elem, emat, mats, bc, ic_d, ic_v, m.d_time, m.end_time, m.mass_scaling,
                     m.contact_flag, einst, name=str(path), contact_pairs=cps)
    finally:
        L.hakai_inp_free(out)
