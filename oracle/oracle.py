"""ctypes wrapper of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the
checker (or the timed CPU baseline), never as part of the product path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# HAKAI_ORACLE_VARIANT=nofma (tools/oracle_muladd_sensitivity.py only): the build whose StaticArrays
# chains round products and sums separately instead of fusing them
LIB = os.path.join(HERE, "_build", "libhakai_oracle%s.so" % (
    "_nofma" if os.environ.get("HAKAI_ORACLE_VARIANT") == "nofma" else ""))
PD, PI64 = POINTER(c_double), POINTER(c_int64)


class MatIn(ctypes.Structure):
    _fields_ = [("density", c_double), ("young", c_double), ("poisson", c_double), ("n_plastic", c_int32),
                ("plastic", PD), ("n_ductile", c_int32), ("ductile", PD)]


class BC(ctypes.Structure):
    _fields_ = [("n_groups", c_int32), ("amp_n", POINTER(c_int32)), ("amp_off", PI64), ("amp_time", PD),
                ("amp_value", PD), ("entry_off", PI64), ("entry_value", PD), ("dof_off", PI64), ("dofs", PI64)]


class View(ctypes.Structure):
    _fields_ = [("nN", c_int64), ("nE", c_int64), ("coordmat", PD), ("elementmat", PI64),
                ("element_material", PI64)]


class St(ctypes.Structure):
    _fields_ = [(n, PD) for n in ("disp", "disp_pre", "disp_new", "d_disp", "velo", "position", "Q", "Qe",
                                  "external_force", "integ_stress", "integ_strain", "integ_yield_stress",
                                  "integ_eq_plastic_strain", "integ_triax_stress", "elementVolume")] + \
               [("element_flag", PI64)]


_L = None


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB):
            raise ImportError(f"{LIB} not built: run `make -C {HERE}`")
        L = ctypes.CDLL(LIB)
        L.hko_model_create.restype = c_void_p
        L.hko_model_create.argtypes = [c_int64, PD, c_int64, PI64, PI64, c_int32, POINTER(MatIn), c_double]
        L.hko_model_destroy.argtypes = [c_void_p]
        L.hko_model_set_bc.argtypes = [c_void_p, POINTER(BC)]
        L.hko_lumped_mass.argtypes = [c_void_p, c_double, PD, PD]
        L.hko_init_yield.argtypes = [c_void_p, PD]
        L.hko_cal_stress_hexa.argtypes = [c_void_p, PD, PD, PD, PD, PD, PD, PD, PI64, PD, c_int]
        L.hko_cal_triax_stress.argtypes = [c_int64, PD, PD]
        L.hko_eigvals_sym3.argtypes = [PD, PD]
        L.hko_run.argtypes = [c_void_p, POINTER(St), PD, c_double, c_int64, c_int, PI64, c_int64, PI64]
        L.hko_node_stress_strain.argtypes = [c_int64, c_int64, PI64, PD, PD, PD, PD, PD, PD, PD, PD, PD]
        L.hko_pusai.argtypes = [PD]
        L.hko_contact_create.restype = c_void_p
        L.hko_contact_create.argtypes = [POINTER(View), c_int, PI64, PD]
        L.hko_contact_create_cp.restype = c_void_p
        L.hko_contact_create_cp.argtypes = [POINTER(View), c_int, PI64, PD, c_int32, POINTER(c_int32), PI64, PI64]
        L.hko_contact_create_ex.restype = c_void_p
        L.hko_contact_create_ex.argtypes = [POINTER(View), c_int, PI64, PD, c_int32, POINTER(c_int32), PI64, PI64,
                                            c_int]
        L.hko_contact_destroy.argtypes = [c_void_p]
        L.hko_contact_set_params.argtypes = [c_void_p, c_double, c_double, c_double, c_double, c_double]
        L.hko_contact_force.restype = c_int64
        L.hko_contact_force.argtypes = [c_void_p, PD, PD, PD, PI64, PD]
        L.hko_contact_element_deleted.argtypes = [c_void_p, PI64, c_int64]
        L.hko_contact_min_size.restype = c_double
        L.hko_contact_min_size.argtypes = [c_void_p]
        L.hko_contact_max_size.restype = c_double
        L.hko_contact_max_size.argtypes = [c_void_p]
        L.hko_contact_n_pairs.restype = c_int
        L.hko_contact_n_pairs.argtypes = [c_void_p]
        L.hko_contact_pair_info.restype = c_int64
        L.hko_contact_pair_info.argtypes = [c_void_p, c_int, PI64]
        L.hko_run_contact.argtypes = [c_void_p, POINTER(St), PD, c_double, c_int64, c_int, PI64, c_int64, PI64,
                                      c_void_p, PI64]
        _L = L
    return _L


def _p(a, t=c_double):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(POINTER(t))


class Oracle:
    """CPU restatement of the reference time loop for one Model (hakai.model.Model)."""

    def __init__(self, model, nthreads: int = 1, contact_indexed: bool = False):
        """contact_indexed: the contact setup/search through sorted face keys and a cell index
        (identical results, tests/test_contact_oracle.py; needed at BASELINE C4's 4 M hex)."""
        self.L = lib()
        self.m = model
        self.nthreads = nthreads
        self._keep = []
        mats = (MatIn * len(model.materials))()
        for i, mt in enumerate(model.materials):
            pl = np.ascontiguousarray(mt.plastic, np.float64).reshape(-1, 2)
            du = np.ascontiguousarray(mt.ductile, np.float64).reshape(-1, 3)
            self._keep += [pl, du]
            mats[i] = MatIn(mt.density, mt.young, mt.poisson, pl.shape[0], _p(pl), du.shape[0], _p(du))
        self._mats = mats
        self.h = self.L.hko_model_create(model.nNode, _p(model.coordmat), model.nElement,
                                         _p(model.elementmat, c_int64), _p(model.element_material, c_int64),
                                         len(model.materials), mats, model.dt)
        a = model.bc_arrays()
        self._bca = a
        bc = BC(len(model.bc), _p(a["amp_n"], c_int32), _p(a["amp_off"], c_int64), _p(a["amp_time"]),
                _p(a["amp_value"]), _p(a["entry_off"], c_int64), _p(a["entry_value"]), _p(a["dof_off"], c_int64),
                _p(a["dofs"], c_int64))
        rc = self.L.hko_model_set_bc(self.h, ctypes.byref(bc))
        if rc != 0:
            raise ValueError("oracle: BC rejected (reference would raise BoundsError)")
        nN, nE = model.nNode, model.nElement
        self.diag_M = np.zeros(3 * nN)
        self.vol0 = np.zeros(nE)
        self.L.hko_lumped_mass(self.h, model.mass_scaling, _p(self.diag_M), _p(self.vol0))
        z = lambda *s: np.zeros(s)  # noqa: E731
        self.s = dict(disp=z(3 * nN), disp_pre=z(3 * nN), disp_new=z(3 * nN), d_disp=z(3 * nN), velo=z(3 * nN),
                      position=model.coordmat.copy(), Q=z(3 * nN), Qe=z(nE, 24), external_force=z(3 * nN),
                      integ_stress=z(8 * nE, 6), integ_strain=z(8 * nE, 6), integ_yield_stress=z(8 * nE),
                      integ_eq_plastic_strain=z(8 * nE), integ_triax_stress=z(8 * nE),
                      elementVolume=self.vol0.copy(), element_flag=np.ones(nE, np.int64))
        self.L.hko_init_yield(self.h, _p(self.s["integ_yield_stress"]))
        dt = model.dt
        for d, v in zip(model.ic_dofs, model.ic_values):      # v2/HAKAI_j.jl:233-239
            self.s["disp_pre"][d - 1] = -v * dt
            self.s["velo"][d - 1] = v
        self.deletions = []
        self.ct = None
        if getattr(model, "contact_flag", 0) >= 1:
            inst = getattr(model, "element_instance", None)
            self._inst = np.ascontiguousarray(inst if inst is not None else np.ones(nE, np.int64), np.int64)
            self._young = np.array([mt.young for mt in model.materials], np.float64)
            self._view = View(nN, nE, _p(model.coordmat), _p(model.elementmat, c_int64),
                              _p(model.element_material, c_int64))
            ncp, cpi, cpo, cpe = model.c_contact_pairs()
            self._cp = (cpi, cpo, cpe)
            self.ct = self.L.hko_contact_create_ex(ctypes.byref(self._view), int(model.contact_flag),
                                                   _p(self._inst, c_int64), _p(self._young), ncp, _p(cpi, c_int32),
                                                   _p(cpo, c_int64), _p(cpe, c_int64), int(contact_indexed))
            cp = getattr(model, "contact_params", None)
            if cp is not None:
                self.L.hko_contact_set_params(self.ct, *[float(x) for x in cp])

    def contact_force(self):
        """cal_contact_force at the current state (position, velo, flags) -> 3nN force (standalone)."""
        f = np.zeros(3 * self.m.nNode)
        n = self.L.hko_contact_force(self.ct, _p(self.s["position"]), _p(self.s["velo"]), _p(self.diag_M),
                                     _p(self.s["element_flag"], c_int64), _p(f))
        return f, n

    def apply_deletions(self, elements):
        """Surface update for elements deleted before this oracle took over a state (1-based ids,
        in deletion order; hko_contact_element_deleted, v2/HAKAI_j.jl:766-804)."""
        for e in elements:
            self.L.hko_contact_element_deleted(self.ct, _p(self._inst, c_int64), int(e))

    def contact_pairs(self):
        out = []
        for c in range(self.L.hko_contact_n_pairs(self.ct)):
            o = np.zeros(4, np.int64)
            nj = self.L.hko_contact_pair_info(self.ct, c, _p(o, c_int64))
            out.append(dict(i_instance=int(o[0]), j_instance=int(o[1]), n_nodes_i=int(o[2]), n_triangles=int(o[3]),
                            n_nodes_j=int(nj)))
        return out

    def _st(self):
        f = {}
        for n, _ in St._fields_:
            a = self.s[n]
            f[n] = _p(a, c_int64 if a.dtype == np.int64 else c_double)
        return St(**f)

    def run(self, t_first: float, n_steps: int):
        st = self._st()
        cap = 1 << 16
        log = np.zeros(2 * cap, np.int64)
        n = c_int64(0)
        self.L.hko_run_contact(self.h, ctypes.byref(st), _p(self.diag_M), float(t_first), int(n_steps),
                               self.nthreads, _p(log, c_int64), cap, ctypes.byref(n), self.ct,
                               _p(self._inst, c_int64) if self.ct else None)
        k = min(n.value, cap)
        self.deletions += [tuple(x) for x in log[:2 * k].reshape(k, 2)]

    def node_stress_strain(self):
        m, s = self.m, self.s
        nN = m.nNode
        out = dict(node_stress=np.zeros((nN, 6)), node_strain=np.zeros((nN, 6)), node_eq_plastic_strain=np.zeros(nN),
                   node_mises_stress=np.zeros(nN), node_triax_stress=np.zeros(nN))
        self.L.hko_node_stress_strain(nN, m.nElement, _p(m.elementmat, c_int64), _p(s["integ_stress"]),
                                      _p(s["integ_strain"]), _p(s["integ_eq_plastic_strain"]),
                                      _p(s["integ_triax_stress"]), _p(out["node_stress"]), _p(out["node_strain"]),
                                      _p(out["node_eq_plastic_strain"]), _p(out["node_mises_stress"]),
                                      _p(out["node_triax_stress"]))
        return out

    def __del__(self):
        try:
            if self.ct:
                self.L.hko_contact_destroy(self.ct)
            self.L.hko_model_destroy(self.h)
        except Exception:
            pass


def pusai() -> np.ndarray:
    out = np.zeros((8, 3, 8))
    lib().hko_pusai(_p(out))
    return out


def cal_stress_hexa(oracle: Oracle, Qe, integ_stress, integ_strain, integ_yield_stress, integ_eq_plastic_strain,
                    position, d_disp, element_flag, elementVolume):
    lib().hko_cal_stress_hexa(oracle.h, _p(Qe), _p(integ_stress), _p(integ_strain), _p(integ_yield_stress),
                              _p(integ_eq_plastic_strain), _p(position), _p(d_disp), _p(element_flag, c_int64),
                              _p(elementVolume), 1)


def cal_triax_stress(integ_stress, integ_triax_stress):
    lib().hko_cal_triax_stress(integ_stress.shape[0], _p(integ_stress), _p(integ_triax_stress))


def eigvals_sym3(s6):
    s = np.ascontiguousarray(s6, np.float64)
    out = np.zeros(3)
    lib().hko_eigvals_sym3(_p(s), _p(out))
    return out
