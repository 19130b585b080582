"""ctypes binding of libhakai_hip.so (include/hakai_hip.h).

The library is built in-tree (``make -C hakai-fem_amd`` or ``__graft_entry__.build()``) and loaded
from ``hakai-fem_amd/lib``. There is deliberately no fallback: if the library is missing this module
raises, and every compute entry point of the library itself fails on a host without a gfx950 GPU.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_uint8, c_void_p

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# HAKAI_LIB: another build of the library (A/B timing of kernel variants, tools/variants.sh)
LIB_PATH = os.environ.get("HAKAI_LIB") or os.path.join(PKG_ROOT, "lib", "libhakai_hip.so")

HAKAI_OK = 0
HAKAI_ERR_ARG = -1
HAKAI_ERR_DEVICE = -2
HAKAI_ERR_IO = -3
HAKAI_ERR_STATE = -4
HAKAI_ERR_MODEL = -5
HAKAI_ERR_COMM = -6

K_ELEMENT, K_NODAL, K_BC, K_EXCHANGE, K_CONTACT, K_CONTACT_SUM = 0, 1, 2, 3, 4, 5
KERNEL_NAMES = {K_ELEMENT: "element", K_NODAL: "nodal", K_BC: "bc", K_EXCHANGE: "exchange", K_CONTACT: "contact",
                K_CONTACT_SUM: "contact_sum"}

PD = POINTER(c_double)
PI64 = POINTER(c_int64)
PI32 = POINTER(c_int32)


class MaterialT(ctypes.Structure):
    _fields_ = [("density", c_double), ("young", c_double), ("poisson", c_double),
                ("n_plastic", c_int32), ("plastic", PD),
                ("n_ductile", c_int32), ("ductile", PD)]


class BCT(ctypes.Structure):
    _fields_ = [("n_groups", c_int32), ("amp_n", PI32), ("amp_off", PI64), ("amp_time", PD),
                ("amp_value", PD), ("entry_off", PI64), ("entry_value", PD), ("dof_off", PI64),
                ("dofs", PI64)]


class StateT(ctypes.Structure):
    _fields_ = [("disp", PD), ("disp_pre", PD), ("velo", PD), ("Q", PD), ("integ_stress", PD),
                ("integ_strain", PD), ("integ_yield_stress", PD), ("integ_eq_plastic_strain", PD),
                ("integ_triax_stress", PD), ("element_flag", PI64), ("Qe", PD)]


class InpModelT(ctypes.Structure):
    _fields_ = [("nNode", c_int64), ("coordmat", PD), ("nElement", c_int64), ("elementmat", PI64),
                ("element_material", PI64), ("element_instance", PI64), ("nMat", c_int32),
                ("materials", POINTER(MaterialT)), ("d_time", c_double), ("end_time", c_double),
                ("mass_scaling", c_double), ("contact_flag", c_int32), ("bc", BCT),
                ("n_ic_dofs", c_int64), ("ic_dofs", PI64), ("ic_values", PD), ("n_instance", c_int32),
                ("instance_node_offset", PI64), ("instance_element_offset", PI64),
                ("instance_nElement", PI64), ("n_cp", c_int32), ("cp_instance", PI32), ("cp_elem_off", PI64),
                ("cp_elems", PI64)]


class HakaiError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hakai error {code}: {msg}")
        self.code = code


_lib = None


def lib() -> ctypes.CDLL:
    """Load libhakai_hip.so (once). Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `make -C {PKG_ROOT}` (the HIP path has no fallback)")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    sig = {
        "hakai_abi_version": (c_int, []),
        "hakai_last_error": (c_char_p, []),
        "hakai_device_count": (c_int, [POINTER(c_int)]),
        "hakai_create": (c_int, [POINTER(c_void_p), c_int]),
        "hakai_destroy": (c_int, [c_void_p]),
        "hakai_upload_model": (c_int, [c_void_p, c_int64, PD, c_int64, PI64, PI64, c_int32,
                                       POINTER(MaterialT), PD]),
        "hakai_set_bc": (c_int, [c_void_p, POINTER(BCT)]),
        "hakai_reset_state": (c_int, [c_void_p, c_int64, PI64, PD, c_double]),
        "hakai_upload_state": (c_int, [c_void_p, POINTER(StateT)]),
        "hakai_download_state": (c_int, [c_void_p, POINTER(StateT)]),
        "hakai_step": (c_int, [c_void_p, c_double, c_int64, c_double]),
        "hakai_step_group": (c_int, [POINTER(c_void_p), c_int32, c_double, c_int64, c_double]),
        "hakai_sync": (c_int, [c_void_p]),
        "hakai_deleted": (c_int, [c_void_p, PI64, PI64, c_int64]),
        "hakai_negative_jacobians": (c_int, [c_void_p, PI64]),
        "hakai_node_stress_strain": (c_int, [c_void_p, PD, PD, PD, PD, PD]),
        "hakai_stress_hexa": (c_int, [c_int, c_int64, c_int64, PD, PD, PD, PD, PD, PD, PD, PI64, PI64,
                                      c_int32, c_int32, POINTER(MaterialT), PI64, PD]),
        "hakai_triax_stress": (c_int, [c_int, c_int64, PD, PD]),
        "hakai_lumped_mass": (c_int, [c_int64, PD, c_int64, PI64, PI64, c_int32, POINTER(MaterialT),
                                      c_double, PD, PD]),
        "hakai_profile_enable": (c_int, [c_void_p, c_int]),
        "hakai_profile_read": (c_int, [c_void_p, c_int, PD, PI64]),
        "hakai_profile_mask": (c_int, [c_void_p, ctypes.c_uint32]),
        "hakai_set_tuning": (c_int, [c_void_p, c_char_p, c_int64]),
        "hakai_set_contact": (c_int, [c_void_p, c_int32, PI64]),
        "hakai_set_contact_cp": (c_int, [c_void_p, c_int32, PI64, c_int32, PI32, PI64, PI64]),
        "hakai_set_contact_global": (c_int, [c_void_p, c_int32, c_int64, PD, c_int64, PI64, PI64, PI64, PD, PI64,
                                             PI64, c_int32, PI32, PI64, PI64]),
        "hakai_set_contact_params": (c_int, [c_void_p, c_double, c_double, c_double, c_double, c_double]),
        "hakai_contact_info": (c_int, [c_void_p, POINTER(c_int32), PI64, c_int32, PD]),
        "hakai_contact_stats": (c_int, [c_void_p, PI64, c_int32]),
        "hakai_contact_force": (c_int, [c_void_p, c_double, c_double, PD]),
        "hakai_comm_unique_id": (c_int, [POINTER(c_uint8)]),
        "hakai_comm_init": (c_int, [c_void_p, c_int, c_int, POINTER(c_uint8)]),
        "hakai_comm_init_local": (c_int, [c_void_p, c_int, c_int, c_int64]),
        "hakai_set_interface": (c_int, [c_void_p, c_int64, PI64, PI32, PI32]),
        "hakai_set_element_offset": (c_int, [c_void_p, c_int64]),
        "hakai_inp_read": (c_int, [c_char_p, POINTER(POINTER(InpModelT))]),
        "hakai_inp_free": (None, [POINTER(InpModelT)]),
        "hakai_write_vtk": (c_int, [c_char_p, c_int, c_int64, PD, c_int64, PI64, PI64, PD, PD, PD, PD, PD,
                                    PD, PD]),
        "hakai_run_inp": (c_int, [c_char_p, c_char_p, c_int, c_int]),
        "hakai_graph_steps": (c_int, [c_void_p, PI64]),
        "hakai_stat": (c_int, [c_void_p, c_char_p, PI64]),
        "hakai_vtk_writer_create": (c_int, [POINTER(c_void_p), c_char_p, c_int64, PD, c_int64, PI64, c_int]),
        "hakai_vtk_writer_submit": (c_int, [c_void_p, c_int, PI64, PD, PD, PD, PD, PD, PD, PD]),
        "hakai_vtk_writer_acquire": (c_int, [c_void_p, c_void_p]),
        "hakai_vtk_writer_commit": (c_int, [c_void_p, c_int]),
        "hakai_vtk_writer_wait": (c_int, [c_void_p]),
        "hakai_vtk_writer_destroy": (None, [c_void_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def exported_symbols() -> list[str]:
    """Names the header declares (checked by the CPU test that the library exports them)."""
    return [
        "hakai_abi_version", "hakai_last_error", "hakai_device_count", "hakai_create", "hakai_destroy",
        "hakai_upload_model", "hakai_set_bc", "hakai_reset_state", "hakai_upload_state",
        "hakai_download_state", "hakai_step", "hakai_step_group", "hakai_sync", "hakai_deleted", "hakai_negative_jacobians",
        "hakai_node_stress_strain", "hakai_stress_hexa", "hakai_triax_stress", "hakai_lumped_mass",
        "hakai_profile_enable", "hakai_profile_mask", "hakai_profile_read", "hakai_set_tuning", "hakai_set_contact",
        "hakai_set_contact_cp", "hakai_set_contact_global", "hakai_set_contact_params", "hakai_contact_info", "hakai_contact_stats", "hakai_contact_force", "hakai_comm_unique_id", "hakai_comm_init",
        "hakai_comm_init_local", "hakai_set_interface", "hakai_set_element_offset", "hakai_inp_read", "hakai_inp_free", "hakai_write_vtk", "hakai_run_inp",
        "hakai_graph_steps", "hakai_stat", "hakai_vtk_writer_create", "hakai_vtk_writer_submit", "hakai_vtk_writer_acquire", "hakai_vtk_writer_commit",
        "hakai_vtk_writer_wait", "hakai_vtk_writer_destroy",
    ]


def check(code: int) -> None:
    if code != 0:
        msg = lib().hakai_last_error()
        raise HakaiError(code, msg.decode() if msg else "")


def ptr(a: np.ndarray | None, ctype=c_double):
    """Pointer to a contiguous numpy array (or NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data_as(POINTER(ctype))


def device_count() -> int:
    n = c_int(0)
    check(lib().hakai_device_count(ctypes.byref(n)))
    return n.value
