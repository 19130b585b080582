"""Host-side mirror of HAKAI's solver interface over the MI355X C ABI.

* ``Solver``             -- the persistent device context: hakai()'s state (v2/HAKAI_j.jl:81-480)
                            and its time loop (:487-951) as ``step(t_first, n)``.
* ``cal_stress_hexa``    -- same name, arguments and in-place semantics as the reference
                            (v2/HAKAI_j.jl:1033), executed by the gfx950 element kernel.
* ``cal_triax_stress``   -- v2/HAKAI_j.jl:982.
* ``hakai``              -- HAKAI(fname): .inp -> out_dir/file%03d.vtk (v2/HAKAI_j.jl:81).
Every call goes to libhakai_hip.so; there is no Python or CPU compute path.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._abi import StateT, check, lib, ptr
from .model import Model

I64 = ctypes.c_int64


@dataclass
class State:
    """Reference-layout state arrays (v2/HAKAI_j.jl:225-230, :430-456)."""
    disp: np.ndarray
    disp_pre: np.ndarray
    velo: np.ndarray
    Q: np.ndarray
    integ_stress: np.ndarray            # (8nE, 6)  == Julia 6 x 8nE
    integ_strain: np.ndarray
    integ_yield_stress: np.ndarray      # (8nE,)
    integ_eq_plastic_strain: np.ndarray
    integ_triax_stress: np.ndarray
    element_flag: np.ndarray            # (nE,) int64
    Qe: np.ndarray | None = None        # (nE, 24) element internal forces of the last step

    @staticmethod
    def empty(nN: int, nE: int) -> "State":
        f = lambda *s: np.zeros(s)  # noqa: E731
        return State(f(3 * nN), f(3 * nN), f(3 * nN), f(3 * nN), f(8 * nE, 6), f(8 * nE, 6), f(8 * nE),
                     f(8 * nE), f(8 * nE), np.ones(nE, np.int64), f(nE, 24))

    def c(self) -> StateT:
        s = StateT()
        for name, _ in StateT._fields_:
            a = getattr(self, name)
            if a is not None:
                setattr(s, name, ptr(a, ctypes.c_int64 if a.dtype == np.int64 else ctypes.c_double))
        return s


class Solver:
    """Persistent device context holding one (rank-local) model."""

    def __init__(self, model: Model, device: int = 0, diag_M: np.ndarray | None = None):
        self.L = lib()
        self.model = model
        self.ctx = ctypes.c_void_p()
        check(self.L.hakai_create(ctypes.byref(self.ctx), device))
        if diag_M is None:
            diag_M, _ = model.lumped_mass()
        self.diag_M = np.ascontiguousarray(diag_M, dtype=np.float64)
        mats, keep = model.c_materials()
        check(self.L.hakai_upload_model(self.ctx, model.nNode, ptr(model.coordmat), model.nElement,
                                        ptr(model.elementmat, I64), ptr(model.element_material, I64),
                                        len(model.materials), mats, ptr(self.diag_M)))
        del keep
        bc, keep = model.c_bc()
        check(self.L.hakai_set_bc(self.ctx, ctypes.byref(bc)))
        del keep
        if getattr(model, "contact_flag", 0) >= 1:
            inst = model.element_instance
            inst = np.ones(model.nElement, np.int64) if inst is None else np.ascontiguousarray(inst, np.int64)
            ncp, cpi, cpo, cpe = model.c_contact_pairs()
            check(self.L.hakai_set_contact_cp(self.ctx, int(model.contact_flag), ptr(inst, I64), ncp,
                                              ptr(cpi, ctypes.c_int32), ptr(cpo, I64), ptr(cpe, I64)))
            if getattr(model, "contact_params", None) is not None:
                check(self.L.hakai_set_contact_params(self.ctx, *[float(x) for x in model.contact_params]))
        self.reset()

    # -- lifecycle ---------------------------------------------------------------------------
    def close(self):
        if self.ctx:
            self.L.hakai_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- state ---------------------------------------------------------------------------------
    def reset(self):
        """Fresh state with the model's initial velocity (v2/HAKAI_j.jl:225-239, :430-465)."""
        m = self.model
        check(self.L.hakai_reset_state(self.ctx, len(m.ic_dofs), ptr(m.ic_dofs, I64), ptr(m.ic_values), m.dt))

    def upload(self, st: State):
        s = st.c()
        check(self.L.hakai_upload_state(self.ctx, ctypes.byref(s)))

    def download(self, st: State | None = None, **only) -> State:
        """Copy the device state back in the reference layout. only=dict(name=True) limits arrays."""
        m = self.model
        if st is None:
            st = State.empty(m.nNode, m.nElement)
        s = st.c()
        if only:
            for name, _ in StateT._fields_:
                if not only.get(name, False):
                    setattr(s, name, None)
        check(self.L.hakai_download_state(self.ctx, ctypes.byref(s)))
        return st

    # -- time loop -------------------------------------------------------------------------------
    def step(self, t_first: float, n_steps: int, d_time: float | None = None):
        check(self.L.hakai_step(self.ctx, float(t_first), int(n_steps),
                                float(self.model.dt if d_time is None else d_time)))

    def sync(self):
        check(self.L.hakai_sync(self.ctx))

    def deleted(self, cap: int = 1 << 16) -> np.ndarray:
        """(step, element 1-based) pairs of the deletions so far, in (step, element) order."""
        n = I64(0)
        log = np.zeros(2 * cap, np.int64)
        check(self.L.hakai_deleted(self.ctx, ctypes.byref(n), ptr(log, I64), cap))
        k = min(n.value, cap)
        return log[:2 * k].reshape(k, 2)

    def negative_jacobians(self) -> int:
        n = I64(0)
        check(self.L.hakai_negative_jacobians(self.ctx, ctypes.byref(n)))
        return n.value

    def node_stress_strain(self):
        nN = self.model.nNode
        ns, nn = np.zeros((nN, 6)), np.zeros((nN, 6))
        ne, nm, nt = np.zeros(nN), np.zeros(nN), np.zeros(nN)
        check(self.L.hakai_node_stress_strain(self.ctx, ptr(ns), ptr(nn), ptr(ne), ptr(nm), ptr(nt)))
        return dict(node_stress=ns, node_strain=nn, node_eq_plastic_strain=ne, node_mises_stress=nm,
                    node_triax_stress=nt)

    # -- contact ----------------------------------------------------------------------------------
    def contact_stats(self) -> dict:
        """Counters of the last contact step (hakai_contact_stats)."""
        st = np.zeros(12, np.int64)
        check(self.L.hakai_contact_stats(self.ctx, ptr(st, I64), 12))
        keys = ("events", "max_events", "candidate_triangles", "touched_nodes", "live_triangles", "live_nodes_i",
                "live_nodes_j", "binned_contact_nodes", "exchange_bytes_per_rank", "hash_buckets",
                "tested_triangles", "exchange_record_bytes_per_rank")
        return {k: int(v) for k, v in zip(keys, st)}

    def contact_info(self):
        """Pairs [(i_instance, j_instance, n_nodes_i, n_triangles, n_nodes_j)], (min, max) element size."""
        n = ctypes.c_int32(0)
        info = np.zeros(5 * 4096, np.int64)
        sizes = np.zeros(2)
        check(self.L.hakai_contact_info(self.ctx, ctypes.byref(n), ptr(info, I64), 4096, ptr(sizes)))
        return [tuple(int(x) for x in info[5 * p:5 * p + 5]) for p in range(n.value)], tuple(sizes)

    def contact_force(self, t: float, d_time: float | None = None) -> np.ndarray:
        """cal_contact_force at the current device state (external_force of step t), 3nN."""
        f = np.zeros(3 * self.model.nNode)
        check(self.L.hakai_contact_force(self.ctx, float(t), float(self.model.dt if d_time is None else d_time),
                                         ptr(f)))
        return f

    # -- profiling (HIP events on the context's own stream) ------------------------------------
    def profile(self, on: bool = True, kernels=None):
        """Time kernels with HIP events on the context's stream (all, or the HAKAI_K_* ids given)."""
        if kernels is None:
            check(self.L.hakai_profile_enable(self.ctx, int(on)))
        else:
            check(self.L.hakai_profile_mask(self.ctx, sum(1 << k for k in kernels) if on else 0))

    def profile_read(self, kernel: int) -> tuple[float, int]:
        ms, n = ctypes.c_double(0), I64(0)
        check(self.L.hakai_profile_read(self.ctx, kernel, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def set_tuning(self, key: str, value: int):
        check(self.L.hakai_set_tuning(self.ctx, key.encode(), int(value)))

    def stat(self, key: str) -> int:
        """Step-loop counter (hakai_stat): graph_steps, own_steps, own_rows, own_entries, own_superbatch, own_slots."""
        n = I64(0)
        check(self.L.hakai_stat(self.ctx, key.encode(), ctypes.byref(n)))
        return n.value

    def graph_steps(self) -> int:
        """Steps run from captured hipGraphs so far (hakai_graph_steps)."""
        n = I64(0)
        check(self.L.hakai_graph_steps(self.ctx, ctypes.byref(n)))
        return n.value

    # -- multi-GPU ---------------------------------------------------------------------------------
    def comm_init(self, rank: int, nranks: int, uid: bytes):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(self.L.hakai_comm_init(self.ctx, rank, nranks, buf))

    def comm_init_local(self, rank: int, nranks: int, group_key: int):
        """Join an in-process group (same device); step the group with ``step_group``."""
        check(self.L.hakai_comm_init_local(self.ctx, rank, nranks, int(group_key)))

    def set_element_offset(self, offset: int):
        check(self.L.hakai_set_element_offset(self.ctx, int(offset)))

    def set_contact_global(self, glob: Model, local_node_global: np.ndarray, rank_elem_off: np.ndarray,
                           glob_diag_M: np.ndarray | None = None):
        """Multi-GPU contact (hakai_set_contact_global): this rank sets up the contact model of the
        global mesh `glob` (its contact_flag, instances, *Contact Pair surfaces and constants) and
        searches the entries of its own elements and nodes.
        Call after comm_init[_local], set_element_offset and set_interface."""
        if glob_diag_M is None:
            glob_diag_M, _ = glob.lumped_mass()
        diag = np.ascontiguousarray(glob_diag_M, np.float64)
        inst = glob.element_instance
        inst = np.ones(glob.nElement, np.int64) if inst is None else np.ascontiguousarray(inst, np.int64)
        ncp, cpi, cpo, cpe = glob.c_contact_pairs()
        l2g = np.ascontiguousarray(local_node_global, np.int64)
        off = np.ascontiguousarray(rank_elem_off, np.int64)
        check(self.L.hakai_set_contact_global(self.ctx, int(glob.contact_flag), glob.nNode, ptr(glob.coordmat),
                                              glob.nElement, ptr(glob.elementmat, I64),
                                              ptr(glob.element_material, I64), ptr(inst, I64), ptr(diag),
                                              ptr(l2g, I64), ptr(off, I64), ncp, ptr(cpi, ctypes.c_int32),
                                              ptr(cpo, I64), ptr(cpe, I64)))
        if glob.contact_flag >= 1 and getattr(glob, "contact_params", None) is not None:
            check(self.L.hakai_set_contact_params(self.ctx, *[float(x) for x in glob.contact_params]))

    def set_interface(self, local_node: np.ndarray, rank_lo: np.ndarray, rank_hi: np.ndarray):
        ln = np.ascontiguousarray(local_node, np.int64)
        lo = np.ascontiguousarray(rank_lo, np.int32)
        hi = np.ascontiguousarray(rank_hi, np.int32)
        check(self.L.hakai_set_interface(self.ctx, len(ln), ptr(ln, I64), ptr(lo, ctypes.c_int32),
                                         ptr(hi, ctypes.c_int32)))


def step_group(solvers: list[Solver], t_first: float, n_steps: int, d_time: float | None = None):
    """Advance an in-process group (hakai_comm_init_local, solvers[r] = rank r) in lockstep
    (hakai_step_group): per step every rank's contact search, then every rank's exchange and update."""
    if not solvers:
        return
    arr = (ctypes.c_void_p * len(solvers))(*[sv.ctx for sv in solvers])
    dt = solvers[0].model.dt if d_time is None else d_time
    check(lib().hakai_step_group(arr, len(solvers), float(t_first), int(n_steps), float(dt)))


def comm_unique_id() -> bytes:
    buf = (ctypes.c_uint8 * 128)()
    check(lib().hakai_comm_unique_id(buf))
    return bytes(buf)


# ---- literal mirrors of the reference functions ---------------------------------------------------
def cal_stress_hexa(Qe, integ_stress, integ_strain, integ_yield_stress, integ_eq_plastic_strain, position,
                    d_disp, elementmat, element_flag, integ_num, Pusai_mat, MATERIAL, element_material,
                    elementMinSize, elementVolume, device: int = 0):
    """cal_stress_hexa (v2/HAKAI_j.jl:1033-1036), arrays in the reference's layout, mutated in place:
    Qe (nE,24) accumulates; integ_* (8nE,6)/(8nE,); position (nN,3); d_disp (3nN,);
    elementmat (nE,8) 1-based; MATERIAL a list of model.Material. Pusai_mat and elementMinSize are
    accepted for signature parity and not needed (the kernel builds Pusai in registers)."""
    from .model import Model
    tmp = Model(position, elementmat, element_material, MATERIAL)
    mats, keep = tmp.c_materials()
    nN, nE = position.shape[0], elementmat.shape[0]
    check(lib().hakai_stress_hexa(device, nN, nE, ptr(Qe), ptr(integ_stress), ptr(integ_strain),
                                  ptr(integ_yield_stress), ptr(integ_eq_plastic_strain),
                                  ptr(np.ascontiguousarray(position, np.float64)),
                                  ptr(np.ascontiguousarray(d_disp, np.float64)),
                                  ptr(tmp.elementmat, I64), ptr(np.ascontiguousarray(element_flag, np.int64), I64),
                                  int(integ_num), len(MATERIAL), mats, ptr(tmp.element_material, I64),
                                  ptr(elementVolume)))
    del keep


def cal_triax_stress(integ_stress, integ_triax_stress, device: int = 0):
    """cal_triax_stress (v2/HAKAI_j.jl:982), in place."""
    st = np.ascontiguousarray(integ_stress, np.float64)
    check(lib().hakai_triax_stress(device, st.shape[0], ptr(st), ptr(integ_triax_stress)))


def hakai(fname: str, out_dir: str = "temp", device: int = 0, verbose: bool = True):
    """HAKAI(fname) (v2/HAKAI_j.jl:81): run the deck on the GPU and write out_dir/file%03d.vtk."""
    check(lib().hakai_run_inp(str(fname).encode(), str(out_dir).encode(), device, int(verbose)))
