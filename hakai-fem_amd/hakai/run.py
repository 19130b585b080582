"""HAKAI(fname) on several GPUs: the reference's driver surface (v2/HAKAI_j.jl:81-978, called by
main() with ARGS[1], :3729-3735) with the mesh split over ranks.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m hakai.run deck.inp out_dir            # one process per GPU, RCCL over xGMI

Every rank reads the deck, computes the global lumped mass (v2/HAKAI_j.jl:183-218) and takes a
contiguous global element range (hakai.dist.range_partition); contact decks pass the global
contact model to every rank, which keeps its own share of it (hakai_set_contact_global). Each step is bit-identical to the
single-GPU run. At the output cadence (floor(time_num/100) steps, :471-480, :932-942) the ranks send
their state to rank 0, which uploads it into an output context holding the whole mesh, takes the
node averages there (cal_node_stress_strain, :3408-3486) and writes out_dir/file%03d.vtk (:3517-3717)
-- the same files, byte for byte, as the one-GPU driver (hakai.hakai / bin/hakai).

`local_ranks=N` runs the same partition as an in-process group on one device (tests).
"""
from __future__ import annotations

import ctypes
import math
import os
import sys
from dataclasses import replace

import numpy as np

from . import dist as _dist
from ._abi import check, lib, ptr
from .model import read_inp
from .solver import Solver, State, comm_unique_id, step_group

I64 = ctypes.c_int64


OUT_KEYS = ("disp", "velo", "integ_stress", "integ_strain", "integ_eq_plastic_strain", "integ_triax_stress",
            "element_flag")


def _gather_state(sv: Solver) -> dict:
    st = sv.download(disp=True, velo=True, integ_stress=True, integ_strain=True, integ_eq_plastic_strain=True,
                     integ_triax_stress=True, element_flag=True)
    return {k: getattr(st, k) for k in OUT_KEYS}


def _out_shapes(n_nodes: int, n_elem: int) -> dict:
    """Shapes and dtypes of a rank's output arrays (as Solver.download returns them)."""
    return {"disp": ((3 * n_nodes,), np.float64), "velo": ((3 * n_nodes,), np.float64),
            "integ_stress": ((8 * n_elem, 6), np.float64), "integ_strain": ((8 * n_elem, 6), np.float64),
            "integ_eq_plastic_strain": ((8 * n_elem,), np.float64),
            "integ_triax_stress": ((8 * n_elem,), np.float64), "element_flag": ((n_elem,), np.int64)}


def gather_parts(tdist, group, rank: int, world: int, part: dict, metas: list, device=None):
    """Rank 0 collects every rank's output arrays for one output step: raw point-to-point transfers
    into preallocated buffers, no pickling (gather_object pickled ~1.8 GB per rank per
    output at C5). device=None: host tensors over `group` (gloo); a CUDA device: the arrays travel
    as device tensors over the NCCL (RCCL, xGMI) group. metas[r] = (l2g, e0, n_elem) of rank r
    (exchanged once at setup). Returns [(meta, arrays)] on rank 0, None elsewhere."""
    import torch
    if rank != 0:
        for k in OUT_KEYS:
            t = torch.from_numpy(np.ascontiguousarray(part[k]))
            tdist.send(t if device is None else t.to(device), 0, group=group)
        return None
    out = [(metas[0][:2], part)]
    for r in range(1, world):
        l2g, e0, ne = metas[r]
        arrs = {}
        for k, (shape, dt) in _out_shapes(len(l2g), ne).items():
            if device is None:
                buf = np.empty(shape, dt)
                tdist.recv(torch.from_numpy(buf), r, group=group)
            else:
                t = torch.empty(shape, dtype=torch.float64 if dt == np.float64 else torch.int64, device=device)
                tdist.recv(t, r, group=group)
                buf = t.cpu().numpy()
            arrs[k] = buf
        out.append(((l2g, e0), arrs))
    return out


class _Output:
    """Rank 0's output context: the whole mesh, no contact, state uploaded at each output."""

    def __init__(self, glob, gdiag, device, out_dir):
        self.glob = glob
        self.sv = Solver(replace(glob, contact_flag=0, contact_pairs=None), device=device, diag_M=gdiag)
        self.out_dir = out_dir
        os.makedirs(out_dir, exist_ok=True)
        # files are formatted and written on the writer's threads while the ranks step on
        self.writer = None
        w = ctypes.c_void_p()
        check(lib().hakai_vtk_writer_create(ctypes.byref(w), out_dir.encode(), glob.nNode, ptr(glob.coordmat),
                                            glob.nElement, ptr(glob.elementmat, I64), 0))
        self.writer = w

    def write(self, idx, parts):
        g = self.glob
        nN, nE = g.nNode, g.nElement
        disp, velo = np.zeros(3 * nN), np.zeros(3 * nN)
        st = State.empty(nN, nE)
        st.Qe = None
        st.disp_pre = st.velo = st.Q = st.integ_yield_stress = None
        for (l2g, e0), a in parts:
            n = l2g - 1
            disp.reshape(-1, 3)[n] = a["disp"].reshape(-1, 3)  # shared nodes: identical on both ranks
            velo.reshape(-1, 3)[n] = a["velo"].reshape(-1, 3)
            ne = a["element_flag"].shape[0]
            st.integ_stress[8 * e0:8 * (e0 + ne)] = a["integ_stress"]
            st.integ_strain[8 * e0:8 * (e0 + ne)] = a["integ_strain"]
            st.integ_eq_plastic_strain[8 * e0:8 * (e0 + ne)] = a["integ_eq_plastic_strain"]
            st.integ_triax_stress[8 * e0:8 * (e0 + ne)] = a["integ_triax_stress"]
            st.element_flag[e0:e0 + ne] = a["element_flag"]
        st.disp = disp
        self.sv.upload(st)
        avg = self.sv.node_stress_strain()
        check(lib().hakai_vtk_writer_submit(self.writer, idx, ptr(st.element_flag, I64), ptr(disp), ptr(velo),
                                            ptr(avg["node_stress"]), ptr(avg["node_strain"]),
                                            ptr(avg["node_eq_plastic_strain"]), ptr(avg["node_mises_stress"]),
                                            ptr(avg["node_triax_stress"])))

    def close(self):
        if self.writer:
            try:
                check(lib().hakai_vtk_writer_wait(self.writer))
            finally:
                lib().hakai_vtk_writer_destroy(self.writer)
                self.writer = None
        self.sv.close()


def _setup_rank(glob, gdiag, rank, world, device, comm):
    loc, diag, iface, l2g, off = _dist.range_partition(glob, rank, world, gdiag)
    sv = Solver(loc, device=device, diag_M=diag)
    # the driver's element arithmetic is the reference's, operation for operation (as hakai_run_inp)
    sv.set_tuning("elem_exact", 0 if os.environ.get("HAKAI_ELEM_EXACT") == "0" else 1)
    sv.set_element_offset(loc.global_element_offset)
    comm(sv)
    sv.set_interface(*iface)
    if glob.contact_flag >= 1:
        sv.set_contact_global(glob, l2g, off, gdiag)
    return sv, (l2g, int(off[rank]))


def hakai_multi(fname: str, out_dir: str = "temp", local_ranks: int = 0, device: int = 0, verbose: bool = True):
    """HAKAI(fname) over torch.distributed's world (one process per GPU, already initialised with the
    nccl backend), or over `local_ranks` contexts of one process on `device`."""
    glob = read_inp(fname)
    gdiag, _ = glob.lumped_mass()
    dt = glob.dt
    time_num = glob.end_time / dt
    n_steps = int(math.floor(time_num)) if time_num >= 1 else 0
    d_out = int(math.floor(time_num / 100))
    if local_ranks:
        world, rank, tdist = local_ranks, 0, None
        key = abs(hash((fname, os.getpid()))) % (1 << 40)
        svs, meta = [], []
        for r in range(world):
            sv, mt = _setup_rank(glob, gdiag, r, world, device, lambda s, r=r: s.comm_init_local(r, world, key))
            svs.append(sv)
            meta.append(mt)
    else:
        import torch
        import torch.distributed as tdist
        world, rank = tdist.get_world_size(), tdist.get_rank()
        device = torch.cuda.current_device()
        obj = [comm_unique_id() if rank == 0 else None]
        tdist.broadcast_object_list(obj, src=0)
        sv, mt = _setup_rank(glob, gdiag, rank, world, device, lambda s: s.comm_init(rank, world, obj[0]))
        svs, meta = [sv], [mt]
        # output transfers: raw arrays as device tensors over the world's NCCL (RCCL) group, or host
        # tensors if the world runs gloo; the partition metadata once
        out_group = None
        out_dev = torch.device("cuda", device) if tdist.get_backend() == "nccl" else None
        metas = [None] * world if rank == 0 else None
        tdist.gather_object((mt[0], mt[1], sv.model.nElement), metas, dst=0)
    if verbose and rank == 0:
        print(f"readInpFile:{fname}\nnNode:{glob.nNode}\nnElement:{glob.nElement}\ncontact_flag:{glob.contact_flag}")
        print(f"mass_scaling:{glob.mass_scaling:g}\ntime_num:{time_num:g}\nranks:{world}")
    out = _Output(glob, gdiag, device, out_dir) if rank == 0 else None

    def output(idx):
        parts = [(mt, _gather_state(sv)) for sv, mt in zip(svs, meta)]
        if tdist is not None:
            parts = gather_parts(tdist, out_group, rank, world, parts[0][1], metas, out_dev)
        if out is not None:
            out.write(idx, parts)

    try:
        output(0)
        i_out, t0, reported = 1, 1, 0
        while t0 <= n_steps:
            t1 = n_steps if d_out <= 0 else min(n_steps, ((t0 + d_out - 1) // d_out) * d_out)
            if local_ranks:
                step_group(svs, t0, t1 - t0 + 1, dt)
            else:
                svs[0].step(t0, t1 - t0 + 1, dt)
            if verbose:
                nd = sum(len(sv.deleted()) for sv in svs)
                if tdist is not None:
                    box = [None] * world
                    tdist.all_gather_object(box, nd)
                    nd = sum(box)
                if rank == 0:
                    for q in range(reported, nd):
                        print(f"Element deleted:{glob.nElement - q - 1}/{glob.nElement}")
                    print(f"\r{t1 * dt:.4e} / {glob.end_time:.4e}     ", end="", flush=True)
                reported = nd
            if d_out > 0 and t1 % d_out == 0:
                output(i_out)
                i_out += 1
            t0 = t1 + 1
        for sv in svs:
            sv.sync()
        if verbose and rank == 0:
            print()
    finally:
        for sv in svs:
            sv.close()
        if out is not None:
            out.close()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        print("usage: python -m torch.distributed.run --nproc-per-node N -m hakai.run deck.inp [out_dir]")
        return 2
    import torch
    import torch.distributed as tdist
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = _dist.rank_device(local_rank, int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))))
    torch.cuda.set_device(device)
    tdist.init_process_group("nccl", device_id=torch.device("cuda", device))
    try:
        hakai_multi(argv[0], argv[1] if len(argv) > 1 else "temp", verbose=True)
    finally:
        tdist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
