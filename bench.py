#!/usr/bin/env python3
"""bench.py -- HAKAI explicit time step on MI355X: M element-updates/s (hex8, 8 Gauss points).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one full pass of the reference time-loop body (v2/HAKAI_j.jl:497-764): nodal central
difference with element-order force assembly, prescribed BCs, fused hex8 B-bar + J2 return +
internal force + triaxiality + ductile-deletion check for every active element (and, for N > 1, the
RCCL interface exchange). Inputs are resident in HBM before timing starts.

Workload (BASELINE.json): N = 1 -> C3, the 2 M-hex elastoplastic tensile bar 20x20x5000
(Tensile5e steel_Ductile, ENCASTRE at z=0, linear v_z field). N > 1 -> weak scaling, each rank owns a
2 M-hex z-slab of the C5 family bar 100x100x(200N) (uniform v_z = -1e5 mm/s into the clamped face);
N = 8 is C5 (16 M hex). Before warm-up an untimed preload advances the bar into its plastic regime
(the share of yielding Gauss points is reported).

Rank 0 prints ONE JSON line. `roofline` is for the dominant (element) kernel, from HIP events on the
library's stream; `cpu_baseline` is the oracle (CPU restatement of v0.0.2, OpenMP element loop)
timed on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_MEASURED_GBS = 6290.0      # measured float4 copy (MI355X_MICROARCH.md)
B_E_PLASTIC = 1832             # compulsory bytes per elastoplastic element
B_E_ELASTIC = 1576
B_N = 224                      # compulsory bytes per node per step (whole step)
B_N_ELEMENT_SIDE = 72          # coord, u, u_pre read by the element kernel, once per node


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--preload", type=int, default=-1, help="untimed steps before warm-up (-1: config default)")
    ap.add_argument("--layers", type=int, default=0, help="override z layers (tests / quick runs)")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--dist-path", action="store_true",
                    help="rehearsal: take the N>1 path (C5 slab, RCCL communicator) even with one rank")
    return ap.parse_args()


def build_rank_model(rank, world, layers_override=0, dist_path=False):
    """Returns (local Model, local diag_M, interface arrays or None, config dict)."""
    from hakai import mesh
    from hakai.dist import slab_partition
    if world == 1 and not dist_path:
        nz = layers_override or 5000
        m = mesh.config_c3(v_end=5e5) if nz == 5000 else mesh.bar_model(
            20, 20, nz, mesh.steel_ductile(), lambda z, L: 5e5 * z / L, name="C3")
        cfg = {"workload": "C3 synthetic elastoplastic tensile bar 20x20x%d hex8 (steel_Ductile, deletion on)" % nz,
               "elements": m.nElement, "nodes": m.nNode, "partition": "single GPU"}
        diag, _ = m.lumped_mass()
        return m, diag, None, cfg, 400
    per = layers_override or 200
    glob = mesh.config_c5(layers=per * world)
    local, diag, iface = slab_partition(glob, rank, world, nx=100, ny=100)
    cfg = {"workload": "C5 family: 100x100x%d elastoplastic impact bar, %d z-slabs of 100x100x%d (2 M hex each)"
           % (per * world, world, per), "elements": glob.nElement, "nodes": glob.nNode,
           "partition": "contiguous element ranges (z-slabs), RCCL point-to-point interface exchange"}
    return local, diag, iface, cfg, 20


def cpu_baseline(seconds, threads):
    """Oracle (CPU restatement of HAKAI v0.0.2, OpenMP element loop like @floop) on a bounded sample
    of the C3 workload: a 20x20xL slice of the same bar, same material and step."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from hakai import mesh
    threads = threads or min(16, os.cpu_count() or 1)
    m = mesh.bar_model(20, 20, 100, mesh.steel_ductile(), lambda z, L: 5e5 * z / L, name="C3-slice")
    o = O.Oracle(m, nthreads=threads)
    o.run(1, 2)  # warm
    n, t0 = 0, time.perf_counter()
    while True:
        o.run(3 + n, 5)
        n += 5
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    rate = m.nElement * n / dt
    return {"value": rate / 1e6, "unit": "M element-updates/s", "cores": threads, "kind": "port",
            "sample": f"oracle (C restatement of v0.0.2) on a 20x20x100 slice of C3 ({m.nElement} hex), "
                      f"{n} steps in {dt:.1f} s, {threads} OpenMP threads"}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if rank == 0:
            print(f"warning: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    import torch
    import torch.distributed as dist
    import hakai
    from hakai._abi import K_ELEMENT, K_EXCHANGE, K_NODAL, K_BC
    from hakai.solver import Solver, comm_unique_id
    multi = world > 1 or a.dist_path
    if multi:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29571")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    model, diag, iface, cfg, preload = build_rank_model(rank, world, a.layers, a.dist_path)
    if a.preload >= 0:
        preload = a.preload
    sv = Solver(model, device=local_rank if multi else 0, diag_M=diag)
    # stream mode throughout: graphs gain nothing at 2 M elements per step, the timed region is
    # stream mode anyway (it records events), and rocprofv3 cannot trace graph launches
    sv.set_tuning("graph", 0)
    if multi:
        uid = comm_unique_id() if rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8, device="cuda")
        dist.broadcast(t, 0)
        sv.comm_init(rank, world, bytes(t.cpu().tolist()))
        sv.set_interface(*iface)
    t = 1
    if preload:
        sv.step(t, preload)
        t += preload
    if a.warmup:
        sv.step(t, a.warmup)
        t += a.warmup
    sv.sync()

    def barrier():
        if multi:
            dist.barrier()
        torch.cuda.synchronize()

    n_active = model.nElement
    # timed region: HIP events around the element kernel only (the roofline figure), so the step
    # loop is not slowed by events around every launch
    sv.profile(True, kernels=[K_ELEMENT])
    barrier()
    t0 = time.perf_counter()
    sv.step(t, a.steps)
    sv.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if multi:
        dist.barrier()
    elapsed = t1 - t0
    t += a.steps
    el_timed = sv.profile_read(K_ELEMENT)
    # per-kernel breakdown from a short extra pass after the timed region (reported, not timed)
    sv.profile(True)
    nb = min(20, max(a.steps, 1))
    sv.step(t, nb)
    sv.sync()
    k_ms = {name: sv.profile_read(k) for k, name in ((K_ELEMENT, "element"), (K_NODAL, "nodal"), (K_BC, "bc"),
                                                        (K_EXCHANGE, "exchange"))}
    sv.profile(False)
    st = sv.download(integ_eq_plastic_strain=True, element_flag=True)
    plastic_frac = float(np.mean(st.integ_eq_plastic_strain > 0))
    n_active = int(st.element_flag.sum())
    n_deleted = model.nElement - n_active
    if multi:
        v = torch.tensor([elapsed, float(n_active)], dtype=torch.float64, device="cuda")
        mx = v.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = v.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0].item())
        n_active_total = sm[1].item()
        g = torch.tensor([plastic_frac], dtype=torch.float64, device="cuda")
        dist.all_reduce(g)
        plastic_frac = g.item() / world
    else:
        n_active_total = n_active
    # element updates: active elements x steps (metric definition)
    updates = n_active_total * a.steps
    value = updates / elapsed / 1e6
    ms_step = elapsed / a.steps * 1e3
    # roofline of the dominant kernel, from HIP events on the library's stream (rank 0)
    el_ms, el_n = el_timed
    el_avg_s = el_ms / max(el_n, 1) / 1e3
    nE_loc, nN_loc = model.nElement, model.nNode
    alg_bytes = B_E_PLASTIC * n_active + B_N_ELEMENT_SIDE * nN_loc
    achieved = alg_bytes / el_avg_s / 1e9
    whole_bytes = B_E_PLASTIC * n_active + B_N * nN_loc
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "element_pmc.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                pm = json.load(f)
            if pm.get("elements") == nE_loc:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    out = {
        "metric": "M element-updates/sec (hex8, 8 Gauss pts) at 1/2/4/8 MI355X; % HBM roofline",
        "value": round(value, 3),
        "unit": "M element-updates/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (structured hex bar, 1% node perturbation, seed 0; no reference checkpoint needed)",
        "config": dict(cfg, preload_steps=preload, plastic_gp_frac=round(plastic_frac, 4),
                       deleted_elements=int(n_deleted),
                       whole_step_roofline_frac=round(whole_bytes * a.steps / elapsed / 1e9 / HBM_PEAK_GBS, 4)
                       if world == 1 else None,
                       kernel_ms_per_step={k: round(v[0] / max(v[1], 1), 4) for k, v in k_ms.items() if v[1]},
                       parallelism=f"dp{world}" if world > 1 else "single"),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "k_element", "alg_bytes_per_launch": int(alg_bytes),
                     "avg_launch_ms": round(el_avg_s * 1e3, 4), "measured_peak_GBs": HBM_MEASURED_GBS},
        "cpu_baseline": None,
    }
    sv.close()
    if rank == 0 and world == 1 and a.cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(a.cpu_seconds, a.cpu_threads)
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if multi:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
