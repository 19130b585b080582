#!/usr/bin/env python3
"""bench.py -- HAKAI explicit time step on MI355X: M element-updates/s (hex8, 8 Gauss points).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W [--strong]
    python bench.py --local-ranks R          # rehearsal of the N-rank path on one GPU

A "step" is one full pass of the reference time-loop body (v2/HAKAI_j.jl:497-764): nodal central
difference with element-order force assembly, prescribed BCs, hex8 B-bar + J2 return + internal
force + triaxiality + ductile-deletion check for every active element (and, for N > 1, the
interface exchange). Inputs are resident in HBM before timing starts.

Element arithmetic (`config.element_mode`): "fused" (default) is the single-pass kernel, which meets
the north star's 1e-6 on the bench workload (tests/test_gpu_fullsize.py, C3 windows against the
oracle) and drifts on the reference's chaotic contact decks only within those decks' own 1-ulp
sensitivity (tools/oracle_conditioning.py, profiles/r03_oracle_conditioning.jsonl); "exact" is the
reference-order kernel, whose trajectories equal the CPU restatement of the reference bit for bit
(tests/test_gpu_exact.py). The line carries the other mode too (`config.other_mode`), timed on the
same workload in the same process.

Workloads (BASELINE.json):
  N = 1 (default)  C3, the 2 M-hex elastoplastic tensile bar 20x20x5000 (Tensile5e steel_Ductile,
                   ENCASTRE at z=0, linear v_z field) -- the configuration the north star is quoted on.
  N > 1 (weak)     each rank owns one C3 bar: the 20x20x(5000N) bar in N z-slabs of 20x20x5000
                   (2 M hex each, the same velocity gradient, preload and plastic share as N = 1),
                   so value_N / (N x value_1) compares the same per-GPU work; N = 8 is 16 M hex.
                   The line also carries `config.c5_strong`: BASELINE config 5, the C5 bar
                   100x100x1600 (16 M hex) split over the same N ranks, timed in the same run, and the
                   same bar on rank 0's GPU alone right after it (`n1_reference`), so `speedup_vs_n1`
                   is a same-run ratio. Every rank builds only its own slab (hakai.dist.bar_slab);
                   `setup_s_per_rank` reports mesh + upload and the first (planning) step per rank.
                   --weak-shape c5: 2 M-hex z-slabs of the C5 bar 100x100x(200N) instead.
  --strong         the whole C5 bar 100x100x1600 (16 M hex) split over N as the headline (N = 1
                   holds all 16 M), so value_N / value_1 is the strong-scaling speed-up.
Before warm-up an untimed preload advances the bar into its plastic regime (the share of yielding
Gauss points is reported).

Rank 0 prints ONE JSON line. `roofline` is for the dominant (element) kernel, from HIP events on the
library's stream; `cpu_baseline` is the oracle (CPU restatement of v0.0.2, OpenMP element loop)
timed on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import datetime
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
C5_LAYERS = 1600               # C5: 100x100x1600


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--preload", type=int, default=-1, help="untimed steps before warm-up (-1: config default)")
    ap.add_argument("--layers", type=int, default=0, help="override z layers (tests / quick runs)")
    ap.add_argument("--element-mode", choices=("exact", "fused"), default="fused",
                    help="element arithmetic of the headline: fused single pass, or reference order (bit-exact)")
    ap.add_argument("--compare-fused", type=int, default=1,
                    help="also time the other element mode on the same workload (config.other_mode)")
    ap.add_argument("--strong", action="store_true", help="strong scaling: C5 16 M hex split over the ranks")
    ap.add_argument("--weak-shape", choices=("c3", "c5"), default="c3",
                    help="N > 1 weak scaling: a C3 bar per rank (default) or 2 M-hex slabs of the C5 bar")
    ap.add_argument("--c5-strong", type=int, default=1,
                    help="N > 1 weak: also time BASELINE config 5 (C5 16 M split over the ranks)")
    ap.add_argument("--c5-steps", type=int, default=50)
    ap.add_argument("--c5-n1-ref", type=int, default=1,
                    help="N > 1 weak: also time the whole C5 bar on rank 0's GPU alone (speedup_vs_n1 of c5_strong)")
    ap.add_argument("--local-ranks", type=int, default=0,
                    help="rehearsal: the N-rank path as an in-process group of R contexts on one GPU")
    ap.add_argument("--same-slab-ref", type=int, default=1,
                    help="N > 1 weak: also time one rank's slab alone (single_gpu_same_slab)")
    ap.add_argument("--breakdown", type=int, default=1,
                    help="per-kernel breakdown pass after the timed region (profiling scripts: 0)")
    ap.add_argument("--deletion-window", type=int, default=1,
                    help="N = 1, C3: also time steps %d-%d (both ductile deletion waves) in both element modes "
                         "(config.deletion_window); the CPU baseline then runs the oracle over that window" %
                         (7941, 7960))
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--dist-path", action="store_true",
                    help="rehearsal: take the N>1 path (C5 slab, RCCL communicator) even with one rank")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="--gpus N > 1 outside torch.distributed.run: print the N rank environments the "
                         "launcher would start (one JSON line each) and exit, touching no GPU")
    return ap.parse_args()


TERM_GRACE_S = 30.0            # launcher: SIGTERM -> SIGKILL grace period for the other ranks
LAUNCH_KEYS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n: int, port: int) -> list[dict]:
    """The environment of each of the n rank processes: rank r drives device r (hakai.dist.rank_device),
    rendezvous on 127.0.0.1 like torch.distributed.run --nnodes=1 --master-addr 127.0.0.1."""
    return [{"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
             "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)} for r in range(n)]


def launch_ranks(a) -> int:
    """`python bench.py --gpus N` (N > 1) without a launcher: start N rank processes, one per GPU, and
    wait for them. This process never touches HIP (it does not even import torch), so it may start
    children; rank 0 prints the JSON line. Any rank failing ends the others and the launch fails with
    that rank's status: a run never falls back to fewer ranks."""
    import signal
    import subprocess
    envs = rank_envs(a.gpus, free_port())
    if a.launch_dry_run:
        for e in envs:
            print(json.dumps(e), flush=True)
        return 0
    argv = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = [subprocess.Popen(argv, env=dict(os.environ, **e)) for e in envs]
    status = 0
    kill_at = None               # SIGTERM sent: ranks still alive at this time get SIGKILL
    try:
        while procs:
            for p in list(procs):
                rc = p.poll()
                if rc is None:
                    continue
                procs.remove(p)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    print(f"bench.py launcher: rank pid {p.pid} exited with {rc}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in procs:
                        q.send_signal(signal.SIGTERM)
                    kill_at = time.monotonic() + TERM_GRACE_S
            if kill_at is not None and procs and time.monotonic() > kill_at:
                # a rank stuck in the driver or in an RCCL collective may ignore SIGTERM
                print(f"bench.py launcher: {len(procs)} rank(s) still alive {TERM_GRACE_S:.0f} s after SIGTERM; "
                      "killing them", file=sys.stderr, flush=True)
                for q in procs:
                    q.kill()
                kill_at = None
            time.sleep(0.2)
    finally:
        for q in procs:          # only reached on an exception in this loop: never leave ranks behind
            q.kill()
            q.wait()
    return status


def check_launch(a, world: int, local_world: int) -> None:
    """Rank count and devices must be what --gpus asks for; every mismatch is fatal (never one rank
    timed silently). That no two ranks drive one GPU is checked after the rendezvous
    (check_distinct_devices): a visibility mask may be set per rank by the launcher or be one mask
    for all ranks, and only the ranks together can tell."""
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}: the launcher and the flag disagree")
    if world > 1 and os.environ.get("HAKAI_RCCL_SHARED_GPU") != "1":
        import torch
        if torch.cuda.device_count() < 1:  # counts devices without initialising the GPU
            raise SystemExit("bench.py: no visible GPU")


def device_identity(device: int) -> str:
    import torch
    p = torch.cuda.get_device_properties(device)
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x} {p.uuid}"


def check_distinct_devices(store, rank: int, world: int, device: int) -> None:
    """Every rank publishes the PCI address of its GPU in the rendezvous store and reads the others':
    two ranks on one GPU (e.g. one global HIP_VISIBLE_DEVICES=0 for --gpus 2) stop here with a clear
    message instead of in RCCL's duplicate-GPU check. HAKAI_RCCL_SHARED_GPU=1 (one-GPU rehearsals
    over sockets) declares the sharing deliberate."""
    me = device_identity(device)
    store.set(f"hakai_bench_dev/{rank}", me)
    ids = [store.get(f"hakai_bench_dev/{r}").decode() for r in range(world)]
    if os.environ.get("HAKAI_RCCL_SHARED_GPU") == "1":
        return
    dup = [r for r in range(world) if r != rank and ids[r] == me]
    if dup:
        raise SystemExit(f"bench.py: rank {rank} and rank(s) {dup} drive the same GPU ({me}); give each rank its "
                         "own GPU (HIP_VISIBLE_DEVICES per rank, or none), or set HAKAI_RCCL_SHARED_GPU=1 for a "
                         "one-GPU rehearsal")


def _bar_counts(nx, ny, nz):
    return nx * ny * nz, (nx + 1) * (ny + 1) * (nz + 1)


def c5_strong_model(rank, world, layers_override=0):
    """BASELINE config 5 (the C5 bar 100x100x1600, 16 M hex) split into `world` z-slabs; each rank
    builds only its own slab (dist.bar_slab, bit-identical to cutting the global bar), so no process
    ever holds the 16 M-hex host arrays unless world == 1."""
    from hakai import mesh
    from hakai.dist import bar_slab
    layers = layers_override or C5_LAYERS
    ne, nn = _bar_counts(100, 100, layers)
    cfg = {"workload": "C5 100x100x%d elastoplastic impact bar (%d hex), split into %d z-slab(s) (strong scaling)"
           % (layers, ne, world), "elements": ne, "nodes": nn,
           "partition": "contiguous element ranges (z-slabs), RCCL point-to-point interface exchange"
           if world > 1 else "single GPU"}
    local, diag, iface = bar_slab(100, 100, layers, rank, world, mesh.steel_ductile(), -1e5,
                                  name=f"C5-100x100x{layers}")
    return local, diag, (iface if world > 1 else None), cfg, 20


def build_rank_model(rank, world, layers_override=0, dist_path=False, strong=False, weak_shape="c3"):
    """Returns (local Model, local diag_M, interface arrays or None, config dict, preload).
    N > 1: every rank builds its own slab directly (dist.bar_slab), never the global bar."""
    from hakai import mesh
    from hakai.dist import bar_slab
    if strong:
        return c5_strong_model(rank, world, layers_override)
    if world == 1 and not dist_path:
        nz = layers_override or 5000
        m = mesh.config_c3(v_end=5e5) if nz == 5000 else mesh.bar_model(
            20, 20, nz, mesh.steel_ductile(), lambda z, L: 5e5 * z / L, name="C3")
        cfg = {"workload": "C3 synthetic elastoplastic tensile bar 20x20x%d hex8 (steel_Ductile, deletion on)" % nz,
               "elements": m.nElement, "nodes": m.nNode, "partition": "single GPU"}
        diag, _ = m.lumped_mass()
        return m, diag, None, cfg, 400
    if weak_shape == "c3":
        per = layers_override or 5000
        ne, nn = _bar_counts(20, 20, per * world)
        local, diag, iface = bar_slab(20, 20, per * world, rank, world, mesh.steel_ductile(),
                                      lambda z, L: 5e5 * z / per, name="C3xN")
        cfg = {"workload": "C3 per rank: 20x20x%d elastoplastic tensile bar (steel_Ductile, deletion on, v_z = "
               "5e5 z/%d mm/s), %d z-slabs of 20x20x%d (2 M hex each, the N = 1 workload)"
               % (per * world, per, world, per), "elements": ne, "nodes": nn,
               "partition": "contiguous element ranges (z-slabs), RCCL point-to-point interface exchange"}
        return local, diag, iface, cfg, 400
    per = layers_override or 200
    ne, nn = _bar_counts(100, 100, per * world)
    local, diag, iface = bar_slab(100, 100, per * world, rank, world, mesh.steel_ductile(), -1e5,
                                  name=f"C5-100x100x{per * world}")
    cfg = {"workload": "C5 family: 100x100x%d elastoplastic impact bar, %d z-slabs of 100x100x%d (2 M hex each)"
           % (per * world, world, per), "elements": ne, "nodes": nn,
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


def cpu_baseline_window(model, s0, end_exact, gpu_dels, steps, threads, report):
    """CPU baseline on the C3 workload itself: the oracle (C restatement of v0.0.2, OpenMP element
    loop) takes the GPU's hand-off state at step DEL_WINDOW_FIRST - 1 and runs the same `steps` steps
    as deletion_window -- the deletion regime, 2 M hex. Its end state is the checker of the GPU's
    reference-order run over the window: report["bitexact_vs_oracle"] (disp, disp_pre, stress,
    strain, eqps, flags, Q and the deletion log compared bit for bit)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    threads = threads or min(16, os.cpu_count() or 1)
    o = O.Oracle(model, nthreads=threads)
    s = o.s
    for k in ("disp", "disp_pre", "velo", "Q", "Qe", "integ_stress", "integ_strain", "integ_yield_stress",
              "integ_eq_plastic_strain", "integ_triax_stress", "element_flag"):
        s[k][...] = getattr(s0, k)
    s["position"][...] = model.coordmat + s0.disp.reshape(-1, 3)
    t0 = time.perf_counter()
    o.run(DEL_WINDOW_FIRST, steps)
    dt = time.perf_counter() - t0
    n_act = (int(s0.element_flag.sum()) + int(s["element_flag"].sum())) / 2
    odel = sorted((int(a), int(b)) for a, b in o.deletions)
    same = {k: bool(np.array_equal(getattr(end_exact, k), s[k]))
            for k in ("disp", "disp_pre", "integ_stress", "integ_strain", "integ_eq_plastic_strain", "element_flag", "Q")}
    report["bitexact_vs_oracle"] = bool(all(same.values()) and odel == gpu_dels)
    report["oracle_compare"] = dict(same, deletions_oracle=len(odel))
    return {"value": n_act * steps / dt / 1e6, "unit": "M element-updates/s", "cores": threads, "kind": "port",
            "sample": f"oracle (C restatement of v0.0.2, {threads} OpenMP threads) on the C3 bar itself "
                      f"({model.nElement} hex), steps {DEL_WINDOW_FIRST}-{DEL_WINDOW_FIRST + steps - 1} (both "
                      f"deletion waves) from the GPU's hand-off state: {steps} steps in {dt:.1f} s; its end state "
                      "checks the GPU's reference-order run of the same window (config.deletion_window)"}


def same_slab_rate(model, diag, exact, preload, warmup, steps):
    """One rank's slab alone on its GPU (no communicator, no interface): wall time of `steps`."""
    import torch
    from hakai.solver import Solver
    sv = Solver(model, device=torch.cuda.current_device(), diag_M=diag)
    sv.set_tuning("graph", 0)
    sv.set_tuning("elem_exact", int(exact))
    sv.step(1, preload + warmup)
    sv.sync()
    t0 = time.perf_counter()
    sv.step(1 + preload + warmup, steps)
    sv.sync()
    el = time.perf_counter() - t0
    n_act = int(sv.download(element_flag=True).element_flag.sum())
    sv.close()
    return el, n_act


class Group:
    """This process's subdomain solvers (one per rank, or R in-process ranks on one device)."""

    def __init__(self, built, ids, R, rank, world, device, exact, tag):
        import torch
        import torch.distributed as dist
        from hakai.solver import Solver, comm_unique_id
        self.R = R
        self.svs = []
        for r, (model, diag, iface, _, _) in zip(ids, built):
            sv = Solver(model, device=device, diag_M=diag)
            # stream mode throughout: graphs gain nothing at 2 M elements per step, the timed region
            # is stream mode anyway (it records events), and rocprofv3 cannot trace graph launches
            sv.set_tuning("graph", 0)
            sv.set_tuning("elem_exact", int(exact))
            if iface is not None:
                sv.set_element_offset(model.global_element_offset)
                if R:
                    sv.comm_init_local(r, R, 7117 + tag)
                else:
                    uid = comm_unique_id() if rank == 0 else bytes(128)
                    tu = torch.tensor(list(uid), dtype=torch.uint8, device="cuda")
                    dist.broadcast(tu, 0)
                    sv.comm_init(rank, world, bytes(tu.cpu().tolist()))
                sv.set_interface(*iface)
            self.svs.append(sv)

    def run(self, t_first, n):
        from hakai.solver import step_group
        if self.R:
            step_group(self.svs, t_first, n)
        else:
            self.svs[0].step(t_first, n)

    def sync(self):
        for sv in self.svs:
            sv.sync()

    def set(self, key, value):
        for sv in self.svs:
            sv.set_tuning(key, value)

    def close(self):
        for sv in self.svs:
            sv.close()
        self.svs = []


def timed(g, t, steps, multi):
    """Barrier + sync, `steps` steps, sync + barrier: (wall seconds, element-kernel (ms, launches) per solver)."""
    import torch
    import torch.distributed as dist
    from hakai._abi import K_ELEMENT, K_EXCHANGE
    for sv in g.svs:
        sv.profile(True, kernels=[K_ELEMENT, K_EXCHANGE])
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.run(t, steps)
    g.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if multi:
        dist.barrier()
    el = [sv.profile_read(K_ELEMENT) for sv in g.svs]
    ex = [sv.profile_read(K_EXCHANGE) for sv in g.svs]
    for sv in g.svs:
        sv.profile(False)
    return elapsed, el, ex


def max_over_ranks(x, multi):
    if not multi:
        return x
    import torch
    import torch.distributed as dist
    v = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    return float(v.item())


def sum_over_ranks(x, multi):
    if not multi:
        return x
    import torch
    import torch.distributed as dist
    v = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(v, op=dist.ReduceOp.SUM)
    return float(v.item())


def gather_floats(x, multi):
    """x from every rank, in rank order (the value itself on one process)."""
    if not multi:
        return [float(x)]
    import torch
    import torch.distributed as dist
    v = torch.tensor([float(x)], dtype=torch.float64, device="cuda")
    out = [torch.zeros_like(v) for _ in range(dist.get_world_size())]
    dist.all_gather(out, v)
    return [float(o.item()) for o in out]


def c5_n1_reference(rank, device, exact, steps, multi, store=None):
    """The whole C5 bar on rank 0's GPU alone (no communicator), same preload/warm-up/steps as the
    N-rank c5_strong run; the other ranks wait at a barrier. Returns the reference dict on rank 0,
    its value broadcast so every rank can form the ratio."""
    import torch
    import torch.distributed as dist
    res = torch.zeros(3, dtype=torch.float64, device="cuda")
    if rank == 0:
        t0 = time.perf_counter()
        b1 = [c5_strong_model(0, 1, 0)]
        g1 = Group(b1, [0], 0, 0, 1, device, exact, 2)
        g1.sync()
        setup = time.perf_counter() - t0
        pre = b1[0][4]
        g1.run(1, pre + 10)
        g1.sync()
        e1, el1, _ = timed(g1, pre + 11, steps, False)
        n1 = active_elements(g1)
        g1.close()
        res[0] = n1 * steps / e1 / 1e6
        res[1] = e1 / steps * 1e3
        res[2] = el1[0][0] / max(el1[0][1], 1)
        del b1
        print(f"bench.py: C5 N = 1 reference on device {device}: setup {setup:.1f} s, "
              f"{res[1].item():.3f} ms/step", file=sys.stderr, flush=True)
    if multi:
        # the other ranks wait on the host (the rendezvous store), not in a device collective: an RCCL
        # broadcast would keep a spinning kernel on every other rank's GPU for the whole reference run
        # (on a shared-GPU rehearsal, on rank 0's GPU itself)
        key = "bench_c5_n1_reference"
        if rank == 0:
            store.set(key, json.dumps([float(x) for x in res.tolist()]))
        else:
            store.wait([key], datetime.timedelta(seconds=1800))
            res = torch.tensor(json.loads(store.get(key).decode()), dtype=torch.float64)
    if res[0].item() <= 0:
        return None
    return {"value": round(res[0].item(), 3), "ms_per_step": round(res[1].item(), 4),
            "element_avg_ms": round(res[2].item(), 4),
            "source": "timed in this run: the same 16 M bar on rank 0's GPU alone, after the N-rank run"}


def active_elements(g):
    return sum(int(sv.download(element_flag=True).element_flag.sum()) for sv in g.svs)


DEL_WINDOW_FIRST = 7941        # C3 (v_end 5e5): first ductile deletion wave at step 7950, second at 7953
DEL_WINDOW_STEPS = 20          # (tests/test_gpu_fullsize.py, tools/diag_fullsize_deletion.py)
DEL_WINDOW_WARM = 100          # untimed steps per mode between the hand-off and the timed window


def deletion_window(g, t, exact, steps):
    """the deletion regime timed. The C3 bar (one context) runs on in the headline
    mode; its state is downloaded at step DEL_WINDOW_FIRST - 1 - DEL_WINDOW_WARM (the hand-off) and
    again at DEL_WINDOW_FIRST - 1 (the checker's start). Each element mode then takes the hand-off,
    runs DEL_WINDOW_WARM untimed steps and times `steps` steps across the two deletion waves with no
    gap in between: the GPU is idle while a state crosses PCIe, and the first ~20 steps after such a
    gap run up to 30 % slow (a clock/power transient: the same hand-off sequence at step 441, far from
    any deletion, shows the same hump, tools/window_control.py, profiles/r06_window_control_trace.json),
    which is not the deletion regime. Last, the reference-order kernel runs the window once more from
    the DEL_WINDOW_FIRST - 1 state (untimed): that run is what the CPU baseline leg checks against the
    oracle, bit for bit.
    Returns (report dict, checker start state, (reference-order end state, its window deletions))."""
    sv = g.svs[0]
    w0, warm = DEL_WINDOW_FIRST, DEL_WINDOW_WARM
    h0 = w0 - 1 - warm
    if t > h0 + 1:
        return None, None, None
    t_run = time.perf_counter()
    g.run(t, h0 + 1 - t)
    g.sync()
    s_h = sv.download()                 # hand-off at step h0
    g.run(h0 + 1, warm)
    g.sync()
    s0 = sv.download()                  # the checker's start, step w0 - 1
    t_run = time.perf_counter() - t_run
    out = {"first_step": w0, "steps": steps, "handoff_step": h0, "warm_steps_per_mode": warm,
           "reached_in_s": round(t_run, 2),
           "what": "C3 (2 M hex) steps %d-%d, both ductile deletion waves (7950, 7953) inside; each mode runs "
                   "steps %d-%d untimed from one hand-off state first, so the timed steps follow continuous "
                   "load (no PCIe gap)" % (w0, w0 + steps - 1, h0 + 1, w0 - 1)}
    n_start = int(s0.element_flag.sum())
    for mode_exact in (exact, not exact):
        g.set("elem_exact", int(mode_exact))
        sv.upload(s_h)
        g.run(h0 + 1, warm)             # (the first step in a mode also plans its owner assembly)
        e, el, _ = timed(g, w0, steps, False)
        dels = [(int(a), int(b)) for a, b in sv.deleted() if w0 <= a < w0 + steps]
        n_act = int(sv.download(element_flag=True).element_flag.sum())
        out["exact" if mode_exact else "fused"] = {
            "value": round((n_start + n_act) / 2 * steps / e / 1e6, 3), "unit": "M element-updates/s",
            "ms_per_step": round(e / steps * 1e3, 4),
            "element_avg_ms": round(el[0][0] / max(el[0][1], 1), 4),
            "deletions": len(dels), "deletion_steps": sorted({d[0] for d in dels}),
            "elements_active_end": n_act}
    # the checked run: reference order from the state at w0 - 1 (untimed)
    g.set("elem_exact", 1)
    sv.upload(s0)
    g.run(w0, steps)
    g.sync()
    dels_exact = sorted((int(a), int(b)) for a, b in sv.deleted() if w0 <= a < w0 + steps)
    end_exact = sv.download()
    out["checked_run"] = {"mode": "exact", "steps": [w0, w0 + steps - 1], "deletions": len(dels_exact),
                          "deletion_steps": sorted({d[0] for d in dels_exact})}
    g.set("elem_exact", int(exact))
    # what the element kernel's ductile test meets in the window: Gauss points (and waves of 8
    # elements = 64 Gauss points) at or above du_skip, where the wave-uniform skip of the deletion
    # test no longer applies (hakai_capi.cpp build_devmat: du_floor = the smallest fracture strain
    # less a relative 2^-40, du_skip = du_floor (1 - 2^-40)), at the window's start and end; and the
    # Gauss points that yielded during the window (eqps grew)
    tab = sv.model.materials[0].ductile
    if tab is not None and len(tab):
        lo, hi = float(np.min(tab[:, 0])), float(np.max(tab[:, 0]))
        du_floor = lo - (abs(hi) + abs(lo)) * 2.0 ** -40
        du_skip = du_floor - du_floor * 2.0 ** -40
        ep0, ep1 = s0.integ_eq_plastic_strain, end_exact.integ_eq_plastic_strain
        nw = ep0.size // 64
        out["ductile_test_load"] = {
            "du_skip": du_skip,
            "gp_frac_at_or_above_du_skip": [round(float(np.mean(e >= du_skip)), 6) for e in (ep0, ep1)],
            "waves_running_the_test_frac": [round(float(np.mean((e[:64 * nw].reshape(nw, 64) >= du_skip).any(axis=1))), 6)
                                            for e in (ep0, ep1)],
            "gp_frac_yielding_in_window": round(float(np.mean(ep1 > ep0)), 4),
            "eqps_max": [round(float(e.max()), 4) for e in (ep0, ep1)],
            "at": [w0 - 1, w0 + steps - 1]}
    f, x = out["fused"], out["exact"]
    out["same_deletions_both_modes"] = (f["deletions"] == x["deletions"]
                                        and f["deletion_steps"] == x["deletion_steps"])
    out["bitexact_vs_oracle"] = None      # filled by the CPU baseline leg (cpu_baseline_window)
    return out, s0, (end_exact, dels_exact)


T_START = time.perf_counter()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    if a.launch_dry_run:
        raise SystemExit("bench.py: --launch-dry-run needs --gpus N > 1 outside torch.distributed.run")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    check_launch(a, world, int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))
    import torch
    import torch.distributed as dist
    from hakai._abi import K_ELEMENT, K_EXCHANGE, K_NODAL, K_BC
    from hakai.dist import rank_device
    R = a.local_ranks if a.local_ranks > 1 else 0
    if R and world > 1:
        raise SystemExit("--local-ranks is a one-process rehearsal")
    nparts = R or world                      # subdomains of the workload
    multi = world > 1 or a.dist_path
    device = 0
    store = None
    if multi:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29571")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        # one GPU per rank; on a box with fewer GPUs than ranks (a rehearsal) the ranks share them
        device = rank_device(local_rank, int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))
        torch.cuda.set_device(device)
        store, _, _ = next(dist.rendezvous("env://", rank, world))
        check_distinct_devices(store, rank, world, device)
        dist.init_process_group("nccl", store=store, rank=rank, world_size=world,
                                device_id=torch.device("cuda", device))
    exact = a.element_mode == "exact"
    ids = list(range(R)) if R else [rank]
    t_setup = time.perf_counter()
    built = [build_rank_model(r, nparts, a.layers, a.dist_path or bool(R), a.strong, a.weak_shape) for r in ids]
    cfg = built[0][3]
    preload = built[0][4] if a.preload < 0 else a.preload
    t_mesh = time.perf_counter() - t_setup
    g = Group(built, ids, R, rank, world, device, exact, 0)
    g.sync()
    t_setup = time.perf_counter() - t_setup

    t = 1
    t_first = 0.0
    if preload >= 1:
        t_first = time.perf_counter()
        g.run(t, 1)              # the preload's first step also plans the owner-computed assembly (host)
        g.sync()
        t_first = time.perf_counter() - t_first
        t += 1
    if preload > 1:
        g.run(t, preload - 1)
        t += preload - 1
    if a.warmup:
        g.run(t, a.warmup)
        t += a.warmup
    g.sync()

    # timed region: HIP events around the element kernel (the roofline figure) and the exchange
    elapsed, el_timed, ex_timed = timed(g, t, a.steps, multi)
    t += a.steps
    n_active = active_elements(g)
    own_steps = sum(sv.stat("own_steps") for sv in g.svs)
    own_rows = sum(max(sv.stat("own_rows"), 0) for sv in g.svs)
    own_entries = sum(max(sv.stat("own_entries"), 0) for sv in g.svs)
    plastic = []
    for sv in g.svs:
        st = sv.download(integ_eq_plastic_strain=True)
        plastic.append(float(np.mean(st.integ_eq_plastic_strain > 0)))
    plastic_frac = float(np.mean(plastic))

    # the same workload with the other element arithmetic (same process, same state, re-warmed)
    other = None
    if a.compare_fused:
        g.set("elem_exact", 0 if exact else 1)
        # the mode's first step re-plans its owner assembly on the host while the GPU idles, and the
        # first ~20 steps after an idle gap run slow (clock/power transient, profiles/r06_window_control_trace.json):
        # 50 untimed steps before the timed ones
        g.run(t, 50)
        t += 50
        g.sync()
        e2, el2, _ = timed(g, t, a.steps, multi)
        t += a.steps
        n2 = active_elements(g)
        g.set("elem_exact", int(exact))
        g.run(t, 2)  # back to the headline mode for anything after this
        t += 2
        g.sync()
        e2 = max_over_ranks(e2, multi)
        n2 = sum_over_ranks(n2, multi)
        other = {"element_mode": "fused" if exact else "exact",
                 "value": round(n2 * a.steps / e2 / 1e6, 3), "unit": "M element-updates/s",
                 "ms_per_step": round(e2 / a.steps * 1e3, 4),
                 "element_avg_ms": round(sum(x[0] for x in el2) / max(el2[0][1], 1) / len(g.svs), 4),
                 "what": ("fused single-pass element kernel (rounding-level differences from the reference order; "
                          "tests/test_gpu_decks.py bounds, tools/oracle_conditioning.py)" if exact else
                          "reference-order element kernel: trajectories bit-identical to the CPU restatement "
                          "of v2/HAKAI_j.jl (tests/test_gpu_exact.py)")}

    # per-kernel times: the element kernel and the exchange from the timed region's own events; the
    # nodal and BC kernels from a short extra pass after it with events around those two only
    k_tot = {}
    for name, rec in (("element", el_timed), ("exchange", ex_timed)):
        ms, n = sum(x[0] for x in rec), sum(x[1] for x in rec)
        if n:
            k_tot[name] = [ms, n]
    if a.breakdown:
        for sv in g.svs:
            sv.profile(True, kernels=[K_NODAL, K_BC])
        nb = min(20, max(a.steps, 1))
        g.run(t, nb)
        t += nb
        g.sync()
        for sv in g.svs:
            for k, name in ((K_NODAL, "nodal"), (K_BC, "bc")):
                ms, n = sv.profile_read(k)
                if n:
                    p = k_tot.setdefault(name, [0.0, 0])
                    p[0] += ms
                    p[1] += n
            sv.profile(False)
    n_elem_local = sum(b[0].nElement for b in built)
    n_node_local = sum(b[0].nNode for b in built)
    elapsed = max_over_ranks(elapsed, multi)
    n_active_total = sum_over_ranks(n_active, multi)
    plastic_frac = sum_over_ranks(plastic_frac, multi) / (world if multi else 1)
    n_deleted = cfg["elements"] - n_active_total
    # element updates: active elements x steps (metric definition)
    updates = n_active_total * a.steps
    value = updates / elapsed / 1e6
    ms_step = elapsed / a.steps * 1e3
    # roofline of the dominant kernel, from HIP events on the library's stream (this process)
    el_ms = sum(x[0] for x in el_timed)
    el_n = max(el_timed[0][1], 1)
    el_avg_s = el_ms / el_n / 1e3 / len(g.svs)   # per subdomain launch
    alg_bytes = (B_E_PLASTIC * n_active + B_N_ELEMENT_SIDE * n_node_local) / len(g.svs)
    # with owner-computed assembly the element kernel also reads its entry lists and writes Q
    # (own_q) and the exported rows: not in §8(d)'s byte model, reported beside it
    alg_bytes_own = alg_bytes + ((24 * n_node_local + 24 * own_rows + 16 * own_entries + 4 * n_elem_local // 32)
                                 / len(g.svs) if own_steps else 0)
    achieved = alg_bytes / el_avg_s / 1e9
    whole_bytes = B_E_PLASTIC * n_active + B_N * n_node_local
    def pmc_of(mode):
        """Calibrated HBM bytes per element launch for `mode` on this workload, measured by separate
        rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/gpu_r6.sh pmc, tools/pmc_report.py):
        profiles/element_pmc.json (fused), profiles/element_pmc_exact.json (reference order). Attached
        only to the one-GPU C3 workload and the mode it was measured in."""
        f = os.path.join(ROOT, "profiles", "element_pmc.json" if mode == "fused" else "element_pmc_exact.json")
        if R or world != 1 or not cfg["workload"].startswith("C3") or not os.path.exists(f):
            return None
        try:
            with open(f) as fh:
                pm = json.load(fh)
        except Exception:
            return None
        if pm.get("elements") != n_elem_local or pm.get("element_mode", "fused") != mode:
            return None
        return pm
    pm_head = pmc_of(a.element_mode)
    traffic = pm_head.get("hbm_bytes_per_launch") if pm_head else None
    if other is not None:
        pm_other = pmc_of(other["element_mode"])
        if pm_other:
            other["traffic"] = pm_other.get("hbm_bytes_per_launch")
            other["traffic_over_algorithmic"] = round(pm_other["traffic_over_algorithmic"], 4)
            other["traffic_kernel_trace_avg_ms"] = round(pm_other["kernel_trace_avg_ms"], 4)
            other["traffic_source"] = "profiles/element_pmc_exact.json" if other["element_mode"] == "exact" \
                else "profiles/element_pmc.json"
    k_ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in k_tot.items()}
    extra = {}
    win, win_s0, win_end = None, None, None
    if (a.deletion_window and nparts == 1 and not a.strong and not multi and cfg["workload"].startswith("C3")
            and built[0][0].nElement == 2_000_000):
        try:  # after the headline's timed region: a failure here is reported, never fatal for its line
            win, win_s0, win_end = deletion_window(g, t, exact, DEL_WINDOW_STEPS)
        except Exception as e:
            win, win_s0, win_end = None, None, None
            extra["deletion_window"] = {"error": str(e)}
        if win is not None:
            extra["deletion_window"] = win
    if nparts > 1:
        ex_ms = sum(x[0] for x in ex_timed) / max(ex_timed[0][1], 1) / len(g.svs)
        extra["exchange_ms_per_step"] = round(max_over_ranks(ex_ms, multi), 4)
    g.close()
    if nparts > 1:
        extra["setup_s_per_rank"] = {"mesh_and_upload": [round(x, 2) for x in gather_floats(t_setup, multi)],
                                     "of_which_mesh": [round(x, 2) for x in gather_floats(t_mesh, multi)],
                                     "first_step_with_planning": [round(x, 2) for x in gather_floats(t_first, multi)]}
    if nparts > 1 and not a.strong and a.c5_strong:
        # BASELINE config 5: the C5 16 M bar split over the same ranks, timed in the same run
        t5s = time.perf_counter()
        b5 = [c5_strong_model(r, nparts, 0) for r in ids]
        g5 = Group(b5, ids, R, rank, world, device, exact, 1)
        g5.sync()
        t5s = time.perf_counter() - t5s
        pre5 = b5[0][4]
        t5 = 1
        g5.run(t5, pre5 + 10)
        t5 += pre5 + 10
        g5.sync()
        e5, el5, ex5 = timed(g5, t5, a.c5_steps, multi)
        n5 = sum_over_ranks(active_elements(g5), multi)
        e5 = max_over_ranks(e5, multi)
        ex5_ms = max_over_ranks(sum(x[0] for x in ex5) / max(ex5[0][1], 1) / len(g5.svs), multi)
        el5_ms = sum(x[0] for x in el5) / max(el5[0][1], 1) / len(g5.svs)
        g5.close()
        v5 = n5 * a.c5_steps / e5 / 1e6
        c5 = {"workload": b5[0][3]["workload"], "elements": b5[0][3]["elements"], "steps": a.c5_steps,
              "value": round(v5, 3), "unit": "M element-updates/s", "ms_per_step": round(e5 / a.c5_steps * 1e3, 4),
              "exchange_ms_per_step": round(ex5_ms, 4), "element_avg_ms_per_rank": round(el5_ms, 4),
              "setup_s_per_rank": [round(x, 2) for x in gather_floats(t5s, multi)],
              "n1_reference": None, "speedup_vs_n1": None}
        del b5
        if a.c5_n1_ref:
            # the same 16 M bar on ONE GPU (rank 0's), same steps, timed in this run after the N-rank
            # run: speedup_vs_n1 is a same-run, same-box ratio
            n1 = c5_n1_reference(rank, device, exact, a.c5_steps, multi, store)
            if n1 is not None:
                c5["n1_reference"] = n1
                c5["speedup_vs_n1"] = round(v5 / n1["value"], 3)
        extra["c5_strong"] = c5
    if world > 1 and not a.strong and a.same_slab_ref:
        # the same slab alone on each GPU, concurrently; the slowest rank, like the timed run
        model, diag = built[0][0], built[0][1]
        e_ref, n_ref = same_slab_rate(model, diag, exact, preload, a.warmup, a.steps)
        e_ref = max_over_ranks(e_ref, multi)
        extra["single_gpu_same_slab"] = {
            "value": round(n_ref * a.steps / e_ref / 1e6, 3), "unit": "M element-updates/s",
            "ms_per_step": round(e_ref / a.steps * 1e3, 4),
            "what": "one rank's slab alone on its GPU (no exchange), same preload/warmup/steps, slowest rank; "
                    "weak-scaling efficiency = value / (n_gpus x this)"}
    if nparts > 1:
        import resource
        rss_gb = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0 ** 2  # ru_maxrss: KiB on Linux
        extra["peak_host_rss_gb_per_rank"] = [round(x, 2) for x in gather_floats(rss_gb, multi)]
        extra["wall_s_rank_process"] = round(time.perf_counter() - T_START, 1)
    out = {
        "metric": "M element-updates/sec (hex8, 8 Gauss pts) at 1/2/4/8 MI355X; % HBM roofline",
        "value": round(value, 3),
        "unit": "M element-updates/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if a.strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (structured hex bar, 1% node perturbation, seed 0; no reference checkpoint needed)",
        "config": dict(cfg, element_mode=a.element_mode,
                       element_mode_what=("reference-order element arithmetic: trajectories bit-identical to the "
                                          "CPU restatement of v2/HAKAI_j.jl (tests/test_gpu_exact.py)" if exact else
                                          "fused single-pass element arithmetic: <=1e-6 against the oracle on this "
                                          "workload (tests/test_gpu_fullsize.py); on the reference's contact decks "
                                          "within their own 1-ulp sensitivity (profiles/r03_oracle_conditioning.jsonl)"),
                       preload_steps=preload, plastic_gp_frac=round(plastic_frac, 4),
                       deleted_elements=int(n_deleted),
                       whole_step_roofline_frac=round(whole_bytes * a.steps / elapsed / 1e9 / HBM_PEAK_GBS, 4)
                       if nparts == 1 else None,
                       kernel_ms_per_step=k_ms,
                       kernel_ms_source=("element, exchange: HIP events around those kernels inside the timed "
                                         "region (the roofline's avg_launch_ms); nodal, bc: a %d-step pass after "
                                         "it with events around those two kernels only" % min(20, max(a.steps, 1))
                                         if a.breakdown else "element, exchange: HIP events inside the timed region"),
                       other_mode=other, **extra,
                       assembly=("owner-computed node sums in LDS (own_assembly), element order" if own_steps
                                 else "fe round trip (element forces gathered by the nodal kernel)"),
                       parallelism=(f"dp{world}" if world > 1 else
                                    (f"rehearsal: {R} in-process ranks on one GPU (device-copy exchange)"
                                     if R else "single"))),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": ("static: rocprofv3 FETCH_SIZE/WRITE_SIZE passes on this kernel, mode and "
                                        "workload, calibrated (profiles/%s, round %s tree; its kernel-trace average "
                                        "%.4f ms); not measured in this run"
                                        % ("element_pmc.json" if a.element_mode == "fused" else "element_pmc_exact.json",
                                           pm_head.get("round", "?"), pm_head.get("kernel_trace_avg_ms", 0.0)))
                     if traffic else None,
                     "traffic_over_algorithmic": round(pm_head["traffic_over_algorithmic"], 4) if traffic else None,
                     "kernel": "k_element_pipe", "alg_bytes_per_launch": int(alg_bytes),
                     "alg_bytes_per_launch_with_assembly_outputs": int(alg_bytes_own),
                     "avg_launch_ms": round(el_avg_s * 1e3, 4), "measured_peak_GBs": HBM_MEASURED_GBS},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not R and not a.strong and a.cpu_baseline:
        try:
            if win is not None:
                out["cpu_baseline"] = cpu_baseline_window(built[0][0], win_s0, win_end[0], win_end[1],
                                                          DEL_WINDOW_STEPS, a.cpu_threads, win)
            else:
                out["cpu_baseline"] = cpu_baseline(a.cpu_seconds, a.cpu_threads)
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if multi:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
