#!/usr/bin/env python3
"""RCCL check of the multi-GPU contact path (hakai_set_contact_global over hakai_comm_init): 2 ranks
(both on device 0 when only one GPU is visible and HAKAI_RCCL_SHARED_GPU=1: hakai.dist.rank_device
makes them separate hosts to RCCL, which then runs its socket transport over loopback), a range-partitioned two-body impact with contact
deletions and the owner-computed search (per step: deletions and binned contact-zone nodes
all-gathered, pair boxes all-reduced, events all-gathered), compared bit for bit with a
single-context run -- once with small exchange capacities, so blocks grow and steps run again.
Launch:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \\
      --master-port 29534 tools/rccl_contact_check.py
Rendezvous and the unique-id broadcast use gloo."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hakai-fem_amd"), os.path.join(ROOT, "tests")]


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    from hakai import dist as hdist
    from hakai import mesh
    from hakai.solver import Solver, comm_unique_id

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = hdist.rank_device(int(os.environ.get("LOCAL_RANK", rank)), int(os.environ.get("LOCAL_WORLD_SIZE", world)))
    dist.init_process_group("gloo")
    glob = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400)
    gdiag, _ = glob.lumped_mass()
    loc, diag, iface, l2g, off = hdist.range_partition(glob, rank, world, gdiag)
    ok = True
    g = gdel = None
    if rank == 0:
        with Solver(glob, device=dev) as g1:
            g1.step(1, glob.n_steps)
            g = g1.download()
            gdel = [tuple(int(v) for v in x) for x in g1.deleted()]
    for caps in (None, 1):
        sv = Solver(loc, device=dev, diag_M=diag)
        sv.set_element_offset(loc.global_element_offset)
        uid = comm_unique_id() if rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        dist.broadcast(t, 0)
        sv.comm_init(rank, world, bytes(t.tolist()))
        sv.set_interface(*iface)
        sv.set_contact_global(glob, l2g, off, gdiag)
        if caps:
            for k in ("contact_exchange_deletions", "contact_exchange_bins", "contact_exchange_events"):
                sv.set_tuning(k, caps)
        sv.step(1, glob.n_steps)
        st = sv.download()
        dels = [tuple(int(v) for v in x) for x in sv.deleted()]
        stats = sv.contact_stats()
        sv.close()
        objs = [None] * world
        dist.all_gather_object(objs, (l2g, loc.global_element_offset, loc.nElement, st.disp, st.element_flag, dels,
                                      stats["candidate_triangles"]))
        if rank == 0:
            alld = sorted(d for o in objs for d in o[5])
            same = alld == gdel
            for l2, e0, ne, disp, flag, _, _ in objs:
                same &= np.array_equal(disp.reshape(-1, 3), g.disp.reshape(-1, 3)[l2 - 1])
                same &= np.array_equal(flag, g.element_flag[e0:e0 + ne])
            print(f"RCCL {world}-rank contact (exchange capacities {caps or 'default'}) vs 1 context bit-exact: {same}; "
                  f"deletions {len(gdel)}; "
                  f"candidates per rank {[o[6] for o in objs]}", flush=True)
            ok &= same
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
