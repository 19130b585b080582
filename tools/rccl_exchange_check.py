#!/usr/bin/env python3
"""RCCL check of the interface exchange (hakai_comm_init + hakai_set_interface: grouped
ncclSend/ncclRecv per step, an ncclAllReduce at setup) at any world size: a deleting elastoplastic
bar split into z-slabs (hakai.dist.slab_partition; middle ranks exchange with both neighbours),
every rank's final displacements, stresses, flags and deletions compared bit for bit with one
context on the whole bar. On a one-GPU box the ranks share the device (HAKAI_RCCL_SHARED_GPU=1,
hakai.dist.rank_device).
Launch:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \\
      --master-port 29537 tools/rccl_exchange_check.py
Rendezvous and the unique-id broadcast use gloo."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hakai-fem_amd"), os.path.join(ROOT, "tests")]

NX = NY = 6
NZ = 48
# --own: the persistent element kernel on a few blocks per rank, so owner-computed assembly runs on
# every rank (k_pack_own / k_fix_own over RCCL) and on the one-context reference
OWN = "--own" in sys.argv[1:]
TUNE = {"elem_pipe_min": 0, "elem_pipe_blocks": 4} if OWN else {}


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
    glob = mesh.bar_model(NX, NY, NZ, mesh.steel_ductile(), lambda z, L: 6e5 * z / L, n_steps=3000, d_time=1e-7)
    if rank == 0:
        with Solver(glob, device=dev) as g1:
            for k, v in TUNE.items():
                g1.set_tuning(k, v)
            g1.step(1, glob.n_steps)
            g = g1.download()
            gdel = sorted(tuple(int(v) for v in x) for x in g1.deleted())
    loc, diag, iface = hdist.slab_partition(glob, rank, world, nx=NX, ny=NY)
    sv = Solver(loc, device=dev, diag_M=diag)
    sv.set_element_offset(loc.global_element_offset)
    for k, v in TUNE.items():
        sv.set_tuning(k, v)
    uid = comm_unique_id() if rank == 0 else bytes(128)
    t = torch.tensor(list(uid), dtype=torch.uint8)
    dist.broadcast(t, 0)
    sv.comm_init(rank, world, bytes(t.tolist()))
    sv.set_interface(*iface)
    sv.step(1, 1000)  # two calls: the exchange state carries over between hakai_step calls
    sv.step(1001, glob.n_steps - 1000)
    st = sv.download()
    dels = [tuple(int(v) for v in x) for x in sv.deleted()]
    own_ok = (sv.stat("own_steps") == glob.n_steps) if OWN else True
    sv.close()
    npl = (NX + 1) * (NY + 1)
    k0 = hdist.partition_ranges(NZ, world)[rank][0]
    objs = [None] * world
    dist.all_gather_object(objs, (k0, st.disp, st.integ_stress, st.element_flag, dels, own_ok))
    ok = True
    if rank == 0:
        same = sorted(d for o in objs for d in o[4]) == gdel and all(o[5] for o in objs)
        for k0r, disp, stress, flag, _, _ in objs:
            n0, e0 = k0r * npl, k0r * NX * NY
            nn, ne = disp.size // 3, flag.size
            same &= np.array_equal(disp, g.disp[3 * n0:3 * (n0 + nn)])
            same &= np.array_equal(stress, g.integ_stress[8 * e0:8 * (e0 + ne)])
            same &= np.array_equal(flag, g.element_flag[e0:e0 + ne])
        tag = " (owner-computed assembly)" if OWN else ""
        print(f"RCCL {world}-rank interface exchange{tag} vs 1 context bit-exact: {same}; deletions {len(gdel)}",
              flush=True)
        ok = bool(same) and len(gdel) > 0
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
