#!/usr/bin/env python3
"""RCCL transport check on whatever GPUs are visible: 2 ranks (both on device 0 when only one GPU
is visible), slab-partitioned deletion bar, hakai_comm_init over RCCL, compared bit for bit with a
single-context run. Launch:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \\
      --master-port 29533 tools/rccl_2rank_check.py
Rendezvous and the unique-id broadcast use gloo, so torch never opens its own RCCL communicator."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hakai-fem_amd"), os.path.join(ROOT, "tests")]


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    from hakai import dist as hdist
    from hakai import device_count
    from hakai.solver import Solver, comm_unique_id
    from util import fast_deletion_bar

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = rank % max(device_count(), 1)
    glob = fast_deletion_bar(2, 2, 12)
    n = 1200
    loc, diag, iface = hdist.slab_partition(glob, rank, world, 2, 2)
    sv = Solver(loc, device=dev, diag_M=diag)
    sv.set_element_offset(loc.global_element_offset)
    uid = comm_unique_id() if rank == 0 else bytes(128)
    t = torch.tensor(list(uid), dtype=torch.uint8)
    dist.broadcast(t, 0)
    sv.comm_init(rank, world, bytes(t.tolist()))
    sv.set_interface(*iface)
    sv.step(1, n)
    st = sv.download()
    dels = [tuple(x) for x in sv.deleted()]
    sv.close()
    ok = True
    if rank == 0:
        with Solver(glob, device=dev) as g1:
            g1.step(1, n)
            g = g1.download()
            gdel = [tuple(x) for x in g1.deleted()]
    objs = [None] * world
    dist.all_gather_object(objs, (loc.global_node_offset, loc.nNode, loc.global_element_offset, loc.nElement,
                                  st.disp, st.integ_stress, dels))
    if rank == 0:
        alld = sorted(d for o in objs for d in o[6])
        ok &= alld == gdel
        for n0, nl, e0, el, disp, stress, _ in objs:
            ok &= np.array_equal(disp, g.disp[3 * n0:3 * (n0 + nl)])
            ok &= np.array_equal(stress, g.integ_stress[8 * e0:8 * (e0 + el)])
        print(f"RCCL {world}-rank vs 1-rank bit-exact: {ok}; deletions {len(gdel)}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
