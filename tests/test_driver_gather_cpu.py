"""The N-GPU driver's output transfer (hakai.run.gather_parts) on CPU: world_size 2 and 3 over gloo.
Every rank's output arrays (node displacements and velocities, Gauss-point stress, strain, eqps,
triaxiality, element flags of its range partition) arrive at rank 0 unchanged, by raw point-to-point
transfers into preallocated buffers (no pickling), and assemble into the global arrays the
single-process driver would hold."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as tdist
import torch.multiprocessing as mp

from hakai import dist
from hakai.run import OUT_KEYS, _out_shapes, gather_parts
from util import fast_deletion_bar


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _part(rank, loc):
    rng = np.random.default_rng(100 + rank)
    out = {}
    for k, (shape, dt) in _out_shapes(loc.nNode, loc.nElement).items():
        out[k] = rng.integers(0, 2, size=shape).astype(dt) if dt == np.int64 else rng.normal(size=shape)
    return out


def _worker(rank, world, port, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        glob = fast_deletion_bar(2, 2, 12)
        gdiag, _ = glob.lumped_mass()
        loc, _, _, l2g, off = dist.range_partition(glob, rank, world, gdiag)
        group = tdist.new_group(backend="gloo")
        metas = [None] * world if rank == 0 else None
        tdist.gather_object((l2g, int(off[rank]), loc.nElement), metas, dst=0, group=group)
        for step in range(2):  # two output steps over the same group
            parts = gather_parts(tdist, group, rank, world, _part(rank + 10 * step, loc), metas)
            if rank == 0:
                ok = len(parts) == world
                for r, ((l2, e0), arrs) in enumerate(parts):
                    lr, _, _, l2r, offr = dist.range_partition(glob, r, world, gdiag)
                    want = _part(r + 10 * step, lr)
                    ok &= np.array_equal(l2, l2r) and e0 == int(offr[r])
                    for k in OUT_KEYS:
                        ok &= arrs[k].dtype == want[k].dtype and np.array_equal(arrs[k], want[k])
                ret[step] = bool(ok)
            else:
                assert parts is None
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_parts_binary_transfer(world):
    port = _free_port()
    ret = mp.Manager().dict()
    mp.spawn(_worker, args=(world, port, ret), nprocs=world, join=True)
    assert ret.get(0) and ret.get(1)
