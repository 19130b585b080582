"""RCCL with more than one rank (hakai_comm_init: grouped ncclSend/ncclRecv interface exchange,
ncclAllReduce / ncclAllGather at setup, the multi-GPU contact search's per-step exchanges),
one process per rank under torch.distributed.run, against one context bit for bit. On a one-GPU box
the ranks share the device (HAKAI_RCCL_SHARED_GPU=1: hakai.dist.rank_device makes them separate
hosts to RCCL, which then connects them with its socket transport over loopback) -- the same RCCL
calls, sizes and buffers as on an N-GPU node, another transport."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    return dict(os.environ, HAKAI_RCCL_SHARED_GPU="1")


def _torchrun(script, n, *args, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, script), *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=_env())
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    return r.stdout


@pytest.mark.parametrize("n", [2, 3])
def test_rccl_interface_exchange_bitexact(n):
    """A deleting bar in z-slabs over n RCCL ranks (the middle rank exchanges with both neighbours)."""
    out = _torchrun("tools/rccl_exchange_check.py", n)
    assert f"RCCL {n}-rank interface exchange vs 1 context bit-exact: True" in out


@pytest.mark.parametrize("n", [2, 3])
def test_rccl_interface_exchange_owner_assembly_bitexact(n):
    """The same over RCCL with owner-computed assembly on every rank (k_pack_own / k_fix_own)."""
    out = _torchrun("tools/rccl_exchange_check.py", n, "--own")
    assert f"RCCL {n}-rank interface exchange (owner-computed assembly) vs 1 context bit-exact: True" in out


@pytest.mark.parametrize("world", [2, 3])
def test_rccl_contact_bitexact(world):
    """Two-body impact with contact deletions over 2 and 3 RCCL ranks (owner-computed search; at 3
    ranks the middle rank exchanges with both neighbours), with the default exchange capacities
    and with one-record blocks that grow (the overflowing steps run again)."""
    out = _torchrun("tools/rccl_contact_check.py", world)
    assert f"RCCL {world}-rank contact (exchange capacities default) vs 1 context bit-exact: True" in out
    assert f"RCCL {world}-rank contact (exchange capacities 1) vs 1 context bit-exact: True" in out


def test_torchrun_driver_writes_the_same_vtk():
    """python -m hakai.run deck.inp over 2 RCCL ranks: 101 VTK files byte-identical to one GPU's."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "driver_torchrun_smoke.py"), "--nproc", "2"],
                       capture_output=True, text=True, timeout=400, cwd=ROOT, env=_env())
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "byte-identical: True" in r.stdout
