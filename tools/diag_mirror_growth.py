"""Diagnostic: exposed-node chunk needs and block growth of the contact mirror over a run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
from hakai import dist, mesh  # noqa: E402
from hakai.solver import Solver  # noqa: E402

cap = int(sys.argv[1]) if len(sys.argv) > 1 else 1
pz = int(sys.argv[2]) if len(sys.argv) > 2 else 2
glob = mesh.two_body_model(plate=(16, 16, pz), impactor=(4, 4, 4), v=-3e5, d_time=2e-8, n_steps=600)
gdiag, _ = glob.lumped_mass()
parts = [dist.range_partition(glob, r, 2, gdiag) for r in range(2)]
svs = []
for r, (loc, diag, iface, l2g, off) in enumerate(parts):
    sv = Solver(loc, diag_M=diag)
    sv.set_element_offset(loc.global_element_offset)
    sv.comm_init_local(r, 2, 9191)
    sv.set_interface(*iface)
    sv.set_contact_global(glob, l2g, off, gdiag)
    sv.set_tuning("contact_mirror_chunks", cap)
    svs.append(sv)
last = None
for t in range(1, glob.n_steps + 1):
    try:
        for sv in svs:
            sv.step(t, 1)
    except Exception as e:
        print("step", t, "error:", e)
        break
    st = svs[0].contact_stats()
    cur = (st["mirror_chunks_sent"], st["mirror_block_bytes"])
    if cur != last:
        print("step", t, "chunks sent (all ranks)", cur[0], "block bytes", cur[1], "deleted", len(svs[0].deleted()) + len(svs[1].deleted()))
        last = cur
for sv in svs:
    sv.close()
