"""Diagnostic: first step where a range-partitioned contact group departs from one context."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from hakai import mesh, dist
from hakai.solver import Solver, step_group


def run(flag, world, nsteps=400):
    glob = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=nsteps,
                               contact_flag=flag)
    gdiag, _ = glob.lumped_mass()
    single = Solver(glob)
    parts = [dist.range_partition(glob, r, world, gdiag) for r in range(world)]
    svs = []
    for r, (loc, diag, iface, l2g, off) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        sv.set_element_offset(loc.global_element_offset)
        sv.comm_init_local(r, world, 77 + flag * 10 + world)
        sv.set_interface(*iface)
        if flag:
            sv.set_contact_global(glob, l2g, off, gdiag)
        svs.append(sv)
    for t in range(1, nsteps + 1):
        single.step(t, 1)
        step_group(svs, t, 1)
        g = single.download(disp=True).disp.reshape(-1, 3)
        for r, sv in enumerate(svs):
            l2g = parts[r][3]
            d = sv.download(disp=True).disp.reshape(-1, 3)
            bad = np.nonzero(np.any(d != g[l2g - 1], axis=1))[0]
            if len(bad):
                print(f"flag {flag} world {world}: step {t} rank {r}: {len(bad)} nodes differ, global ids "
                      f"{(l2g[bad])[:10].tolist()} max |diff| {np.max(np.abs(d - g[l2g - 1])):.3e}")
                if flag:
                    print("  single stats", single.contact_stats())
                    print("  rank stats", sv.contact_stats())
                return
    print(f"flag {flag} world {world}: identical over {nsteps} steps")


for flag in (0, 1):
    run(flag, 2)
