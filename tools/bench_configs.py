#!/usr/bin/env python3
"""Every single-GPU BASELINE configuration in one process (one JSON line each): C2 (1 M-hex elastic
bar), C3 (2 M-hex elastoplastic bar with deletion, the bench.py workload), C4 (4 M-hex two-body
impact with contact) and one 2 M-hex slab of the C5 bar. Per-kernel times from the library's HIP
events; element-updates/s = active elements x steps / wall time of the step loop."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))


def run(name, m, preload, steps):
    from hakai._abi import K_BC, K_CONTACT, K_ELEMENT, K_NODAL
    from hakai.solver import Solver
    with Solver(m) as sv:
        sv.step(1, preload)
        sv.sync()
        sv.profile(True, kernels=[K_ELEMENT])
        t0 = time.perf_counter()
        sv.step(1 + preload, steps)
        sv.sync()
        el = time.perf_counter() - t0
        e_ms, e_n = sv.profile_read(K_ELEMENT)
        sv.profile(True)
        sv.step(1 + preload + steps, 10)
        sv.sync()
        k = {n: sv.profile_read(i) for i, n in ((K_ELEMENT, "element"), (K_NODAL, "nodal"), (K_BC, "bc"),
                                                (K_CONTACT, "contact"))}
        st = sv.download(element_flag=True, integ_eq_plastic_strain=True)
        own = sv.stat("own_steps") > 0
    import numpy as np
    act = int(st.element_flag.sum())
    print(json.dumps({"config": name, "elements": m.nElement, "nodes": m.nNode, "steps": steps, "preload": preload,
                      "M_element_updates_per_s": round(act * steps / el / 1e6, 1),
                      "ms_per_step": round(el / steps * 1e3, 4),
                      "element_ms_timed": round(e_ms / max(e_n, 1), 4),
                      "kernel_ms_per_step": {n: round(v[0] / max(v[1], 1), 4) for n, v in k.items() if v[1]},
                      "plastic_gp_frac": round(float(np.mean(st.integ_eq_plastic_strain > 0)), 4),
                      "deleted": int(m.nElement - act),
                      "assembly": "owner-computed (LDS)" if own else "fe round trip"}), flush=True)


def main():
    from hakai import mesh
    run("C2 elastic bar 20x20x2500", mesh.config_c2(), 50, 200)
    run("C3 elastoplastic bar 20x20x5000 (v_end 5e5, as bench.py)", mesh.config_c3(v_end=5e5), 400, 200)
    run("C4 two-body impact 4 M hex, contact, frictionless", mesh.config_c4(), 30, 50)
    run("C5 slab 100x100x200 (one rank's share)", mesh.config_c5(layers=200), 20, 200)


if __name__ == "__main__":
    main()
