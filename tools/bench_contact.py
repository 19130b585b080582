#!/usr/bin/env python3
"""C4 contact workload (BASELINE configs[3]): plate 200x200x50 + impactor 100x100x200 (4 M hex),
gap 0.1 mm, impactor v = -1e5 mm/s, elastoplastic steel, all-exterior contact, frictionless.

Prints one JSON line: element-updates/s over the timed steps (contact search + force included) and
the per-kernel split from the library's HIP-event timers. --scale divides every edge count.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--preload", type=int, default=30, help="steps before timing (contact starts at ~10)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--ranks", type=int, default=1,
                    help=">1: range-partitioned in-process group on this one GPU (multi-GPU contact, "
                         "owner-computed search; measures the per-rank contact cost incl. the exchanges, not scaling)")
    ap.add_argument("--serial", type=int, default=1,
                    help="multi-rank (tuning group_serial): 1 drains each rank's phase before the next rank's, so "
                         "the per-rank timings are not inflated by the ranks sharing this one GPU; 2 also "
                         "enqueues each phase behind a fixed sleep kernel, so it runs back to back as in a "
                         "pipelined run instead of at the host's enqueue pace")
    ap.add_argument("--tuning", default="", help="extra hakai_set_tuning keys, e.g. contact_exchange_bins=4096")
    ap.add_argument("--profile", type=int, default=1,
                    help="one context: 0 times the steps without the per-kernel event timers, so the steps can "
                         "replay from hipGraphs (HAKAI_GRAPH; events keep a context in stream mode)")
    ap.add_argument("--x-slabs", type=int, default=0,
                    help="1: C4 with its elements numbered x slowest, so the rank ranges are x-slabs that "
                         "share the contact zone (the default z-slab ranges put it on two ranks)")
    a = ap.parse_args()
    a.tuning = [(kv.split("=")[0], int(kv.split("=")[1])) for kv in a.tuning.split(",") if kv]
    if a.ranks > 1:
        return group(a)
    import numpy as np
    from hakai import mesh
    from hakai._abi import K_BC, K_CONTACT, K_ELEMENT, K_NODAL
    from hakai.solver import Solver
    t0 = time.time()
    m = mesh.config_c4(a.scale, x_slabs=bool(a.x_slabs))
    t1 = time.time()
    sv = Solver(m)
    for k, v in a.tuning:
        sv.set_tuning(k, v)
    t2 = time.time()
    pairs, sizes = sv.contact_info()
    sv.step(1, a.preload)
    sv.sync()
    sv.profile(bool(a.profile))
    g0 = sv.stat("graph_steps")
    ts = time.perf_counter()
    sv.step(1 + a.preload, a.steps)
    sv.sync()
    el = time.perf_counter() - ts
    graph_steps = sv.stat("graph_steps") - g0
    k = {n: sv.profile_read(i) for i, n in ((K_ELEMENT, "element"), (K_NODAL, "nodal"), (K_BC, "bc"),
                                            (K_CONTACT, "contact"))} if a.profile else {}
    cstats = sv.contact_stats()
    dl = sv.deleted()
    t_lo, t_hi = 1 + a.preload, a.preload + a.steps
    del_steps = sorted(set(int(x) for x in dl[:, 0])) if len(dl) else []
    f = sv.contact_force(1 + a.preload + a.steps)
    st = sv.download(element_flag=True)
    n_active = int(st.element_flag.sum())
    out = {
        "workload": f"{m.name} two-body impact, scale 1/{a.scale}", "tuning": dict(a.tuning),
        "elements": m.nElement, "nodes": m.nNode,
        "pairs": pairs, "element_size": sizes, "steps": a.steps, "preload": a.preload,
        "value_M_element_updates_per_s": round(n_active * a.steps / el / 1e6, 3),
        "ms_per_step": round(el / a.steps * 1e3, 4),
        "timed_steps_from_graphs": int(graph_steps),
        "kernel_ms_per_step": {n: round(v[0] / max(v[1], 1), 4) for n, v in k.items() if v[1]},
        "deleted_elements": int(len(dl)),
        "timed_steps_with_deletions": sum(1 for x in del_steps if t_lo <= x <= t_hi),
        "first_deletion_step": del_steps[0] if del_steps else None,
        "contact_stats_last_step": cstats,
        "contact_nodes_with_force": int(np.count_nonzero(np.abs(f.reshape(-1, 3)).sum(1))),
        "setup_s": {"mesh": round(t1 - t0, 2), "upload_contact_setup": round(t2 - t1, 2)},
    }
    sv.close()
    print(json.dumps(out), flush=True)


def group(a):
    import numpy as np
    from hakai import dist, mesh
    from hakai._abi import K_BC, K_CONTACT, K_CONTACT_SUM, K_ELEMENT, K_EXCHANGE, K_NODAL
    from hakai.solver import Solver, step_group
    m = mesh.config_c4(a.scale, x_slabs=bool(a.x_slabs))
    gdiag, _ = m.lumped_mass()
    parts = [dist.range_partition(m, r, a.ranks, gdiag) for r in range(a.ranks)]
    svs = []
    t0 = time.time()
    for r, (loc, diag, iface, l2g, off) in enumerate(parts):
        sv = Solver(loc, diag_M=diag)
        sv.set_element_offset(loc.global_element_offset)
        sv.comm_init_local(r, a.ranks, 4242)
        sv.set_interface(*iface)
        sv.set_contact_global(m, l2g, off, gdiag)
        sv.set_tuning("group_serial", a.serial)
        for k, v in a.tuning:
            sv.set_tuning(k, v)
        svs.append(sv)
    t1 = time.time()
    step_group(svs, 1, a.preload)
    for sv in svs:
        sv.sync()
        sv.profile(True)
    # exchange blocks are sized from recent counts; a burst past a capacity reruns the poisoned step
    # and the rest of the call (hakai_stat "exchange_retries"): counted across the timed window
    retries0 = [sv.stat("exchange_retries") for sv in svs]
    ts = time.perf_counter()
    step_group(svs, 1 + a.preload, a.steps)
    for sv in svs:
        sv.sync()
    el = time.perf_counter() - ts
    retries1 = [sv.stat("exchange_retries") for sv in svs]
    ranks = []
    for r, (sv, (loc, *_)) in enumerate(zip(svs, parts)):
        k = {n: sv.profile_read(i) for i, n in ((K_ELEMENT, "element"), (K_NODAL, "nodal"), (K_BC, "bc"),
                                                (K_CONTACT, "contact"), (K_CONTACT_SUM, "contact_sum"),
                                                (K_EXCHANGE, "exchange"))}
        # (the contact search is timed per part: three event pairs per step on a rank)
        per = {n: round(v[0] / (a.steps if n == "contact" else max(v[1], 1)), 4) for n, v in k.items() if v[1]}
        ranks.append({"elements": loc.nElement, "nodes": loc.nNode, "kernel_ms_per_step": per,
                      "contact_total_ms_per_step": round(per.get("contact", 0) + per.get("contact_sum", 0), 4),
                      "exchange_retries_in_timed_window": retries1[r] - retries0[r],
                      "contact_stats_last_step": sv.contact_stats()})
    out = {"workload": f"{m.name} two-body impact, scale 1/{a.scale}, {a.ranks} ranks on ONE GPU (in-process group), "
                       f"owner-computed search, group_serial={a.serial}",
           "elements": m.nElement, "steps": a.steps, "preload": a.preload,
           "group_ms_per_step_all_ranks": round(el / a.steps * 1e3, 4), "setup_s": round(t1 - t0, 2),
           "ranks": ranks}
    for sv in svs:
        sv.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
