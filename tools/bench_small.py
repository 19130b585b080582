"""Per-step wall time of small meshes (the size of the reference's shipped decks), where the step
loop is bound by kernel launches rather than HBM. One JSON line per case.

    python tools/bench_small.py [--steps 2000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hakai-fem_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--only", default="", help="run the cases whose name contains this")
    ap.add_argument("--graphs", default="0,2,16,64", help="graph tuning values to compare")
    ap.add_argument("--tuning", default="", help="extra tuning key=value[,key=value] for every context")
    a = ap.parse_args()
    from hakai import mesh
    from hakai.solver import Solver
    cases = [
        ("tensile5e (5 hex)", mesh.tensile5e_model()),
        ("bar 10x10x20 (2 k hex)", mesh.bar_model(10, 10, 20, mesh.steel_ductile(), lambda z, L: 5e4 * z / L)),
        ("bar 20x20x50 (20 k hex)", mesh.bar_model(20, 20, 50, mesh.steel_ductile(), lambda z, L: 5e4 * z / L)),
        ("two-body contact (plate 24x24x6 + 12x12x12, 5 k hex)", mesh.two_body_model(plate=(24, 24, 6),
                                                                                impactor=(12, 12, 12))),
    ]
    for name, m in cases:
        if a.only not in name:
            continue
        for graph in (int(g) for g in a.graphs.split(",")):
            with Solver(m, device=0) as sv:
                sv.set_tuning("graph", graph)
                for kv in filter(None, a.tuning.split(",")):
                    k, v = kv.split("=")
                    sv.set_tuning(k, int(v))
                sv.step(1, 50)
                sv.sync()
                g0 = sv.graph_steps()
                t0 = time.perf_counter()
                sv.step(51, a.steps)
                t1 = time.perf_counter()
                sv.sync()
                t2 = time.perf_counter()
                gs = sv.graph_steps() - g0
            print(json.dumps({"case": name, "elements": m.nElement, "steps": a.steps, "graph": graph,
                              "tuning": a.tuning,
                              "graph_steps": gs, "us_per_step": round((t2 - t0) / a.steps * 1e6, 2),
                              "host_enqueue_us_per_step": round((t1 - t0) / a.steps * 1e6, 2),
                              "contact": bool(getattr(m, "contact_flag", 0))}), flush=True)


if __name__ == "__main__":
    main()
