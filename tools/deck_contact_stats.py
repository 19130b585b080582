#!/usr/bin/env python3
"""Contact sizes of the reference decks on the GPU path (run to the end, fused mode): live triangles
and nodes, max events per step, candidate triangles and touched nodes of the last step, hash
buckets -- what a small-deck contact kernel would have to hold. One JSON line per deck."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("hakai-fem_amd", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))


def main():
    import numpy as np
    from deck_fixtures import model_from_arrays
    from hakai.solver import Solver
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else \
        ["car_crash_N2k", "car_wall_N2k", "Charpy_test", "bullet_impact", "crash_tube_80_350_solid"]
    for name in names:
        z = np.load(os.path.join(ROOT, "tests", "golden", f"deck_{name}.npz"))
        m = model_from_arrays(z, name)
        with Solver(m) as sv:
            pairs, sizes = sv.contact_info()
            sv.step(1, int(z["steps"]))
            st = sv.contact_stats()
        print(json.dumps({"deck": name, "elements": int(m.nElement), "nodes": int(m.nNode), "pairs": pairs,
                          "stats_last_step": st}), flush=True)


if __name__ == "__main__":
    main()
