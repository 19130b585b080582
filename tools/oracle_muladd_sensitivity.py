#!/usr/bin/env python3
"""What is "bit-exact to the reference" worth? The one arithmetic assumption of the oracle that no
fixture pins: StaticArrays lowers the three element products (Bfinal*d_u, Dmat*de, Bfinal'*sigma;
v2/HAKAI_j.jl:1204-1205, :1330) to muladd, which fuses on FMA hosts (oracle/hakai_oracle.h). This
tool runs the oracle built the other way (oracle/_build/libhakai_oracle_nofma.so: product and sum
rounded separately, HKO_SEPARATE_ROUNDING) on the committed fixtures' workloads and reports how far
the trajectories move:

  * Tensile5e.inp (20 000 steps): the deletion step of element 3 under both lowerings, final
    displacement against tests/golden/tensile5e_oracle.npz;
  * the deleting bar fixture (tests/golden/fast_deletion_bar_oracle.npz);
  * a C3 section slice (20x20x100, C3's material, strain rate and deletion on) through its first
    deletion waves, both lowerings run here;
  * the reference's own decks (tests/golden/deck_*.npz, oracle fixtures of the whole runs).

One JSON line per case: max|u_nofma - u_fma| / max|u_fma| of the final displacement, both deletion
logs' sizes and whether they agree (and the first step where they differ).

    OMP_NUM_THREADS=8 python tools/oracle_muladd_sensitivity.py [case-substring ...]
"""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DECKS = [("Charpy_test", False), ("bullet_impact", False), ("crash_tube_80_350_solid", False),
         ("car_crash_N2k", False), ("car_wall_N2k", True)]
CASES = ["tensile5e", "deletion_bar", "c3_slice"] + ["deck_" + d for d, _ in DECKS]


def child(case):
    """Runs in a subprocess (the oracle library variant is picked at import): prints disp + deletions."""
    sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from hakai import mesh
    threads = int(os.environ.get("OMP_NUM_THREADS", "8"))
    t0 = time.time()
    if case == "tensile5e":
        m, steps, kw = mesh.tensile5e_model(), 20000, {}
    elif case == "deletion_bar":
        from util import fast_deletion_bar
        m = fast_deletion_bar()
        steps, kw = m.n_steps, {}
    elif case == "c3_slice":
        m = mesh.bar_model(20, 20, 100, mesh.steel_ductile(), lambda z, L: 5e5 * z / 5000, name="C3-slice")
        steps, kw = int(os.environ.get("C3_SLICE_STEPS", "8400")), {}
    else:
        from deck_fixtures import model_from_arrays
        name = case[5:]
        z = np.load(os.path.join(ROOT, "tests", "golden", f"deck_{name}.npz"))
        m = model_from_arrays(z, name)
        steps = int(z["steps"])
        kw = {"contact_indexed": dict(DECKS)[name]}
    o = O.Oracle(m, nthreads=threads, **kw)
    o.run(1, steps)
    out = os.environ["SENS_OUT"]
    np.savez(out, disp=o.s["disp"], deletions=np.array(o.deletions, np.int64).reshape(-1, 2),
             steps=steps, secs=time.time() - t0)


def run_variant(case, variant, tmp):
    env = dict(os.environ, SENS_OUT=tmp, HAKAI_ORACLE_VARIANT=variant)
    subprocess.run([sys.executable, os.path.abspath(__file__), "--child", case], env=env, check=True)
    z = np.load(tmp)
    return z["disp"], [tuple(int(v) for v in x) for x in z["deletions"]], int(z["steps"]), float(z["secs"])


def fixture(case):
    g = os.path.join(ROOT, "tests", "golden")
    if case == "tensile5e":
        z = np.load(os.path.join(g, "tensile5e_oracle.npz"))
        return z["disp_out"][-1], [tuple(int(v) for v in x) for x in z["deletions"]]
    if case == "deletion_bar":
        z = np.load(os.path.join(g, "fast_deletion_bar_oracle.npz"))
        return z["disp"], [tuple(int(v) for v in x) for x in z["deletions"]]
    if case.startswith("deck_"):
        z = np.load(os.path.join(g, f"{case}.npz"))
        return z["disp"], [tuple(int(v) for v in x) for x in z["deletions"]]
    return None


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    sel = sys.argv[1:]
    tmp = "/tmp/hakai_sens_%d.npz" % os.getpid()
    for case in CASES:
        if sel and not any(s in case for s in sel):
            continue
        fx = fixture(case)
        if fx is None:  # no committed fixture: both lowerings run here
            d_fma, del_fma, steps, s_fma = run_variant(case, "fma", tmp)
        else:
            d_fma, del_fma = fx
            s_fma = None
        d_sep, del_sep, steps, s_sep = run_variant(case, "nofma", tmp)
        den = float(np.max(np.abs(d_fma)))
        first_diff = None
        for a, b in zip(sorted(del_fma), sorted(del_sep)):
            if a != b:
                first_diff = [list(a), list(b)]
                break
        rec = {"case": case, "steps": steps, "reference_side": "committed fixture" if fx is not None else "fma build, run here",
               "final_disp_rel_diff": float(np.max(np.abs(d_sep - d_fma)) / den) if den > 0 else 0.0,
               "deletions_fma": len(del_fma), "deletions_nofma": len(del_sep),
               "same_deletions": sorted(del_fma) == sorted(del_sep), "first_differing_deletion": first_diff,
               "oracle_s": round(s_sep, 1)}
        if case == "tensile5e":
            rec["element3_deletion_step"] = {"fma": [s for s, e in del_fma if e == 3],
                                             "nofma": [s for s, e in del_sep if e == 3]}
        if case == "c3_slice" and del_fma:
            rec["first_deletion_step"] = {"fma": min(s for s, _ in del_fma), "nofma": min(s for s, _ in del_sep)
                                          if del_sep else None}
        print(json.dumps(rec), flush=True)
    if os.path.exists(tmp):
        os.remove(tmp)


if __name__ == "__main__":
    main()
