"""HAKAI(fname) end to end on the GPU (reader -> setup -> device time loop -> 101 VTK files), timed
with the VTK writer asynchronous (default) and synchronous, to show what output costs the driver
surface (the reference writes synchronously on one thread, v2/HAKAI_j.jl:471-480, :932-942).

    python tools/bench_driver.py [--nz 250] [--steps 2000] [--out /tmp/hakai_drv]

Prints one JSON line per mode: wall seconds of `bin/hakai deck out`, bytes written, and the
device-only seconds of the same step count (Solver.step without outputs)."""
import argparse
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hakai-fem_amd"), os.path.join(ROOT, "tests")]

MODES = {"async": {}, "sync": {"HAKAI_VTK_SYNC": "1"}, "sync1": {"HAKAI_VTK_SYNC": "1", "HAKAI_VTK_THREADS": "1"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nz", type=int, default=250)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--out", default="/tmp/hakai_drv")
    ap.add_argument("--modes", default="async,sync,sync1")
    a = ap.parse_args()
    from hakai import mesh
    from hakai.solver import Solver
    from inp_writer import write_inp
    m = mesh.bar_model(20, 20, a.nz, mesh.steel_ductile(), lambda z, L: 5e4 * z / L, n_steps=a.steps, name="drv")
    os.makedirs(a.out, exist_ok=True)
    deck = os.path.join(a.out, "drv.inp")
    write_inp(deck, m)
    with Solver(m, device=0) as sv:  # device-only time of the same steps
        sv.step(1, 10)
        sv.sync()
        t = time.perf_counter()
        sv.step(11, a.steps - 10)
        sv.sync()
        dev_s = (time.perf_counter() - t) * a.steps / max(1, a.steps - 10)
    for mode in a.modes.split(","):
        out = os.path.join(a.out, mode)
        shutil.rmtree(out, ignore_errors=True)
        env = dict(os.environ, **MODES[mode])
        t = time.perf_counter()
        subprocess.run([os.path.join(ROOT, "hakai-fem_amd", "bin", "hakai"), deck, out, "--quiet"], env=env,
                       check=True)
        wall = time.perf_counter() - t
        files = sorted(os.listdir(out))
        nbytes = sum(os.path.getsize(os.path.join(out, f)) for f in files)
        print(json.dumps({"mode": mode, "elements": m.nElement, "nodes": m.nNode, "steps": a.steps,
                          "files": len(files), "bytes": nbytes, "wall_s": round(wall, 3),
                          "device_steps_s": round(dev_s, 3),
                          "vtk_threads": env.get("HAKAI_VTK_THREADS", env.get("OMP_NUM_THREADS", "all"))}),
              flush=True)
        shutil.rmtree(out, ignore_errors=True)


if __name__ == "__main__":
    main()
