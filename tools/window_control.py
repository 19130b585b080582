#!/usr/bin/env python3
"""Control for bench.py's deletion window: the same hand-off sequence far from any deletion.

The first version of bench.deletion_window (round 6) ran C3 to step 7940, downloaded the state, and
per element mode uploaded it, ran one untimed step, uploaded it again and timed 20 steps. Under
rocprofv3 --kernel-trace (tools/gpu_r6.sh wcontrol) this script repeats exactly that sequence at step
--first (default 441, the idle regime where no Gauss point is near the ductile table), so the per-step
element times of the two windows can be compared: the hump that showed up here too came from the
hand-off itself (the GPU idle while the state crosses PCIe), not from the deletion regime
(profiles/r06_window_control_trace.json). bench.py now runs 100 untimed steps per mode after the
hand-off instead."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))

from hakai import mesh  # noqa: E402
from hakai.solver import Solver  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--first", type=int, default=441)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    m = mesh.config_c3(v_end=5e5)
    diag, _ = m.lumped_mass()
    sv = Solver(m, diag_M=diag)
    sv.set_tuning("graph", 0)
    sv.step(1, a.first - 1)
    sv.sync()
    s0 = sv.download()
    for exact in (0, 1):
        sv.set_tuning("elem_exact", exact)
        sv.upload(s0)
        sv.step(a.first, 1)
        sv.sync()
        sv.upload(s0)
        t0 = time.perf_counter()
        sv.step(a.first, a.steps)
        sv.sync()
        print(f"mode {'exact' if exact else 'fused'}: {(time.perf_counter() - t0) / a.steps * 1e3:.4f} ms/step", flush=True)
    sv.close()


if __name__ == "__main__":
    main()
