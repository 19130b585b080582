"""Find the first ductile deletion of the full-size C3 bar (2 M hex) for a few initial stretch rates.

Run on the GPU box: python tools/diag_fullsize_deletion.py [max_steps]. Prints one line per chunk of
steps and the first deletion step per variant, so tests/test_gpu_fullsize.py can pin a window.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))

from hakai import mesh  # noqa: E402
from hakai.solver import Solver  # noqa: E402


def main():
    max_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
    for v_end in (5e5, 1e6, 2e6):
        m = mesh.config_c3(v_end=v_end)
        t0 = time.time()
        with Solver(m) as sv:
            t, chunk, first = 1, 1000, None
            while t <= max_steps:
                sv.step(t, chunk)
                t += chunk
                d = sv.deleted()
                if len(d) and first is None:
                    first = int(d[0][0])
                    print(f"v_end {v_end:g}: first deletion step {first}, {len(d)} deletions by step {t - 1}, "
                          f"first ten {d[:10].tolist()}", flush=True)
                    break
                if (t - 1) % 5000 == 0:
                    print(f"v_end {v_end:g}: step {t - 1}, no deletion ({time.time() - t0:.1f} s)", flush=True)
        if first is None:
            print(f"v_end {v_end:g}: no deletion within {max_steps} steps", flush=True)


if __name__ == "__main__":
    main()
