#!/usr/bin/env python3
"""Golden vectors from the reference's own input decks (run HERE, where /root/reference exists).

For each deck: parse it with hakai.read_inp (readInpFile), run the oracle (the C restatement of
HAKAI v0.0.2) for `steps` steps, and save the flattened model plus the oracle's displacement,
element flags and deletion log to tests/golden/deck_<name>.npz. tests/test_gpu_decks.py runs the
GPU path on the same arrays. The decks are v0.0.0/v0.0.1 inputs the v0.0.2 solver also reads.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import hakai  # noqa: E402
import oracle as O  # noqa: E402
from deck_fixtures import model_to_arrays  # noqa: E402

REF = "/root/reference"
DECKS = [  # (deck, steps, indexed oracle contact)
    ("HAKAI-v0.0.0/input/Charpy-test.inp", 6200, False),               # contact + deletion
    ("HAKAI-v0.0.1/input/crash-tube-80-350-solid.inp", 2000, False),   # self-contact option
    ("HAKAI-v0.0.0/input/bullet-impact.inp", 12000, False),            # projectile + deletion
    ("HAKAI-v0.0.2/input/car-crash-N2k.inp", 0, False),                # v0.0.2, whole run
    ("HAKAI-v0.0.2/input/car-wall-N2k.inp", 0, True),                  # v0.0.2 self-contact, whole run
]


def main():
    out = os.path.join(ROOT, "tests", "golden")
    sel = sys.argv[1:]
    for deck, steps, indexed in DECKS:
        if sel and not any(x in deck for x in sel):
            continue
        m = hakai.read_inp(os.path.join(REF, deck))
        steps = steps or m.n_steps
        o = O.Oracle(m, nthreads=int(os.environ.get("OMP_NUM_THREADS", "4")), contact_indexed=indexed)
        t0 = time.time()
        o.run(1, steps)
        f, nev = o.contact_force()
        name = os.path.splitext(os.path.basename(deck))[0].replace("-", "_")
        a = model_to_arrays(m)
        a.update(steps=np.array(steps), disp=o.s["disp"], disp_pre=o.s["disp_pre"],
                 element_flag=o.s["element_flag"], deletions=np.array(o.deletions, np.int64).reshape(-1, 2),
                 contact_force_next=f)
        np.savez_compressed(os.path.join(out, f"deck_{name}.npz"), **a)
        print(f"{deck}: {steps} steps in {time.time() - t0:.1f} s, {len(o.deletions)} deletions, "
              f"{nev} contact events at step {steps + 1}")


if __name__ == "__main__":
    main()
