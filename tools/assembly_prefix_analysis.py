#!/usr/bin/env python3
"""How much of the element-force round trip (fe, 24 B per element-node written by the element
kernel and gathered back by the nodal kernel) an order-preserving pre-reduction inside the element
kernel's 32-element batches could remove (candidate (a)).

The nodal sum must be the reference's serial one, Q_n = ((f_e1 + f_e2) + f_e3) + ... over the node's
incident elements in ascending order (v2/HAKAI_j.jl:668-675). A batch can only hand over a PREFIX
partial (f_e1 + ... + f_ek) whose elements all sit in the batch of e1; any later pair would
re-associate the sum. This counts, on the bench meshes' connectivity, the fe entries such prefixes
save. CPU only; prints one JSON line per mesh."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))


def analyse(em, batch=32):
    nN = int(em.max())
    inc = [[] for _ in range(nN)]
    for e, row in enumerate(em):
        for n in row:
            inc[n - 1].append(e)
    hist = np.zeros(9, np.int64)
    entries = saved = 0
    for lst in inc:
        lst.sort()
        b0 = lst[0] // batch
        k = 1
        while k < len(lst) and lst[k] // batch == b0:
            k += 1
        hist[k] += 1
        entries += len(lst)
        saved += k - 1  # a prefix of k entries becomes one partial
    return entries, saved, hist


def main():
    from hakai import mesh
    out = []
    for name, m in (("C3 slice 20x20x50 (same connectivity pattern as 20x20x5000)", mesh.config_c3(100)),
                    ("C5 slab 100x100x20", mesh.config_c5(layers=20))):
        entries, saved, hist = analyse(m.elementmat)
        fe_bytes = 24 * entries
        out.append({"mesh": name, "elements": int(m.nElement), "nodes": int(m.nNode), "fe_entries": entries,
                    "entries_saved_by_prefix_partials": saved, "fraction_saved": round(saved / entries, 4),
                    "prefix_length_histogram": hist.tolist(),
                    "fe_round_trip_bytes_saved_per_element": round(2 * 24 * saved / m.nElement, 1),
                    "fe_round_trip_bytes_per_element": round(2 * fe_bytes / m.nElement, 1)})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
