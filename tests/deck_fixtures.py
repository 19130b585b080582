"""Reference decks as test vectors: a parsed deck (readInpFile's ModelType, v2/readInpFile_j.jl:129-150)
flattened into an .npz together with the oracle's state after a number of steps.

The GPU box has no /root/reference, so tools/make_deck_golden.py parses the shipped decks HERE
(hakai.read_inp) and runs the oracle on them; the GPU tests rebuild the Model from the arrays.
"""
from __future__ import annotations

import numpy as np

from hakai.model import BCGroup, Material, Model


def model_to_arrays(m: Model) -> dict:
    a = {"coordmat": m.coordmat, "elementmat": m.elementmat, "element_material": m.element_material,
         "element_instance": (m.element_instance if m.element_instance is not None
                              else np.ones(m.nElement, np.int64)),
         "scalars": np.array([m.d_time, m.end_time, m.mass_scaling, m.contact_flag], np.float64),
         "ic_dofs": m.ic_dofs, "ic_values": m.ic_values, "n_mat": np.array(len(m.materials))}
    for i, mt in enumerate(m.materials):
        a[f"mat{i}_elastic"] = np.array([mt.density, mt.young, mt.poisson])
        a[f"mat{i}_plastic"] = np.asarray(mt.plastic, np.float64).reshape(-1, 2)
        a[f"mat{i}_ductile"] = np.asarray(mt.ductile, np.float64).reshape(-1, 3)
    a["n_bc"] = np.array(len(m.bc))
    for g, grp in enumerate(m.bc):
        a[f"bc{g}_n"] = np.array(len(grp.entries))
        for j, (d, v) in enumerate(grp.entries):
            a[f"bc{g}_{j}_dofs"] = np.asarray(d, np.int64)
            a[f"bc{g}_{j}_value"] = np.array(float(v))
        if grp.amp_time is not None:
            a[f"bc{g}_amp"] = np.stack([np.asarray(grp.amp_time, np.float64), np.asarray(grp.amp_value, np.float64)])
    cps = m.contact_pairs or []
    a["n_cp"] = np.array(len(cps))
    for k, cp in enumerate(cps):
        for s in range(2):
            a[f"cp{k}_{s}_inst"] = np.array(int(cp[s][0]))
            a[f"cp{k}_{s}_elems"] = np.asarray(cp[s][1], np.int64)
    return a


def model_from_arrays(z, name: str = "deck") -> Model:
    mats = [Material(f"mat{i}", *[float(x) for x in z[f"mat{i}_elastic"]], z[f"mat{i}_plastic"].copy(),
                     z[f"mat{i}_ductile"].copy()) for i in range(int(z["n_mat"]))]
    bc = []
    for g in range(int(z["n_bc"])):
        ents = [(z[f"bc{g}_{j}_dofs"].copy(), float(z[f"bc{g}_{j}_value"])) for j in range(int(z[f"bc{g}_n"]))]
        amp = z[f"bc{g}_amp"] if f"bc{g}_amp" in z else None
        bc.append(BCGroup(ents, None if amp is None else amp[0].copy(), None if amp is None else amp[1].copy()))
    cps = None
    if int(z["n_cp"]) > 0:
        cps = [tuple((int(z[f"cp{k}_{s}_inst"]), z[f"cp{k}_{s}_elems"].copy()) for s in range(2))
               for k in range(int(z["n_cp"]))]
    d_time, end_time, ms, cf = (float(x) for x in z["scalars"])
    return Model(z["coordmat"].copy(), z["elementmat"].copy(), z["element_material"].copy(), mats, bc,
                 z["ic_dofs"].copy(), z["ic_values"].copy(), d_time, end_time, ms, int(cf),
                 z["element_instance"].copy(), name=name, contact_pairs=cps)
