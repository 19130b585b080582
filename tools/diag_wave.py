#!/usr/bin/env python3
"""Per-wave clock totals of the persistent element kernel (diagnostic build, -DHK_DIAG_WAVE):
where a wave's time goes -- block-barrier wait, summing pass, the rest (element compute) -- and
whether the waves of a block run at systematically different speeds.

    tools/variants.sh diagw "-DHK_DIAG_WAVE"
    HAKAI_LIB=hakai-fem_amd/lib/variants/diagw.so python tools/diag_wave.py [--config c3] [--steps 20]

Prints one JSON line per element mode."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hakai-fem_amd"))
from hakai import mesh  # noqa: E402
from hakai._abi import lib  # noqa: E402
from hakai.solver import Solver  # noqa: E402

KW, NW = 8, 8192
ap = argparse.ArgumentParser()
ap.add_argument("--config", choices=("c3", "c5slab", "c5", "c4"), default="c3")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--preload", type=int, default=400)
ap.add_argument("--modes", default="exact,fused")
ap.add_argument("--tuning", default="", help="extra key=value[,key=value] for every mode")
a = ap.parse_args()

L = lib()
L.hk_diag_reset.restype = ctypes.c_int
L.hk_diag_read.restype = ctypes.c_int
L.hk_diag_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]

if a.config == "c3":
    m = mesh.config_c3(v_end=5e5)
elif a.config == "c5slab":
    m = mesh.config_c5(layers=200)
elif a.config == "c5":
    m = mesh.config_c5(layers=1600)
else:
    m = mesh.config_c4()
diag, _ = m.lumped_mass()
sv = Solver(m, diag_M=diag)
sv.set_tuning("graph", 0)
for kv in filter(None, a.tuning.split(",")):
    k, v = kv.split("=")
    sv.set_tuning(k, int(v))
sv.step(1, a.preload)
t = a.preload + 1
for mode in a.modes.split(","):
    sv.set_tuning("elem_exact", 1 if mode == "exact" else 0)
    sv.step(t, 10)
    t += 10
    sv.sync()
    assert L.hk_diag_reset() == 0
    sv.step(t, a.steps)
    t += a.steps
    sv.sync()
    buf = (ctypes.c_uint64 * (KW * NW))()
    assert L.hk_diag_read(buf, KW * NW) == 0
    d = np.frombuffer(buf, dtype=np.uint64).reshape(NW, KW).astype(np.float64)
    live = d[:NW // 2, 5] > 0  # (rows NW/2.. hold the phase clocks of -DHK_DIAG_PHASE builds)
    n = int(live.sum())
    w = d[:n]
    launches = w[:, 5]
    loop, bar, pas, npass, batches = (w[:, j] / launches for j in range(5))
    hw = d[:n, 6].astype(np.int64)
    simd = (hw >> 4) & 3
    widx = np.arange(n) % 4
    blk = loop.reshape(-1, 4)
    out = {"mode": mode, "config": a.config, "waves": n, "launches": int(launches[0]), "steps": a.steps,
           "own_steps": sv.stat("own_steps"),
           "loop_kcycles_per_launch": {"mean": round(loop.mean() / 1e3, 2), "min": round(loop.min() / 1e3, 2),
                                       "max": round(loop.max() / 1e3, 2)},
           "barrier_frac": round(bar.sum() / loop.sum(), 4), "pass_frac": round(pas.sum() / loop.sum(), 4),
           "passes_per_launch": round(npass.mean(), 2), "batches_per_launch": round(batches.mean(), 2),
           "barrier_cycles_per_pass": round(bar.sum() / max(npass.sum(), 1), 1),
           "pass_cycles_per_pass": round(pas.sum() / max(npass.sum(), 1), 1),
           "compute_cycles_per_batch": round((loop - bar - pas).sum() / max(batches.sum(), 1), 1),
           "block_loop_spread_frac": round(float(np.mean((blk.max(1) - blk.min(1)) / blk.mean(1))), 4),
           "barrier_frac_by_wave_in_block": [round(bar[widx == i].sum() / loop[widx == i].sum(), 4) for i in range(4)],
           "pass_frac_by_wave_in_block": [round(pas[widx == i].sum() / loop[widx == i].sum(), 4) for i in range(4)],
           "compute_frac_by_wave_in_block": [round((loop - bar - pas)[widx == i].sum() / loop[widx == i].sum(), 4)
                                             for i in range(4)],
           "barrier_frac_by_simd": [round(bar[simd == i].sum() / max(loop[simd == i].sum(), 1), 4) for i in range(4)],
           "waves_by_simd": [int((simd == i).sum()) for i in range(4)]}
    ph = d[NW // 2:NW // 2 + n]
    if ph.sum() > 0:  # -DHK_DIAG_PHASE: the reference-order step's phases, cycles per batch
        names = ("issue", "node_wait+lds", "jacobian+P2", "bvbar", "de_chain", "stress", "force", "writeback")
        out["phase_cycles_per_batch"] = {nm: round(ph[:, j].sum() / max(batches.sum() * launches[0], 1), 1)
                                         for j, nm in enumerate(names)}
    print(json.dumps(out), flush=True)
sv.close()
