#!/usr/bin/env python3
"""Kernel resource report: VGPRs, AGPRs, SGPRs, spills, static LDS and the compiler's waves per SIMD.

Compiles a HIP source for gfx950 with the Makefile's flags (its -ffp-contract per file) and `-Rpass-analysis=kernel-resource-usage`
(the compiler's own per-kernel report, no GPU needed) and prints one JSON object. The element
kernel's template arguments are named (`hk::k_element_pipe<DO_DELETE, STORE_TRIAX, ANY_PLASTIC,
LDS_MATS, NT, EXACT, OS>`, csrc/hakai_kernels.hip), so the two instantiations the C3 bench times are
easy to find: fused `<1,0,1,1,3,0,2>` and reference order `<1,0,1,1,3,1,2>` (its owner path; the fe
fallback is OS = 0).

    python tools/kernel_resources.py [--src csrc/hakai_kernels.hip] [--remarks FILE] > out.json

LDS: the static `__shared__` bytes only; the launch adds the owner-sum slots and staged materials
as dynamic LDS (launch_pipe), which the "lds_dynamic_note" field says. Waves per SIMD are the
compiler's figure (VGPR- and static-LDS-limited)."""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hakai-fem_amd")
FLAGS = ["--offload-arch=gfx950", "-std=c++17", "-O3", "-fPIC", "-munsafe-fp-atomics"]
CONTRACT = {"hakai_kernels.hip": "-ffp-contract=on", "hakai_contact.hip": "-ffp-contract=off"}  # as the Makefile
FIELDS = {"TotalSGPRs": "sgprs", "VGPRs": "vgprs", "AGPRs": "agprs", "ScratchSize [bytes/lane]": "scratch_bytes_per_lane",
          "Occupancy [waves/SIMD]": "waves_per_simd", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill",
          "LDS Size [bytes/block]": "lds_static_bytes", "Dynamic Stack": "dynamic_stack"}
PIPE_ARGS = ("DO_DELETE", "STORE_TRIAX", "ANY_PLASTIC", "LDS_MATS", "NT", "EXACT", "OS")


def parse(text):
    """Per-kernel records from the compiler's remarks (one 'Function Name:' line opens a record)."""
    out, cur = [], None
    for line in text.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass-analysis=kernel-resource-usage\]", line)
        if not m:
            continue
        body = m.group(1).strip()
        if body.startswith("Function Name:"):
            cur = {"symbol": body.split(":", 1)[1].strip()}
            out.append(cur)
            continue
        if cur is None or ":" not in body:
            continue
        k, v = (s.strip() for s in body.rsplit(":", 1))
        if k in FIELDS:
            cur[FIELDS[k]] = (v == "True") if k == "Dynamic Stack" else int(v)
    for r in out:
        r.update(describe(r["symbol"]))
    return out


def describe(sym):
    """Readable name; the element kernel's template arguments by name."""
    m = re.match(r"_ZN2hk(\d+)(\w+?)I(.*)EEvNS_\d+\w+E$", sym)
    if not m:
        m2 = re.match(r"_ZN2hk(\d+)", sym)
        if m2:
            n = int(m2.group(1))
            return {"kernel": sym[len(m2.group(0)):len(m2.group(0)) + n]}
        return {"kernel": sym}
    n = int(m.group(1))
    name = (m.group(2) + "I" + m.group(3))[:n]
    targs = re.findall(r"L([bi])(\d+)E", sym[len("_ZN2hk") + len(m.group(1)) + n:])
    vals = [bool(int(v)) if t == "b" else int(v) for t, v in targs]
    d = {"kernel": name, "template_args": vals}
    if name == "k_element_pipe" and len(vals) == len(PIPE_ARGS):
        d["args"] = dict(zip(PIPE_ARGS, vals))
        d["mode"] = "reference_order" if d["args"]["EXACT"] else "fused"
        d["assembly"] = f"owner OS={d['args']['OS']}" if d["args"]["OS"] else "fe"
    return d


def flags(src):
    return FLAGS + ([CONTRACT[os.path.basename(src)]] if os.path.basename(src) in CONTRACT else [])


def compile_remarks(src):
    with tempfile.TemporaryDirectory() as td:
        p = subprocess.run(["/opt/rocm/bin/hipcc", *flags(src), "-I", os.path.join(PKG, "csrc"), "-c", src,
                            "-o", os.path.join(td, "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
    if p.returncode:
        sys.exit(p.stderr[-4000:])
    return p.stderr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(PKG, "csrc", "hakai_kernels.hip"))
    ap.add_argument("--remarks", help="parse this saved remarks file instead of compiling")
    a = ap.parse_args()
    text = open(a.remarks).read() if a.remarks else compile_remarks(a.src)
    ks = parse(text)
    bench = {}
    for r in ks:
        if r.get("args") and r["args"]["DO_DELETE"] and not r["args"]["STORE_TRIAX"] and r["args"]["NT"] == 3 \
                and r["args"]["ANY_PLASTIC"] and r["args"]["LDS_MATS"]:
            bench[f"{r['mode']} {r['assembly']}"] = {k: r.get(k) for k in ("vgprs", "agprs", "sgprs", "vgpr_spill",
                                                                          "sgpr_spill", "scratch_bytes_per_lane",
                                                                          "lds_static_bytes", "waves_per_simd")}
    print(json.dumps({"source": os.path.relpath(a.src, ROOT), "arch": "gfx950", "flags": flags(a.src),
                      "c3_bench_instantiations": bench,
                      "lds_dynamic_note": "static __shared__ only; launch_pipe adds owner-sum slots and staged "
                                          "materials as dynamic LDS",
                      "kernels": ks}, indent=1))


if __name__ == "__main__":
    main()
