"""The Julia binding (julia/HakaiHIP.jl) against the C header (include/hakai_hip.h), on CPU.

Julia is not installed here or on the GPU box, so the shim cannot run; this test checks it
mechanically instead: every `ccall((:hakai_*, lib), Ret, (ArgTypes...), ...)` names a function the
header declares, with the same number of arguments and, argument by argument, a Julia type that
passes the C type (Cint <-> int, Int64 <-> int64_t, Ptr{Float64} or Ref{Float64} <-> double*, ...),
and every Julia struct mirrors its C struct field by field. It also checks that the whole-loop seam
binds what SURVEY §8(b) / VERDICT r1 listed (BCs, downloads, deletions, node averages, VTK)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hakai_hip.h")
SHIM = os.path.join(ROOT, "julia", "HakaiHIP.jl")

# C type (normalised) -> Julia types that pass it through ccall
SCALAR = {"int": {"Cint"}, "int32_t": {"Int32"}, "int64_t": {"Int64"}, "uint32_t": {"UInt32"},
          "double": {"Float64"}}
POINTEE = {"double": "Float64", "int64_t": "Int64", "int32_t": "Int32", "uint8_t": "UInt8", "int": "Cint",
           "hakai_material_t": "Material", "hakai_bc_t": "BC", "hakai_state_t": "State"}
OPAQUE = {"hakai_ctx", "hakai_vtk_writer"}


def _strip_comments(src):
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def c_prototypes():
    src = _strip_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"((?:const\s+)?[A-Za-z_]\w*\s*\**)\s*\b(hakai_\w+)\s*\(([^)]*)\)\s*;", src, flags=re.S):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        params = [] if args.strip() in ("", "void") else [a.strip() for a in args.split(",")]
        out[name] = (" ".join(ret.split()), params)
    return out


def c_param_type(p):
    """'const double* coordmat' -> ('double', 1); 'uint8_t id[128]' -> ('uint8_t', 1)."""
    p = p.replace("const ", "")
    arr = "[" in p
    p = re.sub(r"\[.*\]", "", p)
    stars = p.count("*")
    toks = p.replace("*", " ").split()
    base = toks[0]
    return base, stars + (1 if arr else 0)


def julia_accepts(c, jl):
    base, stars = c
    jl = jl.replace(" ", "")
    if stars == 0:
        return jl in SCALAR[base]
    if base == "char" and stars == 1:
        return jl == "Cstring"
    if base in OPAQUE:
        if stars == 1:
            return jl == "Ptr{Cvoid}"
        return jl in ("Ref{Ptr{Cvoid}}", "Ptr{Ptr{Cvoid}}")
    t = POINTEE[base]
    return stars == 1 and jl in (f"Ptr{{{t}}}", f"Ref{{{t}}}")


def julia_ccalls():
    src = open(SHIM).read()
    src = re.sub(r"#[^\n]*", "", src)
    calls = []
    for m in re.finditer(r"ccall\(\(:(\w+),\s*lib\),\s*", src):
        i = m.end()
        # return type up to the next top-level comma
        depth, j = 0, i
        while not (src[j] == "," and depth == 0):
            depth += src[j] in "({"
            depth -= src[j] in ")}"
            j += 1
        ret = src[i:j].strip()
        k = src.index("(", j)
        depth, e = 0, k
        while True:
            depth += src[e] in "({"
            depth -= src[e] in ")}"
            if depth == 0:
                break
            e += 1
        inner = src[k + 1:e]
        args, depth, cur = [], 0, ""
        for ch in inner:
            if ch == "," and depth == 0:
                args.append(cur.strip())
                cur = ""
                continue
            depth += ch in "({"
            depth -= ch in ")}"
            cur += ch
        if cur.strip():
            args.append(cur.strip())
        calls.append((m.group(1), ret, args))
    return calls


def test_every_ccall_matches_the_header():
    protos = c_prototypes()
    calls = julia_ccalls()
    assert len(calls) >= 30
    for name, ret, args in calls:
        assert name in protos, f"{name}: not declared in include/hakai_hip.h"
        cret, params = protos[name]
        want_ret = {"int": "Cint", "void": "Cvoid", "const char*": "Cstring"}[cret.replace(" *", "*")]
        assert ret == want_ret, (name, ret, cret)
        assert len(args) == len(params), f"{name}: {len(args)} Julia argument types, header has {len(params)}"
        for jl, p in zip(args, params):
            assert julia_accepts(c_param_type(p), jl), f"{name}: Julia {jl} does not pass C '{p}'"


def c_struct_fields(name):
    src = _strip_comments(open(HEADER).read())
    m = re.search(r"typedef\s+struct\s*\{([^{}]*)\}\s*" + name + r"\s*;", src, flags=re.S)
    fields = []
    for decl in m.group(1).split(";"):
        decl = decl.strip()
        if not decl:
            continue
        first, *more = [d.strip() for d in decl.split(",")]   # "double density, young, poisson"
        base = c_param_type(first)
        fields.append((re.split(r"[\s*]+", first)[-1], base))
        fields += [(d.replace("*", "").strip(), (base[0], d.count("*"))) for d in more]
    return fields


def julia_struct_fields(name):
    src = open(SHIM).read()
    m = re.search(r"\nstruct\s+" + name + r"\b[^\n]*\n(.*?)\nend", src, flags=re.S)
    out = []
    for line in m.group(1).split("\n"):
        line = line.split("#")[0].strip()
        if line:
            f, t = line.split("::")
            out.append((f.strip(), t.strip()))
    return out


@pytest.mark.parametrize("c_name,jl_name", [("hakai_material_t", "Material"), ("hakai_bc_t", "BC"),
                                            ("hakai_state_t", "State")])
def test_julia_structs_mirror_c_structs(c_name, jl_name):
    cf, jf = c_struct_fields(c_name), julia_struct_fields(jl_name)
    assert [f for f, _ in cf] == [f for f, _ in jf], (c_name, cf, jf)
    for (f, ct), (_, jt) in zip(cf, jf):
        base, stars = ct
        ok = julia_accepts(ct, jt) and not jt.startswith("Ref")
        assert ok, f"{c_name}.{f}: Julia {jt} vs C {base}{'*' * stars}"


def test_loop_seam_is_bound():
    """The whole-loop replacement binds everything the reference's hakai() loop touches
    (v2/HAKAI_j.jl:487-951): setup, BCs, IC, contact, stepping, downloads at output cadence,
    deletion log, node averages and VTK output; the driver surface and the literal drop-ins."""
    names = {n for n, _, _ in julia_ccalls()}
    need = {"hakai_create", "hakai_destroy", "hakai_upload_model", "hakai_set_bc", "hakai_reset_state",
            "hakai_step", "hakai_download_state", "hakai_upload_state", "hakai_deleted",
            "hakai_node_stress_strain", "hakai_set_contact_cp", "hakai_set_contact_params", "hakai_set_tuning",
            "hakai_vtk_writer_create", "hakai_vtk_writer_submit", "hakai_vtk_writer_wait",
            "hakai_vtk_writer_destroy", "hakai_run_inp", "hakai_stress_hexa", "hakai_triax_stress",
            "hakai_lumped_mass", "hakai_comm_init", "hakai_set_interface", "hakai_set_element_offset"}
    assert need <= names, sorted(need - names)
    src = open(SHIM).read()
    assert "function hakai_gpu(" in src and "set_bc(c, MODEL.BC)" in src and "reset_state(c, MODEL.IC" in src
