"""The VTK writer (write_vtk, v2/HAKAI_j.jl:3517-3717) on the CPU: the parallel to_chars writer, its
asynchronous submit and zero-copy acquire/commit paths all produce the bytes of a plain serial
"%1.6e" rendering of the reference's file layout, for any thread count. Host code only, no GPU."""
import ctypes
import os

import numpy as np
import pytest

import hakai
from hakai import _abi
from hakai._abi import check, ptr

I64 = ctypes.c_int64


def serial_vtk(coordmat, elementmat, flag, disp, velo, ns, nn, ne, nm, nt):
    """Line-by-line restatement of write_vtk's output (v2/HAKAI_j.jl:3564-3712) with Python's
    printf-style "%1.6e" (the reference's @printf format) and its |x| < 1e-16 flush (:3530-3558)."""
    def f16(x):
        return 0.0 if abs(x) < 1e-16 else x

    def e(x):  # Julia's @printf spells non-finite values NaN / Inf / -Inf
        if not np.isfinite(x):
            return "NaN" if np.isnan(x) else ("Inf" if x > 0 else "-Inf")
        return "%1.6e" % x

    nN, nE = coordmat.size // 3, flag.size
    out = ["# vtk DataFile Version 2.0\nTest\nASCII\nDATASET UNSTRUCTURED_GRID\n", f"POINTS {nN} float\n"]
    X = coordmat.reshape(-1, 3)
    out += [f"{e(a)} {e(b)} {e(c)}\n" for a, b, c in X]
    draw = int(flag.sum())
    out.append(f"CELLS {draw} {draw * 9}\n")
    em = elementmat.reshape(-1, 8)
    out += ["8 " + " ".join(str(int(v) - 1) for v in em[i]) + "\n" for i in range(nE) if flag[i] == 1]
    out.append(f"CELL_TYPES {draw}\n")
    out += ["12\n"] * draw
    out.append(f"POINT_DATA {nN}\nVECTORS DISPLACEMENT float\n")
    out += [f"{e(f16(a))} {e(f16(b))} {e(f16(c))}\n" for a, b, c in disp.reshape(-1, 3)]

    def scal(name, vals):
        out.append(f"SCALARS {name} float 1\nLOOKUP_TABLE default\n")
        out.extend(e(f16(v)) + "\n" for v in vals)

    for c, n in enumerate(("Vx", "Vy", "Vz")):
        scal(n, velo.reshape(-1, 3)[:, c])
    for c, n in enumerate(("E11", "E22", "E33", "E12", "E23", "E13")):
        scal(n, nn.reshape(-1, 6)[:, c])
    scal("EQ_PSTRAIN", ne)
    for c, n in enumerate(("S11", "S22", "S33", "S12", "S23", "S13")):
        scal(n, ns.reshape(-1, 6)[:, c])
    scal("MISES_STRESS", nm)
    scal("TRIAX_STRESS", nt)
    return "".join(out).encode()


def random_fields(nN, nE, seed):
    rng = np.random.default_rng(seed)

    def vals(n):
        # mixed magnitudes, exact zeros, values around the 1e-16 flush, round-half cases, huge/tiny
        v = rng.standard_normal(n) * 10.0 ** rng.integers(-20, 12, n)
        v[rng.random(n) < 0.05] = 0.0
        k = rng.random(n) < 0.02
        v[k] = 1e-16 * rng.choice([-1.0, 1.0, 0.999999, 1.000001], int(k.sum()))
        k = rng.random(n) < 0.02
        v[k] = rng.integers(0, 10 ** 8, int(k.sum())) / 1e7 + 5e-8  # ties in the 7th digit
        v[rng.random(n) < 0.001] = 1e-310  # subnormal
        v[rng.random(n) < 0.001] = -1.7e308
        return v

    coord = vals(3 * nN)
    em = rng.integers(1, nN + 1, 8 * nE).astype(np.int64)
    flag = (rng.random(nE) < 0.8).astype(np.int64)
    return dict(coordmat=coord, elementmat=em, flag=flag, disp=vals(3 * nN), velo=vals(3 * nN), ns=vals(6 * nN),
                nn=vals(6 * nN), ne=vals(nN), nm=vals(nN), nt=vals(nN))


def field_ptrs(d):
    return (ptr(d["flag"], I64), ptr(d["disp"]), ptr(d["velo"]), ptr(d["ns"]), ptr(d["nn"]), ptr(d["ne"]),
            ptr(d["nm"]), ptr(d["nt"]))


@pytest.mark.parametrize("nN,nE", [(1, 1), (37, 11), (20000, 9000)])
def test_write_vtk_matches_serial_printf(tmp_path, nN, nE):
    d = random_fields(nN, nE, seed=nN)
    check(hakai.lib().hakai_write_vtk(str(tmp_path).encode(), 7, nN, ptr(d["coordmat"]), nE,
                                      ptr(d["elementmat"], I64), *field_ptrs(d)))
    got = (tmp_path / "file007.vtk").read_bytes()
    want = serial_vtk(d["coordmat"], d["elementmat"], d["flag"], d["disp"], d["velo"], d["ns"], d["nn"], d["ne"],
                      d["nm"], d["nt"])
    assert got == want


def test_write_vtk_non_finite_values_as_julia(tmp_path):
    """A diverged state: NaN and +-Inf print as Julia's @printf does ("NaN", "Inf", "-Inf")."""
    d = random_fields(37, 11, seed=5)
    d["disp"][::7] = np.nan
    d["velo"][1::5] = np.inf
    d["ns"][2::3] = -np.inf
    d["nm"][0] = -np.nan
    check(hakai.lib().hakai_write_vtk(str(tmp_path).encode(), 1, 37, ptr(d["coordmat"]), 11,
                                      ptr(d["elementmat"], I64), *field_ptrs(d)))
    got = (tmp_path / "file001.vtk").read_bytes()
    want = serial_vtk(d["coordmat"], d["elementmat"], d["flag"], d["disp"], d["velo"], d["ns"], d["nn"], d["ne"],
                      d["nm"], d["nt"])
    assert got == want
    assert b"NaN" in got and b"\nInf\n" in got and b"-Inf" in got and b"nan" not in got and b"inf" not in got


@pytest.mark.parametrize("threads", [1, 3, 16])
def test_async_writer_sequence_and_zero_copy(tmp_path, threads):
    """Three files through one writer (submit, then acquire/commit), each byte-identical to the
    serial rendering of its own snapshot even though the caller overwrites its arrays right after
    submit returns."""
    L = hakai.lib()
    nN, nE = 12345, 5000
    d0 = random_fields(nN, nE, seed=1)
    w = ctypes.c_void_p()
    check(L.hakai_vtk_writer_create(ctypes.byref(w), str(tmp_path).encode(), nN, ptr(d0["coordmat"]), nE,
                                    ptr(d0["elementmat"], I64), threads))
    try:
        want = {}
        for idx in range(2):
            d = random_fields(nN, nE, seed=10 + idx)
            check(L.hakai_vtk_writer_submit(w, idx, *field_ptrs(d)))
            want[idx] = serial_vtk(d0["coordmat"], d0["elementmat"], d["flag"], d["disp"], d["velo"], d["ns"],
                                   d["nn"], d["ne"], d["nm"], d["nt"])
            for k in ("disp", "velo", "ns", "nn", "ne", "nm", "nt"):
                d[k][:] = np.nan  # the writer works on its own snapshot
            d["flag"][:] = 0
        # zero-copy: fill the writer's buffers in place
        a = (ctypes.c_void_p * 8)()
        check(L.hakai_vtk_writer_acquire(w, ctypes.byref(a)))
        d = random_fields(nN, nE, seed=99)
        sizes = [nE, 3 * nN, 3 * nN, 6 * nN, 6 * nN, nN, nN, nN]
        keys = ["flag", "disp", "velo", "ns", "nn", "ne", "nm", "nt"]
        for p, n, k in zip(a, sizes, keys):
            ct = ctypes.c_int64 if k == "flag" else ctypes.c_double
            dst = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ct)), shape=(n,))
            dst[:] = d[k]
        check(L.hakai_vtk_writer_commit(w, 2))
        want[2] = serial_vtk(d0["coordmat"], d0["elementmat"], d["flag"], d["disp"], d["velo"], d["ns"], d["nn"],
                             d["ne"], d["nm"], d["nt"])
        check(L.hakai_vtk_writer_wait(w))
    finally:
        L.hakai_vtk_writer_destroy(w)
    for idx, b in want.items():
        assert (tmp_path / f"file{idx:03d}.vtk").read_bytes() == b, idx


def test_async_writer_error_surfaces(tmp_path):
    """A file that cannot be created fails at wait (or the next submit) with HAKAI_ERR_IO."""
    L = hakai.lib()
    blocker = tmp_path / "not_a_dir"
    blocker.write_text("x")
    d = random_fields(10, 3, seed=5)
    w = ctypes.c_void_p()
    check(L.hakai_vtk_writer_create(ctypes.byref(w), str(blocker / "sub").encode(), 10, ptr(d["coordmat"]), 3,
                                    ptr(d["elementmat"], I64), 2))
    try:
        check(L.hakai_vtk_writer_submit(w, 0, *field_ptrs(d)))
        with pytest.raises(hakai.HakaiError) as ei:
            check(L.hakai_vtk_writer_wait(w))
        assert ei.value.code == _abi.HAKAI_ERR_IO
        check(L.hakai_vtk_writer_wait(w))  # the error is reported once
    finally:
        L.hakai_vtk_writer_destroy(w)
