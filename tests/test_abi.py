"""CPU checks of the C-ABI boundary: the library loads, exports every function include/hakai_hip.h
declares, and refuses compute without a gfx950 device (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import hakai
from hakai import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hakai_hip.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hakai_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    assert declared_functions() == sorted(_abi.exported_symbols())


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (hakai_[a-z0-9_]+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    L = hakai.lib()
    for f in declared_functions():
        assert hasattr(L, f)


def test_abi_version_and_errors():
    L = hakai.lib()
    assert L.hakai_abi_version() == 1
    with pytest.raises(hakai.HakaiError) as ei:
        _abi.check(L.hakai_inp_read(b"/nonexistent.inp", ctypes.byref(ctypes.POINTER(_abi.InpModelT)())))
    assert ei.value.code == _abi.HAKAI_ERR_IO


def test_no_cpu_fallback_without_device():
    if hakai.device_count() > 0:
        pytest.skip("a GPU is visible")
    ctx = ctypes.c_void_p()
    rc = hakai.lib().hakai_create(ctypes.byref(ctx), 0)
    assert rc == _abi.HAKAI_ERR_DEVICE
    assert b"no CPU fallback" in hakai.lib().hakai_last_error()
    Qe = np.zeros((1, 24))
    z = np.zeros((8, 6))
    with pytest.raises(hakai.HakaiError):
        hakai.cal_triax_stress(z, np.zeros(8))


def test_struct_layouts_match_header():
    """ctypes mirrors of the header structs: field offsets follow the C ABI (x86-64 SysV)."""
    assert ctypes.sizeof(_abi.MaterialT) == 3 * 8 + 8 + 8 + 8 + 8
    assert ctypes.sizeof(_abi.BCT) == 8 + 8 * 8
    assert ctypes.sizeof(_abi.StateT) == 11 * 8
    assert _abi.InpModelT.bc.offset % 8 == 0


def test_lumped_mass_host_helper():
    from hakai import mesh
    m = mesh.tensile5e_model()
    diag, vol = m.lumped_mass()
    assert np.allclose(vol, 500.0, rtol=1e-12)              # 10 x 10 x 5 mm bricks
    assert np.isclose(diag[0::3].sum(), 7.8e-9 * 2500.0, rtol=1e-12)
    assert np.array_equal(diag[0::3], diag[1::3]) and np.array_equal(diag[0::3], diag[2::3])
