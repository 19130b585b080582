"""The exact element kernel's x/3.0 (div3 in csrc/hakai_kernels.hip: q = x*y, y = RN(1/3), then
q + (x - 3q)*y with fused multiply-adds) must equal IEEE division bit for bit. Checked here on the
CPU with the same three operations (gcc, -mfma) against `x / 3.0` on 2e7 doubles: random bit
patterns over the exponent range the kernel meets, multiples of 3 (exact quotients), values next to
powers of two, and signed zeros."""
import ctypes
import os
import subprocess

import numpy as np

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <string.h>
static double div3(double x) {
    const double y = 1.0 / 3.0;
    const double q = x * y;
    const double r = fma(-q, 3.0, x);
    const double q1 = fma(r, y, q);
    return x == 0.0 ? x : q1;
}
/* number of x with div3(x) != x / 3.0 (bitwise) */
int64_t check(const double* x, int64_t n) {
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) {
        const double a = div3(x[i]), b = x[i] / 3.0;
        if (memcmp(&a, &b, sizeof a) != 0) ++bad;
    }
    return bad;
}
"""


def _lib(tmp_path):
    c = tmp_path / "div3.c"
    so = tmp_path / "div3.so"
    c.write_text(SRC)
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", "-shared", "-fPIC", "-o", str(so), str(c), "-lm"],
                   check=True)
    L = ctypes.CDLL(str(so))
    L.check.restype = ctypes.c_int64
    L.check.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    return L


def test_div3_equals_ieee_division(tmp_path):
    L = _lib(tmp_path)
    rng = np.random.default_rng(0)
    n = 10_000_000
    # random mantissas, exponents 2^-200 .. 2^200, both signs
    mant = rng.integers(0, 1 << 52, size=n, dtype=np.uint64)
    expo = rng.integers(1023 - 200, 1023 + 200, size=n, dtype=np.uint64)
    sign = rng.integers(0, 2, size=n, dtype=np.uint64)
    x = ((sign << np.uint64(63)) | (expo << np.uint64(52)) | mant).view(np.float64)
    # exact quotients, neighbours of powers of two and of multiples of 3, signed zeros
    m3 = (rng.integers(1, 1 << 50, size=n // 4) * 3).astype(np.float64) * np.exp2(rng.integers(-60, 60, n // 4))
    p2 = np.exp2(rng.integers(-100, 100, n // 4).astype(np.float64))
    near = np.concatenate([np.nextafter(p2, 0), np.nextafter(p2, np.inf), p2 * 3, np.nextafter(p2 * 3, 0)])
    extra = np.concatenate([m3, np.nextafter(m3, 0), np.nextafter(m3, np.inf), near, [0.0, -0.0, 1.0, -3.0]])
    for arr in (x, extra):
        a = np.ascontiguousarray(arr, np.float64)
        assert L.check(a.ctypes.data, a.size) == 0
