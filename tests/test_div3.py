"""The exact element kernel's divisions must equal IEEE division bit for bit:
  * x/3.0 (div3 in csrc/hakai_kernels.hip since round 6: RN(x*yh + RN(x*yl)), yh = RN(1/3),
    yl = RN(1/3 - yh), one multiply and one fused multiply-add), checked against `x / 3.0` on 2e7
    doubles: random bit patterns over the exponent range the kernel meets, multiples of 3 (exact
    quotients), values next to powers of two, signed zeros (bit for bit: -0/3 = -0);
  * a/b given rb = RN(1/b) (div_cr: two Newton-Markstein corrections of a*rb), checked against
    `a / b` on 2e7 random pairs over the kernel's exponent range and on pairs whose quotient lies
    next to a rounding midpoint (the hard cases of correct rounding).
Same operations on the CPU (gcc, -mfma, no contraction)."""
import ctypes
import os
import subprocess

import numpy as np

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <string.h>
static double div3(double x) {
    const double yh = 1.0 / 3.0;
    const double yl = 0x1.5555555555555p-56;  /* RN(1/3 - yh) */
    return fma(x, yh, x * yl);
}
/* number of x with div3(x) != x / 3.0 (bitwise, signed zeros included) */
int64_t check(const double* x, int64_t n) {
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) {
        const double a = div3(x[i]), b = x[i] / 3.0;
        if (memcmp(&a, &b, sizeof a) != 0) ++bad;
    }
    return bad;
}
static double div_cr(double a, double b, double rb) {
    const double q0 = a * rb;
    const double q1 = fma(fma(-q0, b, a), rb, q0);
    return fma(fma(-q1, b, a), rb, q1);
}
/* pairs with div_cr(a, b) != a / b (bitwise); *one: pairs where ONE correction would not do */
int64_t check_div(const double* a, const double* b, int64_t n, int64_t* one) {
    int64_t bad = 0, b1 = 0;
    for (int64_t i = 0; i < n; ++i) {
        const double rb = 1.0 / b[i];
        const double x = div_cr(a[i], b[i], rb), y = a[i] / b[i];
        const double q0 = a[i] * rb, q1 = fma(fma(-q0, b[i], a[i]), rb, q0);
        if (memcmp(&x, &y, sizeof x) != 0) ++bad;
        if (memcmp(&q1, &y, sizeof q1) != 0) ++b1;
    }
    *one = b1;
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
    L.check_div.restype = ctypes.c_int64
    L.check_div.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    return L


def _rand_doubles(rng, n, lo, hi, signed=True):
    mant = rng.integers(0, 1 << 52, size=n, dtype=np.uint64)
    expo = rng.integers(1023 + lo, 1023 + hi, size=n, dtype=np.uint64)
    sign = rng.integers(0, 2, size=n, dtype=np.uint64) if signed else np.zeros(n, np.uint64)
    return ((sign << np.uint64(63)) | (expo << np.uint64(52)) | mant).view(np.float64)


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


def test_div_cr_equals_ieee_division(tmp_path):
    L = _lib(tmp_path)
    rng = np.random.default_rng(1)
    n = 10_000_000
    one = ctypes.c_int64(0)
    # random pairs: numerators over the stresses' range, positive divisors (q, V of the kernel)
    a = _rand_doubles(rng, n, -60, 60)
    b = _rand_doubles(rng, n, -30, 30, signed=False)
    assert L.check_div(a.ctypes.data, b.ctypes.data, n, ctypes.byref(one)) == 0
    # quotients next to a rounding midpoint: a = RN(b * (q + ulp(q)/2)) for random q, b
    m = n // 2
    q = _rand_doubles(rng, m, -20, 20)
    b2 = _rand_doubles(rng, m, -20, 20, signed=False)
    mid = q.astype(np.longdouble) + (np.spacing(q).astype(np.longdouble) / 2)
    a2 = np.ascontiguousarray((b2.astype(np.longdouble) * mid).astype(np.float64))
    for da in (0, 1, -1):  # and their neighbours
        aa = np.ascontiguousarray(a2 if da == 0 else np.nextafter(a2, da * np.inf))
        assert L.check_div(aa.ctypes.data, b2.ctypes.data, m, ctypes.byref(one)) == 0
    # exact quotients and zeros
    b3 = _rand_doubles(rng, m, -20, 20, signed=False)
    q3 = (rng.integers(1, 1 << 40, size=m).astype(np.float64)) * np.exp2(rng.integers(-30, 30, m))
    a3 = np.ascontiguousarray(q3 * b3)
    ok = (a3 / b3) == q3
    a3, b3 = np.ascontiguousarray(a3[ok]), np.ascontiguousarray(b3[ok])
    assert L.check_div(a3.ctypes.data, b3.ctypes.data, a3.size, ctypes.byref(one)) == 0
