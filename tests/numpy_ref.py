"""Independent NumPy restatement of the reference element routine -- TEST INFRASTRUCTURE.

Written from v2/HAKAI_j.jl directly (not from the C oracle) with matrix algebra, so agreement with
oracle/hakai_oracle.c at ~1e-12 relative pins the C oracle against a second implementation.
"""
import numpy as np

DELTA = np.array([[-1, -1, -1], [1, -1, -1], [1, 1, -1], [-1, 1, -1],
                  [-1, -1, 1], [1, -1, 1], [1, 1, 1], [-1, 1, 1]], dtype=np.float64)   # v2/HAKAI_j.jl:1900-1907


def pusai():
    """cal_Pusai_hexa (v2/HAKAI_j.jl:1895-1943): P[k] is 3x8 dN/d(xi,eta,zeta) at Gauss point k."""
    g = 1.0 / np.sqrt(3.0)
    gc = np.array([[-g, -g, -g], [-g, -g, g], [-g, g, -g], [-g, g, g],
                   [g, -g, -g], [g, -g, g], [g, g, -g], [g, g, g]])
    P = np.zeros((8, 3, 8))
    for k in range(8):
        xi, eta, ze = gc[k]
        for i in range(8):
            d = DELTA[i]
            P[k, 0, i] = 1.0 / 8.0 * d[0] * (1.0 + eta * d[1]) * (1.0 + ze * d[2])
            P[k, 1, i] = 1.0 / 8.0 * d[1] * (1.0 + xi * d[0]) * (1.0 + ze * d[2])
            P[k, 2, i] = 1.0 / 8.0 * d[2] * (1.0 + xi * d[0]) * (1.0 + eta * d[1])
    return P


def dmat(young, poisson):
    """v2/HAKAI_j.jl:149-160."""
    d1, d2, d3 = 1.0 - poisson, poisson, (1.0 - 2.0 * poisson) / 2.0
    M = np.array([[d1, d2, d2, 0, 0, 0], [d2, d1, d2, 0, 0, 0], [d2, d2, d1, 0, 0, 0],
                  [0, 0, 0, d3, 0, 0], [0, 0, 0, 0, d3, 0], [0, 0, 0, 0, 0, d3]])
    return young / (1.0 + poisson) / (1.0 - 2.0 * poisson) * M


def b_std(P2):
    """Standard 6x24 strain-displacement matrix, Voigt (xx,yy,zz,xy,yz,xz), engineering shear."""
    B = np.zeros((6, 24))
    for i in range(8):
        px, py, pz = P2[:, i]
        B[0, 3 * i] = px
        B[1, 3 * i + 1] = py
        B[2, 3 * i + 2] = pz
        B[3, 3 * i], B[3, 3 * i + 1] = py, px
        B[4, 3 * i + 1], B[4, 3 * i + 2] = pz, py
        B[5, 3 * i], B[5, 3 * i + 2] = pz, px
    return B


def element_update(X, du, sig, eps, eqps, ys, mat):
    """One element (X 3x8 current position, du 24): returns new (sig, eps, eqps, ys) of its 8 GPs,
    Qe (24) and V. Follows cal_stress_hexa (v2/HAKAI_j.jl:1114-1353) with numpy linear algebra."""
    P = pusai()
    E, nu = mat.young, mat.poisson
    D = dmat(E, nu)
    G = E / 2.0 / (1.0 + nu)
    pl = np.asarray(mat.plastic).reshape(-1, 2)
    Hd = np.diff(pl[:, 0]) / np.diff(pl[:, 1]) if len(pl) > 1 else np.zeros(0)
    # B-bar (cal_BVbar_hexa, :1705-1784): |det| and inverse scaled by 1/|det|
    BV = np.zeros((6, 24))
    V = 0.0
    for k in range(8):
        J = P[k] @ X.T
        dJ = abs(np.linalg.det(J))
        V += dJ
        P2 = np.linalg.solve(J, P[k]) * np.sign(np.linalg.det(J))
        for r in range(3):
            BV[r] += (P2.T.reshape(-1) / 3.0) * dJ
    BV /= V
    Qe = np.zeros(24)
    sig, eps, eqps, ys = sig.copy(), eps.copy(), eqps.copy(), ys.copy()
    for k in range(8):
        J = P[k] @ X.T
        det = np.linalg.det(J)
        P2 = np.linalg.solve(J, P[k])
        B = b_std(P2)
        vol = np.tile(P2.T.reshape(-1), (3, 1)) / 3.0   # rows 1-3: -P2/3 + BVbar (cal_Bfinal :1482-1490)
        B[:3] += -vol + BV[:3]
        de = B @ du
        s = sig[k] + D @ de
        if len(pl):
            m = (s[0] + s[1] + s[2]) / 3.0
            dev = s - np.array([m, m, m, 0, 0, 0])
            q = np.sqrt(1.5 * (dev[0] ** 2 + dev[1] ** 2 + dev[2] ** 2 + 2 * dev[3] ** 2 + 2 * dev[4] ** 2
                               + 2 * dev[5] ** 2))
            if q > ys[k]:
                p = len(pl) - 2
                for j in range(1, len(pl)):
                    if eqps[k] <= pl[j, 1]:
                        p = j - 1
                        break
                H = Hd[p]
                dep = (q - ys[k]) / (3 * G + H)
                s = dev * (ys[k] + H * dep) / q + np.array([m, m, m, 0, 0, 0])
                eqps[k] += dep
                ys[k] += H * dep
        eps[k] = eps[k] + de
        sig[k] = s
        Qe += det * (B.T @ s)
    return sig, eps, eqps, ys, Qe, V


def triax(s):
    """cal_triax_stress via numpy eigvalsh."""
    T = np.array([[s[0], s[3], s[5]], [s[3], s[1], s[4]], [s[5], s[4], s[2]]])
    p = np.linalg.eigvalsh(T)
    oeq = np.sqrt(0.5 * ((p[0] - p[1]) ** 2 + (p[1] - p[2]) ** 2 + (p[2] - p[0]) ** 2))
    return 0.0 if oeq < 1e-10 else (p.sum() / 3.0) / oeq
