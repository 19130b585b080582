"""Independent pure-Python restatement of HAKAI v0.0.2's all-exterior contact (tests only).

Written from v2/HAKAI_j.jl directly, loop for loop, to pin the C oracle (oracle/hakai_oracle_contact.c):
  get_element_face :1944-1992, get_surface_triangle :1996-2164 (its O(F^2) scan, kept literally),
  add_surface_triangle :2167-2245 with the CT update of :766-804, cal_contact_force :2248-2706.
Float128 accumulation (:435) is replaced by exact rational accumulation (fractions.Fraction) rounded
once to float, i.e. the correctly rounded sum.
"""
from __future__ import annotations

import math
from fractions import Fraction

import numpy as np


def element_faces(coord, elem, e_ids):
    """faces (F,4) oriented, sorted keys (F,4), owner element (1-based) for elements e_ids (1-based)."""
    faces, keys, owner = [], [], []
    for e in e_ids:
        el = [int(x) for x in elem[e - 1]]
        fl = [el[0:4], el[4:8], [el[0], el[1], el[5], el[4]], [el[1], el[2], el[6], el[5]],
              [el[2], el[3], el[7], el[6]], [el[3], el[0], el[4], el[7]]]
        ctr = [0.0, 0.0, 0.0]
        for n in el:
            for c in range(3):
                ctr[c] += coord[n - 1, c]
        ctr = [x / 8 for x in ctr]
        for f in fl:
            x1, x2, x4 = coord[f[0] - 1], coord[f[1] - 1], coord[f[3] - 1]
            v1 = [x2[c] - x1[c] for c in range(3)]
            v2 = [x4[c] - x1[c] for c in range(3)]
            nv = [v1[1] * v2[2] - v1[2] * v2[1], v1[2] * v2[0] - v1[0] * v2[2], v1[0] * v2[1] - v1[1] * v2[0]]
            vc = [ctr[c] - x1[c] for c in range(3)]
            if nv[0] * vc[0] + nv[1] * vc[1] + nv[2] * vc[2] > 0.:
                f = [f[0], f[3], f[2], f[1]]
            faces.append(f)
            keys.append(sorted(f))
            owner.append(e)
    return faces, keys, owner


def surface_triangle(faces, keys, owner, contact=None, e0=0, nE=None):
    """contact: instance-local 1-based element list of a *Contact Pair surface (None = all);
    filtering applies only when its length differs from nE (v2/HAKAI_j.jl:2087)."""
    F = len(faces)
    dp = []
    surf = []
    for j in range(F - 1):               # j = 1 : nE*6-1
        if j in dp:
            continue
        u = True
        for k in range(j + 1, F):
            if keys[j] == keys[k]:
                u = False
                dp.append(k)
                break
        if u:
            surf.append((faces[j], owner[j]))
    if contact is not None and len(contact) != nE:
        cs = set(int(x) for x in contact)
        surf = [(f, e) for f, e in surf if e - e0 in cs]
    tri, tri_e = [], []
    for f, e in surf:
        tri += [[f[0], f[1], f[2]], [f[2], f[3], f[0]]]
        tri_e += [e, e]
    nodes = sorted(set(n for t in tri for n in t))
    return tri, tri_e, nodes


class ContactRef:
    def __init__(self, model):
        coord, elem = model.coordmat, model.elementmat
        inst = model.element_instance if model.element_instance is not None else np.ones(model.nElement, np.int64)
        ni = int(inst.max())
        self.inst_elems = [[e + 1 for e in range(model.nElement) if inst[e] == i + 1] for i in range(ni)]
        self.inst = []
        for i in range(ni):
            self.inst.append(element_faces(coord, elem, self.inst_elems[i]))
        young = [model.materials[model.element_material[es[0] - 1] - 1].young for es in self.inst_elems]
        cps = getattr(model, "contact_pairs", None)
        if cps:
            cp = [(c[0][0] - 1, c[1][0] - 1, list(c[0][1]), list(c[1][1])) for c in cps]
        elif ni > 1:
            cp = [(i, j, None, None) for i in range(ni) for j in range(i if model.contact_flag == 2 else i + 1, ni)]
        else:
            cp = [(0, 0, None, None)]
        self.ct = []
        for a, b, la, lb in cp:
            for (pi, pj, li, lj) in ([(a, b, la, lb)] if a == b else [(a, b, la, lb), (b, a, lb, la)]):
                e0i, e0j = self.inst_elems[pi][0] - 1, self.inst_elems[pj][0] - 1
                _, _, ni_nodes = surface_triangle(*self.inst[pi], li, e0i, len(self.inst_elems[pi]))
                tri, tri_e, nj_nodes = surface_triangle(*self.inst[pj], lj, e0j, len(self.inst_elems[pj]))
                self.ct.append(dict(i=pi, j=pj, nodes_i=list(ni_nodes), nodes_j=list(nj_nodes), tri=tri,
                                    tri_e=tri_e, young=young[pj]))
        sizes = []
        for e in range(model.nElement):
            p = coord[elem[e] - 1]
            for q in (1, 3, 4):
                d = p[0] - p[q]
                sizes.append(math.sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]))
        self.min_size, self.max_size = min(sizes), max(sizes)
        self.elem = elem
        self.einst = inst
        cpar = getattr(model, "contact_params", None) or (0.25, 1.0, 1.0, 0.0, 0.0)
        self.myu, self.kc_o, self.kc_s, self.Cr_o, self.Cr_s = cpar

    def element_deleted(self, e):
        ii = int(self.einst[e - 1]) - 1
        faces, keys, owner = self.inst[ii]
        mine = [k for k in range(len(faces)) if owner[k] == e]
        add_f, add_e = [], []
        for j in mine:
            for k in range(len(faces)):
                if owner[k] == e:
                    continue
                if keys[j] == keys[k]:
                    add_f.append(faces[k])
                    add_e.append(owner[k])
                    break
        tri, tri_e = [], []
        for f, ow in zip(add_f, add_e):
            tri += [[f[0], f[1], f[2]], [f[2], f[3], f[0]]]
            tri_e += [ow, ow]
        nodes = sorted(set(n for t in tri for n in t))
        for c in self.ct:
            if c["i"] == ii:
                for n in nodes:
                    if n not in c["nodes_i"]:
                        c["nodes_i"].append(n)
            elif c["j"] == ii:
                for n in nodes:
                    if n not in c["nodes_j"]:
                        c["nodes_j"].append(n)
                c["tri_e"] += tri_e
                c["tri"] += tri

    def force(self, position, velo, diag_M, element_flag):
        """position (nN,3), velo (3nN,) -> contact force (3nN,), number of events."""
        nN = position.shape[0]
        acc = [Fraction(0)] * (3 * nN)
        d_lim = self.min_size * 0.3
        n_ev = 0
        norm = lambda a, b, c: math.sqrt(a * a + b * b + c * c)  # noqa: E731
        for c in self.ct:
            self_ = c["i"] == c["j"]
            P = position
            pi = np.array([P[n - 1] for n in c["nodes_i"]])
            pj = np.array([P[n - 1] for n in c["nodes_j"]])
            mni, mxi, mnj, mxj = pi.min(0), pi.max(0), pj.min(0), pj.max(0)
            rmn = [max(mni[d], mnj[d]) for d in range(3)]
            rmx = [min(mxi[d], mxj[d]) for d in range(3)]
            if any(rmn[d] > rmx[d] for d in range(3)):
                continue
            amn = [min(mni[d], mnj[d]) for d in range(3)]
            ddiv = self.max_size * (0.6 if self_ else 1.1)
            mapi = [[math.ceil((P[n - 1][d] - amn[d]) / ddiv) for d in range(3)] for n in c["nodes_i"]]
            kc, Cr = (self.kc_s, self.Cr_s) if self_ else (self.kc_o, self.Cr_o)
            for t, ele in zip(c["tri"], c["tri_e"]):
                if element_flag[ele - 1] == 0:
                    continue
                j0, j1, j2 = t
                q0, q1, q2 = P[j0 - 1], P[j1 - 1], P[j2 - 1]
                if any(q0[d] < rmn[d] and q1[d] < rmn[d] and q2[d] < rmn[d] for d in range(3)):
                    continue
                if any(q0[d] > rmx[d] and q1[d] > rmx[d] and q2[d] > rmx[d] for d in range(3)):
                    continue
                cx, cy, cz = [(q0[d] + q1[d] + q2[d]) / 3.0 for d in range(3)]
                Rmax = max(max(norm(q0[0] - cx, q0[1] - cy, q0[2] - cz), norm(q1[0] - cx, q1[1] - cy, q1[2] - cz)),
                           norm(q2[0] - cx, q2[1] - cy, q2[2] - cz))
                v1 = [q1[d] - q0[d] for d in range(3)]
                v2 = [q2[d] - q0[d] for d in range(3)]
                L1, L2 = norm(*v1), norm(*v2)
                Lmax = max(L1, L2)
                n1 = v1[1] * v2[2] - v1[2] * v2[1]
                n2 = v1[2] * v2[0] - v1[0] * v2[2]
                n3 = v1[0] * v2[1] - v1[1] * v2[0]
                mg = math.sqrt(n1 * n1 + n2 * n2 + n3 * n3)
                nx, ny, nz = n1 / mg, n2 / mg, n3 / mg
                d12 = v1[0] * v2[0] + v1[1] * v2[1] + v1[2] * v2[2]
                S = 0.5 * math.sqrt(L1 * L1 * L2 * L2 - d12 * d12)
                A11, A21, A31, A12, A22, A32, A13, A23, A33 = v1[0], v1[1], v1[2], v2[0], v2[1], v2[2], -nx, -ny, -nz
                mj = [math.ceil((q0[d] - amn[d]) / ddiv) for d in range(3)]
                el = [int(x) for x in self.elem[ele - 1]]
                for k, i in enumerate(c["nodes_i"]):
                    if any(abs(mj[d] - mapi[k][d]) > 1 for d in range(3)):
                        continue
                    if self_ and i in el:
                        continue
                    p = P[i - 1]
                    if p[0] < rmn[0] or p[1] < rmn[1] or p[2] < rmn[2]:
                        continue
                    if p[0] > rmx[0] or p[1] > rmx[1] or p[2] > rmx[2]:
                        continue
                    if norm(p[0] - cx, p[1] - cy, p[2] - cz) >= Rmax:
                        continue
                    bx, by, bz = p[0] - q0[0], p[1] - q0[1], p[2] - q0[2]
                    v = (A11 * A22 * A33 + A12 * A23 * A31 + A13 * A21 * A32 - A11 * A23 * A32 - A12 * A21 * A33
                         - A13 * A22 * A31)
                    x1 = ((A22 * A33 - A23 * A32) * bx + (A13 * A32 - A12 * A33) * by + (A12 * A23 - A13 * A22) * bz) / v
                    x2 = ((A23 * A31 - A21 * A33) * bx + (A11 * A33 - A13 * A31) * by + (A13 * A21 - A11 * A23) * bz) / v
                    d = ((A21 * A32 - A22 * A31) * bx + (A12 * A31 - A11 * A32) * by + (A11 * A22 - A12 * A21) * bz) / v
                    if not (0.0 <= x1 and 0.0 <= x2 and x1 + x2 <= 1.0 and d > 0.0 and d <= d_lim):
                        continue
                    vx = velo[i * 3 - 3] - velo[j0 * 3 - 3]
                    vy = velo[i * 3 - 2] - velo[j0 * 3 - 2]
                    vz = velo[i * 3 - 1] - velo[j0 * 3 - 1]
                    mag = norm(vx, vy, vz)
                    vex = vey = vez = 0.0
                    if mag > 0.0:
                        vex, vey, vez = vx / mag, vy / mag, vz / mag
                    kk = c["young"] * S / Lmax * kc
                    F = kk * d
                    fx, fy, fz = F * nx, F * ny, F * nz
                    Cd = 2 * math.sqrt(diag_M[i - 1] * kk) * Cr
                    fcx, fcy, fcz = -Cd * vx, -Cd * vy, -Cd * vz
                    dvn = vex * nx + vey * ny + vez * nz
                    vsx, vsy, vsz = vex - dvn * nx, vey - dvn * ny, vez - dvn * nz
                    fx += -self.myu * F * vsx + fcx
                    fy += -self.myu * F * vsy + fcy
                    fz += -self.myu * F * vsz + fcz
                    for q, val in enumerate((fx, fy, fz)):
                        acc[3 * (i - 1) + q] += Fraction(val)
                        for tn in (j0, j1, j2):
                            acc[3 * (tn - 1) + q] += Fraction(-val / 3.0)
                    n_ev += 1
        return np.array([float(a) for a in acc]), n_ev
