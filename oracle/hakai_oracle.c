/*
 * hakai_oracle.c -- TEST INFRASTRUCTURE ONLY (see hakai_oracle.h).
 *
 * Line-faithful C restatement of HAKAI v0.0.2's explicit time step. Every function cites the
 * reference lines it follows ("v2/" = /root/reference/HAKAI-v0.0.2/Julia/). Compile with
 * -ffp-contract=off: Julia does not contract a*b+c unless asked (muladd), so only the
 * StaticArrays products use fma() explicitly.
 */
#include "hakai_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* One term of a StaticArrays product chain (v2/HAKAI_j.jl:1204-1205, :1330): muladd, which the
 * reference's Julia lowers to a fused multiply-add on FMA hosts. HKO_SEPARATE_ROUNDING builds the
 * sensitivity variant (libhakai_oracle_nofma.so, tools/oracle_muladd_sensitivity.py) with the
 * product and the sum rounded separately, to measure what that lowering assumption is worth. */
#ifdef HKO_SEPARATE_ROUNDING
#define HKO_MULADD(a, b, c) ((a) * (b) + (c))
#else
#define HKO_MULADD(a, b, c) fma((a), (b), (c))
#endif

typedef struct {
    double density, young, poisson, G;
    double Dmat[36];          /* column-major 6x6, v2/HAKAI_j.jl:150-160 */
    int32_t npp;              /* plastic rows */
    double* plastic;          /* [npp][2] */
    double* Hd;               /* [npp-1], v2/readInpFile_j.jl:763-768 */
    int32_t nd;
    double* ductile;          /* [nd][3] */
} hko_mat;

struct hko_model {
    int64_t nN, nE;
    const double* coordmat;
    const int64_t* elementmat;
    const int64_t* element_material;
    int32_t nmat;
    hko_mat* mat;
    double d_time;
    double pusai[8][3][8];
    /* boundary conditions (copied) */
    int32_t n_groups;
    int32_t* amp_n;
    int64_t* amp_off;
    double* amp_time;
    double* amp_value;
    int64_t* entry_off;
    double* entry_value;
    int64_t* dof_off;
    int64_t* dofs;
};

/* cal_Pusai_hexa, v2/HAKAI_j.jl:1895-1943 */
void hko_pusai(double out[8][3][8]) {
    static const double delta[8][3] = {{-1.0, -1.0, -1.0}, {1.0, -1.0, -1.0}, {1.0, 1.0, -1.0},
                                       {-1.0, 1.0, -1.0},  {-1.0, -1.0, 1.0}, {1.0, -1.0, 1.0},
                                       {1.0, 1.0, 1.0},    {-1.0, 1.0, 1.0}};
    const double g = 1.0 / sqrt(3.0);
    const double gc[8][3] = {{-g, -g, -g}, {-g, -g, g}, {-g, g, -g}, {-g, g, g},
                             {g, -g, -g},  {g, -g, g},  {g, g, -g},  {g, g, g}};
    for (int k = 0; k < 8; ++k) {
        const double gzai = gc[k][0], eta = gc[k][1], tueta = gc[k][2];
        for (int i = 0; i < 8; ++i) {
            out[k][0][i] = 1.0 / 8.0 * delta[i][0] * (1.0 + eta * delta[i][1]) * (1.0 + tueta * delta[i][2]);
            out[k][1][i] = 1.0 / 8.0 * delta[i][1] * (1.0 + gzai * delta[i][0]) * (1.0 + tueta * delta[i][2]);
            out[k][2][i] = 1.0 / 8.0 * delta[i][2] * (1.0 + gzai * delta[i][0]) * (1.0 + eta * delta[i][1]);
        }
    }
}

hko_model* hko_model_create(int64_t nN, const double* coordmat, int64_t nE, const int64_t* elementmat,
                            const int64_t* element_material, int32_t nmat, const hko_material_in* mats,
                            double d_time) {
    hko_model* m = (hko_model*)calloc(1, sizeof(hko_model));
    m->nN = nN;
    m->nE = nE;
    m->coordmat = coordmat;
    m->elementmat = elementmat;
    m->element_material = element_material;
    m->nmat = nmat;
    m->d_time = d_time;
    m->mat = (hko_mat*)calloc((size_t)(nmat > 0 ? nmat : 1), sizeof(hko_mat));
    for (int32_t i = 0; i < nmat; ++i) {
        hko_mat* o = &m->mat[i];
        const hko_material_in* in = &mats[i];
        o->density = in->density;
        o->young = in->young;
        o->poisson = in->poisson;
        /* v2/HAKAI_j.jl:143-160 */
        const double young = in->young, poisson = in->poisson;
        o->G = young / 2. / (1.0 + poisson);
        const double d1 = (1.0 - poisson), d2 = poisson, d3 = (1.0 - 2.0 * poisson) / 2.0;
        const double c = young / (1.0 + poisson) / (1.0 - 2.0 * poisson);
        const double M[6][6] = {{d1, d2, d2, 0, 0, 0}, {d2, d1, d2, 0, 0, 0}, {d2, d2, d1, 0, 0, 0},
                                {0, 0, 0, d3, 0, 0},   {0, 0, 0, 0, d3, 0},   {0, 0, 0, 0, 0, d3}};
        for (int r = 0; r < 6; ++r)
            for (int cc = 0; cc < 6; ++cc) o->Dmat[r + 6 * cc] = c * M[r][cc];
        o->npp = in->n_plastic;
        o->plastic = (double*)calloc((size_t)(2 * (o->npp > 0 ? o->npp : 1)), sizeof(double));
        if (o->npp > 0) memcpy(o->plastic, in->plastic, sizeof(double) * 2 * (size_t)o->npp);
        o->Hd = (double*)calloc((size_t)(o->npp > 1 ? o->npp - 1 : 1), sizeof(double));
        for (int32_t r = 0; r + 1 < o->npp; ++r) /* v2/readInpFile_j.jl:763-768 */
            o->Hd[r] = (o->plastic[2 * (r + 1)] - o->plastic[2 * r]) /
                       (o->plastic[2 * (r + 1) + 1] - o->plastic[2 * r + 1]);
        o->nd = in->n_ductile;
        o->ductile = (double*)calloc((size_t)(3 * (o->nd > 0 ? o->nd : 1)), sizeof(double));
        if (o->nd > 0) memcpy(o->ductile, in->ductile, sizeof(double) * 3 * (size_t)o->nd);
    }
    hko_pusai(m->pusai);
    return m;
}

static void free_bc(hko_model* m) {
    free(m->amp_n); free(m->amp_off); free(m->amp_time); free(m->amp_value);
    free(m->entry_off); free(m->entry_value); free(m->dof_off); free(m->dofs);
    m->amp_n = NULL; m->amp_off = NULL; m->amp_time = NULL; m->amp_value = NULL;
    m->entry_off = NULL; m->entry_value = NULL; m->dof_off = NULL; m->dofs = NULL;
    m->n_groups = 0;
}

void hko_model_destroy(hko_model* m) {
    if (!m) return;
    for (int32_t i = 0; i < m->nmat; ++i) {
        free(m->mat[i].plastic);
        free(m->mat[i].Hd);
        free(m->mat[i].ductile);
    }
    free(m->mat);
    free_bc(m);
    free(m);
}

int hko_model_set_bc(hko_model* m, const hko_bc* bc) {
    free_bc(m);
    const int32_t G = bc->n_groups;
    m->n_groups = G;
    if (G == 0) return 0;
    int64_t n_amp = 0;
    for (int32_t g = 0; g < G; ++g) {
        const int64_t end = bc->amp_off[g] + bc->amp_n[g];
        if (end > n_amp) n_amp = end;
    }
    const int64_t n_ent = bc->entry_off[G];
    const int64_t n_dof = bc->dof_off[n_ent];
    m->amp_n = (int32_t*)malloc(sizeof(int32_t) * (size_t)G);
    m->amp_off = (int64_t*)malloc(sizeof(int64_t) * (size_t)G);
    m->amp_time = (double*)malloc(sizeof(double) * (size_t)(n_amp + 1));
    m->amp_value = (double*)malloc(sizeof(double) * (size_t)(n_amp + 1));
    m->entry_off = (int64_t*)malloc(sizeof(int64_t) * (size_t)(G + 1));
    m->entry_value = (double*)malloc(sizeof(double) * (size_t)(n_ent + 1));
    m->dof_off = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_ent + 1));
    m->dofs = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_dof + 1));
    memcpy(m->amp_n, bc->amp_n, sizeof(int32_t) * (size_t)G);
    memcpy(m->amp_off, bc->amp_off, sizeof(int64_t) * (size_t)G);
    if (n_amp) {
        memcpy(m->amp_time, bc->amp_time, sizeof(double) * (size_t)n_amp);
        memcpy(m->amp_value, bc->amp_value, sizeof(double) * (size_t)n_amp);
    }
    memcpy(m->entry_off, bc->entry_off, sizeof(int64_t) * (size_t)(G + 1));
    if (n_ent) memcpy(m->entry_value, bc->entry_value, sizeof(double) * (size_t)n_ent);
    memcpy(m->dof_off, bc->dof_off, sizeof(int64_t) * (size_t)(n_ent + 1));
    if (n_dof) memcpy(m->dofs, bc->dofs, sizeof(int64_t) * (size_t)n_dof);
    for (int32_t g = 0; g < G; ++g)
        if (m->amp_n[g] == 1) return -2; /* reference raises BoundsError (a_t[2]) */
    return 0;
}

/* my3det, v2/HAKAI_j.jl:3235-3243; m3 row-major [3][3] */
static double my3det(const double m3[3][3]) {
    return (m3[0][0] * m3[1][1] * m3[2][2] + m3[0][1] * m3[1][2] * m3[2][0] + m3[0][2] * m3[1][0] * m3[2][1] -
            m3[0][0] * m3[1][2] * m3[2][1] - m3[0][1] * m3[1][0] * m3[2][2] - m3[0][2] * m3[1][1] * m3[2][0]);
}

/* v2/HAKAI_j.jl:183-218 */
void hko_lumped_mass(const hko_model* m, double mass_scaling, double* diag_M, double* elementVolume) {
    const int64_t nE = m->nE, nN = m->nN;
    for (int64_t e = 0; e < nE; ++e) {
        double X[3][8];
        for (int i = 0; i < 8; ++i) {
            const int64_t n = m->elementmat[8 * e + i] - 1;
            for (int c = 0; c < 3; ++c) X[c][i] = m->coordmat[3 * n + c];
        }
        double V = 0.;
        for (int k = 0; k < 8; ++k) {
            /* J = Pusai_mat[k] * e_position' (3x8 * 8x3), summed in node order */
            double J[3][3];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) {
                    double acc = m->pusai[k][a][0] * X[b][0];
                    for (int i = 1; i < 8; ++i) acc = acc + m->pusai[k][a][i] * X[b][i];
                    J[a][b] = acc;
                }
            V = V + my3det(J);
        }
        elementVolume[e] = V;
    }
    for (int64_t i = 0; i < 3 * nN; ++i) diag_M[i] = 0.0;
    for (int64_t e = 0; e < nE; ++e) {
        const double density = m->mat[m->element_material[e] - 1].density;
        const double node_mass = density * elementVolume[e] / 8.0;
        for (int c = 0; c < 3; ++c)
            for (int i = 0; i < 8; ++i) diag_M[(m->elementmat[8 * e + i] - 1) * 3 + c] += node_mass;
    }
    for (int64_t i = 0; i < 3 * nN; ++i) diag_M[i] = diag_M[i] * mass_scaling;
}

/* v2/HAKAI_j.jl:456-465 */
void hko_init_yield(const hko_model* m, double* y) {
    for (int64_t e = 0; e < m->nE; ++e) {
        const hko_mat* mt = &m->mat[m->element_material[e] - 1];
        for (int k = 0; k < 8; ++k) y[8 * e + k] = (mt->npp > 0) ? mt->plastic[0] : 0.0;
    }
}

/* cal_BVbar_hexa, v2/HAKAI_j.jl:1705-1784. X[c][i]; BVbar[r][j] (6x24, rows 3-5 stay 0). */
static double cal_BVbar_hexa(const double P[8][3][8], const double X[3][8], double BVbar[6][24],
                             int64_t* neg_count) {
    double V = 0.0;
    for (int k = 0; k < 8; ++k) {
        double J11 = 0.0, J12 = 0.0, J13 = 0.0, J21 = 0.0, J22 = 0.0, J23 = 0.0, J31 = 0.0, J32 = 0.0,
               J33 = 0.0;
        const double(*P1)[8] = P[k];
        for (int i = 0; i < 8; ++i) {
            J11 += P1[0][i] * X[0][i];
            J12 += P1[0][i] * X[1][i];
            J13 += P1[0][i] * X[2][i];
            J21 += P1[1][i] * X[0][i];
            J22 += P1[1][i] * X[1][i];
            J23 += P1[1][i] * X[2][i];
            J31 += P1[2][i] * X[0][i];
            J32 += P1[2][i] * X[1][i];
            J33 += P1[2][i] * X[2][i];
        }
        const double v = (J11 * J22 * J33 + J12 * J23 * J31 + J13 * J21 * J32 - J11 * J23 * J32 -
                          J12 * J21 * J33 - J13 * J22 * J31);
        double detJi = v;
        if (detJi < 0) { /* :1736-1739 */
            detJi = fabs(detJi);
            if (neg_count) ++*neg_count;
        }
        V += detJi;
        const double div_v = 1.0 / detJi;
        const double iJ11 = (J22 * J33 - J23 * J32) * div_v;
        const double iJ21 = (J23 * J31 - J21 * J33) * div_v;
        const double iJ31 = (J21 * J32 - J22 * J31) * div_v;
        const double iJ12 = (J13 * J32 - J12 * J33) * div_v;
        const double iJ22 = (J11 * J33 - J13 * J31) * div_v;
        const double iJ32 = (J12 * J31 - J11 * J32) * div_v;
        const double iJ13 = (J12 * J23 - J13 * J22) * div_v;
        const double iJ23 = (J13 * J21 - J11 * J23) * div_v;
        const double iJ33 = (J11 * J22 - J12 * J21) * div_v;
        for (int i = 0; i < 8; ++i) {
            const double Pix = iJ11 * P1[0][i] + iJ12 * P1[1][i] + iJ13 * P1[2][i];
            const double Piy = iJ21 * P1[0][i] + iJ22 * P1[1][i] + iJ23 * P1[2][i];
            const double Piz = iJ31 * P1[0][i] + iJ32 * P1[1][i] + iJ33 * P1[2][i];
            for (int r = 0; r < 3; ++r) {
                BVbar[r][i * 3 + 0] += Pix / 3.0 * detJi;
                BVbar[r][i * 3 + 1] += Piy / 3.0 * detJi;
                BVbar[r][i * 3 + 2] += Piz / 3.0 * detJi;
            }
        }
    }
    for (int r = 0; r < 6; ++r) /* BVbar .= BVbar / V */
        for (int j = 0; j < 24; ++j) BVbar[r][j] = BVbar[r][j] / V;
    return V;
}

/* cal_Bfinal, v2/HAKAI_j.jl:1415-1519. Bfinal must be zero on entry (:1198). */
static double cal_Bfinal(double Bfinal[6][24], const double BVbar[6][24], const double P1[3][8],
                         const double X[3][8]) {
    double J11 = 0.0, J12 = 0.0, J13 = 0.0, J21 = 0.0, J22 = 0.0, J23 = 0.0, J31 = 0.0, J32 = 0.0, J33 = 0.0;
    for (int i = 0; i < 8; ++i) {
        J11 += P1[0][i] * X[0][i];
        J12 += P1[0][i] * X[1][i];
        J13 += P1[0][i] * X[2][i];
        J21 += P1[1][i] * X[0][i];
        J22 += P1[1][i] * X[1][i];
        J23 += P1[1][i] * X[2][i];
        J31 += P1[2][i] * X[0][i];
        J32 += P1[2][i] * X[1][i];
        J33 += P1[2][i] * X[2][i];
    }
    const double v = (J11 * J22 * J33 + J12 * J23 * J31 + J13 * J21 * J32 - J11 * J23 * J32 -
                      J12 * J21 * J33 - J13 * J22 * J31);
    const double detJi = v;
    const double div_v = 1.0 / v;
    const double iJ11 = (J22 * J33 - J23 * J32) * div_v;
    const double iJ21 = (J23 * J31 - J21 * J33) * div_v;
    const double iJ31 = (J21 * J32 - J22 * J31) * div_v;
    const double iJ12 = (J13 * J32 - J12 * J33) * div_v;
    const double iJ22 = (J11 * J33 - J13 * J31) * div_v;
    const double iJ32 = (J12 * J31 - J11 * J32) * div_v;
    const double iJ13 = (J12 * J23 - J13 * J22) * div_v;
    const double iJ23 = (J13 * J21 - J11 * J23) * div_v;
    const double iJ33 = (J11 * J22 - J12 * J21) * div_v;
    for (int i = 0; i < 8; ++i) {
        const double Pix = iJ11 * P1[0][i] + iJ12 * P1[1][i] + iJ13 * P1[2][i];
        const double Piy = iJ21 * P1[0][i] + iJ22 * P1[1][i] + iJ23 * P1[2][i];
        const double Piz = iJ31 * P1[0][i] + iJ32 * P1[1][i] + iJ33 * P1[2][i];
        const int c0 = i * 3, c1 = i * 3 + 1, c2 = i * 3 + 2;
        Bfinal[0][c0] += Pix;
        Bfinal[1][c1] += Piy;
        Bfinal[2][c2] += Piz;
        Bfinal[3][c0] += Piy;
        Bfinal[3][c1] += Pix;
        Bfinal[4][c1] += Piz;
        Bfinal[4][c2] += Piy;
        Bfinal[5][c0] += Piz;
        Bfinal[5][c2] += Pix;
        for (int r = 0; r < 3; ++r) {
            Bfinal[r][c0] += -Pix / 3.0 + BVbar[r][c0];
            Bfinal[r][c1] += -Piy / 3.0 + BVbar[r][c1];
            Bfinal[r][c2] += -Piz / 3.0 + BVbar[r][c2];
        }
    }
    return detJi;
}

/* One element of the @floop body, v2/HAKAI_j.jl:1114-1353. */
static void stress_one_element(const hko_model* m, int64_t e, double* Qe, double* integ_stress,
                               double* integ_strain, double* integ_yield_stress,
                               double* integ_eq_plastic_strain, const double* position,
                               const double* d_disp, double* elementVolume, int64_t* neg_count) {
    const int64_t mat_id = m->element_material[e] - 1;
    const hko_mat* mt = &m->mat[mat_id];
    const double G = mt->G;
    const double* Dm = mt->Dmat;
    const int32_t npp = mt->npp;
    double d_u[24], X[3][8];
    for (int i = 0; i < 8; ++i) {
        const int64_t n = m->elementmat[8 * e + i] - 1;
        d_u[3 * i + 0] = d_disp[3 * n + 0];
        d_u[3 * i + 1] = d_disp[3 * n + 1];
        d_u[3 * i + 2] = d_disp[3 * n + 2];
        X[0][i] = position[3 * n + 0];
        X[1][i] = position[3 * n + 1];
        X[2][i] = position[3 * n + 2];
    }
    double BVbar[6][24];
    memset(BVbar, 0, sizeof(BVbar));
    const double V = cal_BVbar_hexa(m->pusai, X, BVbar, neg_count);
    elementVolume[e] = V;
    const double W = 1.0;
    for (int i = 0; i < 8; ++i) {
        double Bfinal[6][24];
        memset(Bfinal, 0, sizeof(Bfinal));
        const double detJ = cal_Bfinal(Bfinal, BVbar, m->pusai[i], X);
        /* d_e_vec = Bfinal * d_u ; d_o_vec = Dmat * d_e_vec (StaticArrays muladd chains) */
        double de[6], dsig[6];
        for (int r = 0; r < 6; ++r) {
            double acc = Bfinal[r][0] * d_u[0];
            for (int j = 1; j < 24; ++j) acc = HKO_MULADD(Bfinal[r][j], d_u[j], acc);
            de[r] = acc;
        }
        for (int r = 0; r < 6; ++r) {
            double acc = Dm[r + 0] * de[0];
            for (int j = 1; j < 6; ++j) acc = HKO_MULADD(Dm[r + 6 * j], de[j], acc);
            dsig[r] = acc;
        }
        const int64_t idx = e * 8 + i;
        double pre[6], fin[6];
        for (int r = 0; r < 6; ++r) pre[r] = integ_stress[6 * idx + r];
        for (int r = 0; r < 6; ++r) fin[r] = pre[r] + dsig[r];
        if (npp > 0) { /* :1227-1289 */
            double tri[6], dev[6];
            for (int r = 0; r < 6; ++r) tri[r] = pre[r] + dsig[r];
            const double mean = (tri[0] + tri[1] + tri[2]) / 3.0;
            dev[0] = tri[0] - mean;
            dev[1] = tri[1] - mean;
            dev[2] = tri[2] - mean;
            dev[3] = tri[3];
            dev[4] = tri[4];
            dev[5] = tri[5];
            const double q = sqrt(1.5 * (dev[0] * dev[0] + dev[1] * dev[1] + dev[2] * dev[2] +
                                         2 * (dev[3] * dev[3]) + 2 * (dev[4] * dev[4]) + 2 * (dev[5] * dev[5])));
            const double y = integ_yield_stress[idx];
            if (q > y) {
                int32_t p_index = 1; /* 1-based like the reference */
                for (int32_t j = 2; j <= npp; ++j) {
                    if (integ_eq_plastic_strain[idx] <= mt->plastic[2 * (j - 1) + 1]) {
                        p_index = j - 1;
                        break;
                    }
                    if (j == npp) p_index = j - 1;
                }
                const double H = mt->Hd[p_index - 1];
                const double d_ep = (q - y) / (3 * G + H);
                const double s = y + H * d_ep;
                for (int r = 0; r < 3; ++r) fin[r] = dev[r] * s / q + mean;
                for (int r = 3; r < 6; ++r) fin[r] = dev[r] * s / q + 0.0;
                integ_eq_plastic_strain[idx] += d_ep;
                integ_yield_stress[idx] += H * d_ep;
            }
        }
        for (int r = 0; r < 6; ++r) integ_strain[6 * idx + r] += de[r];
        for (int r = 0; r < 6; ++r) integ_stress[6 * idx + r] = fin[r];
        /* q_vec_i = Bfinal' * final_stress ; Qe[:,e] += W*W*W*detJ*q_vec_i */
        for (int j = 0; j < 24; ++j) {
            double acc = Bfinal[0][j] * fin[0];
            for (int r = 1; r < 6; ++r) acc = HKO_MULADD(Bfinal[r][j], fin[r], acc);
            Qe[24 * e + j] += W * W * W * detJ * acc;
        }
    }
}

void hko_cal_stress_hexa(const hko_model* m, double* Qe, double* integ_stress, double* integ_strain,
                         double* integ_yield_stress, double* integ_eq_plastic_strain, const double* position,
                         const double* d_disp, const int64_t* element_flag, double* elementVolume,
                         int nthreads) {
    const int64_t nE = m->nE;
#ifdef _OPENMP
    if (nthreads > 1) {
#pragma omp parallel for schedule(static) num_threads(nthreads)
        for (int64_t e = 0; e < nE; ++e) {
            if (element_flag[e] == 0) continue;
            stress_one_element(m, e, Qe, integ_stress, integ_strain, integ_yield_stress,
                               integ_eq_plastic_strain, position, d_disp, elementVolume, NULL);
        }
        return;
    }
#else
    (void)nthreads;
#endif
    for (int64_t e = 0; e < nE; ++e) {
        if (element_flag[e] == 0) continue; /* :1116-1118 */
        stress_one_element(m, e, Qe, integ_stress, integ_strain, integ_yield_stress, integ_eq_plastic_strain,
                           position, d_disp, elementVolume, NULL);
    }
}

/* StaticArrays _eig for a 3x3 Hermitian (closed form after Smith 1961): values only. */
void hko_eigvals_sym3(const double s[6], double out[3]) {
    const double a11 = s[0], a22 = s[1], a33 = s[2];
    const double a12 = s[3], a13 = s[5], a23 = s[4]; /* T = [ox txy txz; txy oy tyz; txz tyz oz] */
    const double p1 = a12 * a12 + a13 * a13 + a23 * a23;
    if (p1 == 0) {
        if (a11 < a22) {
            if (a22 < a33) { out[0] = a11; out[1] = a22; out[2] = a33; }
            else if (a33 < a11) { out[0] = a33; out[1] = a11; out[2] = a22; }
            else { out[0] = a11; out[1] = a33; out[2] = a22; }
        } else {
            if (a11 < a33) { out[0] = a22; out[1] = a11; out[2] = a33; }
            else if (a33 < a22) { out[0] = a33; out[1] = a22; out[2] = a11; }
            else { out[0] = a22; out[1] = a33; out[2] = a11; }
        }
        return;
    }
    const double q = (a11 + a22 + a33) / 3;
    const double p2 = (a11 - q) * (a11 - q) + (a22 - q) * (a22 - q) + (a33 - q) * (a33 - q) + 2 * p1;
    const double p = sqrt(p2 / 6);
    const double invp = 1.0 / p;
    const double b11 = (a11 - q) * invp, b22 = (a22 - q) * invp, b33 = (a33 - q) * invp;
    const double b12 = a12 * invp, b13 = a13 * invp, b23 = a23 * invp;
    /* det(B): x0 . (x1 x x2) with columns x0=(b11,b12,b13), x1=(b12,b22,b23), x2=(b13,b23,b33) */
    const double cx = b22 * b33 - b23 * b23;
    const double cy = b23 * b13 - b12 * b33;
    const double cz = b12 * b23 - b22 * b13;
    const double r = (b11 * cx + b12 * cy + b13 * cz) / 2;
    double phi;
    const double pi = 3.14159265358979323846;
    if (r <= -1) phi = pi / 3;
    else if (r >= 1) phi = 0.0;
    else phi = acos(r) / 3;
    const double eig3 = q + 2 * p * cos(phi);
    const double eig1 = q + 2 * p * cos(phi + (2 * pi / 3));
    const double eig2 = 3 * q - eig1 - eig3;
    out[0] = eig1;
    out[1] = eig2;
    out[2] = eig3;
}

/* cal_triax_stress, v2/HAKAI_j.jl:982-1022 */
void hko_cal_triax_stress(int64_t n, const double* st, double* tx) {
    for (int64_t i = 0; i < n; ++i) tx[i] = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        double p[3];
        hko_eigvals_sym3(&st[6 * i], p);
        const double oeq = sqrt(0.5 * ((p[0] - p[1]) * (p[0] - p[1]) + (p[1] - p[2]) * (p[1] - p[2]) +
                                       (p[2] - p[0]) * (p[2] - p[0])));
        if (oeq < 1E-10) continue;
        tx[i] = (p[0] + p[1] + p[2]) / 3.0 / oeq;
    }
}

/* Amplitude interpolation, v2/HAKAI_j.jl:586-600 */
static double bc_amp(const hko_model* m, int32_t g, double current_time) {
    const int32_t n = m->amp_n[g];
    if (n <= 0) return 1.0;
    const double* a_t = m->amp_time + m->amp_off[g];
    const double* a_v = m->amp_value + m->amp_off[g];
    int32_t ti = 0;
    for (int32_t j = 0; j < n - 1; ++j) {
        if (current_time >= a_t[j] && current_time <= a_t[j + 1]) {
            ti = j;
            break;
        }
    }
    return a_v[ti] + (a_v[ti + 1] - a_v[ti]) * (current_time - a_t[ti]) / (a_t[ti + 1] - a_t[ti]);
}

int hko_run(const hko_model* m, hko_state* s, const double* diag_M, double t_first, int64_t n_steps,
            int nthreads, int64_t* del_log, int64_t del_cap, int64_t* del_n) {
    return hko_run_contact(m, s, diag_M, t_first, n_steps, nthreads, del_log, del_cap, del_n, NULL, NULL);
}

int hko_run_contact(const hko_model* m, hko_state* s, const double* diag_M, double t_first, int64_t n_steps,
                    int nthreads, int64_t* del_log, int64_t del_cap, int64_t* del_n, hko_contact* ct,
                    const int64_t* element_instance) {
    const int64_t nN = m->nN, nE = m->nE, fn = 3 * nN;
    const double d_time = m->d_time;
    int64_t* deleted = ct ? (int64_t*)malloc(sizeof(int64_t) * (size_t)(nE > 0 ? nE : 1)) : NULL;
    for (int64_t it = 0; it < n_steps; ++it) {
        const double t = t_first + (double)it;
        int64_t n_deleted = 0;
        /* :497-498 (no concentrated loads in the reader) */
        for (int64_t i = 0; i < fn; ++i) s->external_force[i] = 0.0;
        /* :500-560 contact force into external_force */
        if (ct) hko_contact_force(ct, s->position, s->velo, diag_M, s->element_flag, s->external_force);
        /* :562-567, diag_C = 0 (:217-218) */
        for (int64_t i = 0; i < fn; ++i) {
            const double dC = 0.0 * diag_M[i]; /* diag_C .= diag_M * C with C = 0 */
            s->disp_new[i] = 1.0 / (diag_M[i] / (d_time * d_time) + dC / 2.0 / d_time) *
                             (s->external_force[i] - s->Q[i] +
                              diag_M[i] / (d_time * d_time) * (2.0 * s->disp[i] - s->disp_pre[i]) +
                              dC / 2.0 / d_time * s->disp_pre[i]);
        }
        /* :585-617 */
        for (int32_t g = 0; g < m->n_groups; ++g) {
            const double amp = bc_amp(m, g, t * d_time);
            for (int64_t en = m->entry_off[g]; en < m->entry_off[g + 1]; ++en) {
                const double v = m->entry_value[en];
                for (int64_t d = m->dof_off[en]; d < m->dof_off[en + 1]; ++d) s->disp_new[m->dofs[d] - 1] = v * amp;
            }
        }
        /* :624-629 */
        for (int64_t i = 0; i < fn; ++i) {
            s->d_disp[i] = s->disp_new[i] - s->disp[i];
            s->disp_pre[i] = s->disp[i];
            s->disp[i] = s->disp_new[i];
            s->velo[i] = s->d_disp[i] / d_time;
        }
        /* :644-653 */
        for (int64_t i = 0; i < nN; ++i) {
            s->position[3 * i + 0] = m->coordmat[3 * i + 0] + s->disp[3 * i + 0];
            s->position[3 * i + 1] = m->coordmat[3 * i + 1] + s->disp[3 * i + 1];
            s->position[3 * i + 2] = m->coordmat[3 * i + 2] + s->disp[3 * i + 2];
        }
        /* :662-667 */
        for (int64_t i = 0; i < 24 * nE; ++i) s->Qe[i] = 0.0;
        hko_cal_stress_hexa(m, s->Qe, s->integ_stress, s->integ_strain, s->integ_yield_stress,
                            s->integ_eq_plastic_strain, s->position, s->d_disp, s->element_flag,
                            s->elementVolume, nthreads);
        /* :668-675 serial element-order assembly */
        for (int64_t i = 0; i < fn; ++i) s->Q[i] = 0.0;
        for (int64_t e = 0; e < nE; ++e)
            for (int i = 0; i < 8; ++i) {
                const int64_t n = m->elementmat[8 * e + i] - 1;
                s->Q[0 + n * 3] += s->Qe[24 * e + 0 + i * 3];
                s->Q[1 + n * 3] += s->Qe[24 * e + 1 + i * 3];
                s->Q[2 + n * 3] += s->Qe[24 * e + 2 + i * 3];
            }
        /* :677 */
        hko_cal_triax_stress(8 * nE, s->integ_stress, s->integ_triax_stress);
        /* :684-764 (flag_fracture is always 1) */
        for (int64_t e = 0; e < nE; ++e) {
            const hko_mat* mt = &m->mat[m->element_material[e] - 1];
            const int32_t nd = mt->nd;
            if (nd <= 0) continue;
            double v_e = 0.0, t_e = 0.0;
            for (int j = 0; j < 8; ++j) {
                v_e += s->integ_eq_plastic_strain[j + e * 8];
                t_e += s->integ_triax_stress[j + e * 8];
            }
            v_e /= 8;
            t_e /= 8;
            if (t_e < 0) continue;
            const double* du = mt->ductile;
            double fr_e = du[3 * (nd - 1) + 0];
            for (int32_t j = 0; j + 1 < nd; ++j) {
                if (t_e >= du[3 * j + 1] && t_e < du[3 * (j + 1) + 1]) {
                    fr_e = du[3 * j] + (du[3 * (j + 1)] - du[3 * j]) / (du[3 * (j + 1) + 1] - du[3 * j + 1]) *
                                           (t_e - du[3 * j + 1]);
                    break;
                }
            }
            if (v_e >= fr_e && s->element_flag[e] == 1) {
                s->element_flag[e] = 0;
                if (deleted) deleted[n_deleted++] = e + 1;
                if (del_n) {
                    if (*del_n < del_cap) {
                        del_log[2 * *del_n + 0] = (int64_t)t;
                        del_log[2 * *del_n + 1] = e + 1;
                    }
                    ++*del_n;
                }
                for (int j = 0; j < 8; ++j)
                    for (int r = 0; r < 6; ++r) {
                        s->integ_stress[6 * (j + e * 8) + r] = 0.0;
                        s->integ_strain[6 * (j + e * 8) + r] = 0.0;
                    }
            }
        }
        /* :766-804 surface update */
        for (int64_t q = 0; q < n_deleted; ++q) hko_contact_element_deleted(ct, element_instance, deleted[q]);
    }
    free(deleted);
    return 0;
}

/* v2/HAKAI_j.jl:3408-3486 */
void hko_node_stress_strain(int64_t nN, int64_t nE, const int64_t* elementmat, const double* integ_stress,
                            const double* integ_strain, const double* eqps, const double* triax,
                            double* node_stress, double* node_strain, double* node_eqps, double* node_mises,
                            double* node_triax) {
    if (nN <= 0) return;
    for (int64_t i = 0; i < 6 * nN; ++i) {
        node_stress[i] = 0.0;
        node_strain[i] = 0.0;
    }
    for (int64_t i = 0; i < nN; ++i) {
        node_eqps[i] = 0.0;
        node_triax[i] = 0.0;
    }
    double* inc = (double*)calloc((size_t)nN, sizeof(double));
    for (int64_t e = 0; e < nE; ++e) {
        double es[6], en[6], ee, et;
        for (int c = 0; c < 6; ++c) {
            /* sum!(zeros(1,6), rows) / integ_num */
            double a = 0.0, b = 0.0;
            for (int k = 0; k < 8; ++k) {
                a += integ_stress[6 * (8 * e + k) + c];
                b += integ_strain[6 * (8 * e + k) + c];
            }
            es[c] = a / 8;
            en[c] = b / 8;
        }
        double a = 0.0, b = 0.0;
        for (int k = 0; k < 8; ++k) {
            a += eqps[8 * e + k];
            b += triax[8 * e + k];
        }
        ee = a / 8;
        et = b / 8;
        for (int k = 0; k < 8; ++k) {
            const int64_t n = elementmat[8 * e + k] - 1;
            for (int c = 0; c < 6; ++c) {
                node_stress[6 * n + c] += es[c];
                node_strain[6 * n + c] += en[c];
            }
            node_eqps[n] += ee;
            node_triax[n] += et;
        }
    }
    for (int64_t e = 0; e < nE; ++e)
        for (int k = 0; k < 8; ++k) inc[elementmat[8 * e + k] - 1] += 1;
    for (int64_t i = 0; i < nN; ++i) {
        for (int c = 0; c < 6; ++c) {
            node_stress[6 * i + c] /= inc[i];
            node_strain[6 * i + c] /= inc[i];
        }
        node_eqps[i] /= inc[i];
        node_triax[i] /= inc[i];
    }
    for (int64_t i = 0; i < nN; ++i) {
        const double ox = node_stress[6 * i + 0], oy = node_stress[6 * i + 1], oz = node_stress[6 * i + 2];
        const double txy = node_stress[6 * i + 3], tyz = node_stress[6 * i + 4], txz = node_stress[6 * i + 5];
        node_mises[i] = sqrt(0.5 * ((ox - oy) * (ox - oy) + (oy - oz) * (oy - oz) + (ox - oz) * (ox - oz) +
                                    6 * (txy * txy + tyz * tyz + txz * txz)));
    }
    free(inc);
}
