/*
 * hakai_oracle_contact.c -- TEST INFRASTRUCTURE ONLY (see hakai_oracle.h).
 *
 * Literal C restatement of HAKAI v0.0.2's all-exterior contact ("v2/" =
 * /root/reference/HAKAI-v0.0.2/Julia/):
 *   setup          v2/HAKAI_j.jl:244-402  (pairs, CT lists), :404-421 (element sizes)
 *   get_element_face       :1944-1992
 *   get_surface_triangle   :1996-2164  (the O(F^2) exterior scan and its quirks)
 *   add_surface_triangle   :2167-2245, applied after deletions at :766-804
 *   cal_contact_force      :2248-2706  (CPU path; Float128 per-thread accumulation :435 -> __float128)
 * Node ids are global (the reference works on part-local ids plus instance node offsets, the
 * same numbers). The face-orientation test uses the model's (instance) coordinates.
 */
#define _GNU_SOURCE /* qsort_r */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "hakai_oracle.h"

typedef struct {
    int64_t n, cap;
    int64_t* v;
} ivec;

static void iv_push(ivec* a, int64_t x) {
    if (a->n == a->cap) {
        a->cap = a->cap ? 2 * a->cap : 64;
        a->v = (int64_t*)realloc(a->v, sizeof(int64_t) * (size_t)a->cap);
    }
    a->v[a->n++] = x;
}

/* Julia unique!: keep first occurrences, in order. */
static void iv_unique_inplace(ivec* a) {
    int64_t w = 0;
    for (int64_t i = 0; i < a->n; ++i) {
        int dup = 0;
        for (int64_t j = 0; j < w; ++j)
            if (a->v[j] == a->v[i]) { dup = 1; break; }
        if (!dup) a->v[w++] = a->v[i];
    }
    a->n = w;
}

static int cmp_i64(const void* x, const void* y) {
    const int64_t a = *(const int64_t*)x, b = *(const int64_t*)y;
    return a < b ? -1 : a > b;
}

typedef struct {
    int64_t nE, e0;          /* elements e0+1 .. e0+nE (global, 1-based) */
    int64_t* faces;          /* [6nE][4] global node ids, oriented */
    int64_t* sorted;         /* [6nE][4] */
    int64_t* face_ele;       /* [6nE] global element id (1-based) */
    int64_t* order;          /* indexed mode: face indices sorted by (sorted key, index) */
    double young;
} inst_t;

typedef struct {
    int i_inst, j_inst;      /* 0-based */
    ivec nodes_i, nodes_j, tri, tri_ele;   /* tri: 3 per triangle */
    char *in_i, *in_j;       /* indexed mode: membership of nodes_i / nodes_j (node id -> 0/1) */
    double young;
} ct_t;

struct hko_contact {
    hko_model_view view;
    const hko_model_view* mv;
    int n_inst;
    inst_t* inst;
    int n_ct;
    ct_t* ct;
    double elementMinSize, elementMaxSize;
    double myu, kc_o, kc_s, Cr_o, Cr_s;
    /* Indexed mode (a checker for models too large for the literal loops, e.g. BASELINE C4 at
     * 4 M hex): the same face matches, lists, candidate node sets and event order as the literal
     * restatement, found through sorted face keys, membership tables and a cell index instead of
     * the reference's O(F^2) face scan, O(n^2) unique! and O(T x N) node loop. Every result is
     * identical by construction; tests/test_contact_oracle.py checks it against the literal mode. */
    int indexed;
};

static double my3norm(double a, double b, double c) { return sqrt(a * a + b * b + c * c); }

/* get_element_face, v2/HAKAI_j.jl:1944-1992 */
static void element_faces(const hko_model_view* mv, inst_t* I) {
    const int64_t nE = I->nE;
    I->faces = (int64_t*)malloc(sizeof(int64_t) * 24 * (size_t)nE);
    I->sorted = (int64_t*)malloc(sizeof(int64_t) * 24 * (size_t)nE);
    I->face_ele = (int64_t*)malloc(sizeof(int64_t) * 6 * (size_t)nE);
    static const int fidx[6][4] = {{0, 1, 2, 3}, {4, 5, 6, 7}, {0, 1, 5, 4}, {1, 2, 6, 5}, {2, 3, 7, 6}, {3, 0, 4, 7}};
    for (int64_t j = 0; j < nE; ++j) {
        const int64_t e = I->e0 + j;
        const int64_t* el = mv->elementmat + 8 * e;
        double ctr[3] = {0, 0, 0};
        for (int a = 0; a < 8; ++a) /* sum!(zeros(3,1), cdmat[:,elem]) / 8 */
            for (int c = 0; c < 3; ++c) ctr[c] += mv->coordmat[3 * (el[a] - 1) + c];
        for (int c = 0; c < 3; ++c) ctr[c] /= 8;
        for (int k = 0; k < 6; ++k) {
            int64_t* f = I->faces + 4 * (6 * j + k);
            for (int q = 0; q < 4; ++q) f[q] = el[fidx[k][q]];
            const double* x1 = mv->coordmat + 3 * (f[0] - 1);
            const double* x2 = mv->coordmat + 3 * (f[1] - 1);
            const double* x4 = mv->coordmat + 3 * (f[3] - 1);
            const double v1[3] = {x2[0] - x1[0], x2[1] - x1[1], x2[2] - x1[2]};
            const double v2[3] = {x4[0] - x1[0], x4[1] - x1[1], x4[2] - x1[2]};
            const double nv[3] = {v1[1] * v2[2] - v1[2] * v2[1], v1[2] * v2[0] - v1[0] * v2[2],
                                  v1[0] * v2[1] - v1[1] * v2[0]};
            const double vc[3] = {ctr[0] - x1[0], ctr[1] - x1[1], ctr[2] - x1[2]};
            if (nv[0] * vc[0] + nv[1] * vc[1] + nv[2] * vc[2] > 0.) {
                const int64_t t1 = f[1];
                f[1] = f[3];
                f[3] = t1;  /* [f1, f4, f3, f2] */
            }
            int64_t* s = I->sorted + 4 * (6 * j + k);
            memcpy(s, f, 4 * sizeof(int64_t));
            qsort(s, 4, sizeof(int64_t), cmp_i64);
            I->face_ele[6 * j + k] = e + 1;
        }
    }
}

static int same4(const int64_t* a, const int64_t* b) {
    return a[0] == b[0] && a[1] == b[1] && a[2] == b[2] && a[3] == b[3];
}

static int cmp_key4(const int64_t* a, const int64_t* b) {
    for (int q = 0; q < 4; ++q)
        if (a[q] != b[q]) return a[q] < b[q] ? -1 : 1;
    return 0;
}

static int cmp_face_r(const void* x, const void* y, void* arg) {
    const int64_t* sorted = (const int64_t*)arg;
    const int64_t a = *(const int64_t*)x, b = *(const int64_t*)y;
    const int c = cmp_key4(sorted + 4 * a, sorted + 4 * b);
    return c ? c : (a < b ? -1 : a > b);
}

/* indexed mode: faces ordered by (key, index) */
static void face_order(inst_t* I) {
    const int64_t F = 6 * I->nE;
    I->order = (int64_t*)malloc(sizeof(int64_t) * (size_t)(F > 0 ? F : 1));
    for (int64_t j = 0; j < F; ++j) I->order[j] = j;
    qsort_r(I->order, (size_t)F, sizeof(int64_t), cmp_face_r, I->sorted);
}

/* first position in I->order whose face key is >= key */
static int64_t order_lower(const inst_t* I, const int64_t* key) {
    int64_t lo = 0, hi = 6 * I->nE;
    while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (cmp_key4(I->sorted + 4 * I->order[mid], key) < 0) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/* The exterior-face marks of the literal scan below (j = 1:6nE-1, first later match of j marks
 * that match as seen): within a run of equal keys in index order, faces pair up two by two and an
 * odd run keeps its last face, unless that face is the instance's last (never visited as j). */
static void exterior_marks_indexed(const inst_t* I, char* keep) {
    const int64_t F = 6 * I->nE;
    int64_t a = 0;
    while (a < F) {
        int64_t b = a + 1;
        while (b < F && same4(I->sorted + 4 * I->order[a], I->sorted + 4 * I->order[b])) ++b;
        if ((b - a) & 1) {
            const int64_t last = I->order[b - 1];
            if (last < F - 1) keep[last] = 1;
        }
        a = b;
    }
}

/* get_surface_triangle, v2/HAKAI_j.jl:1996-2164. contact: instance-local 1-based element list of a
 * *Contact Pair surface (n_contact < 0: all elements); like the reference the exterior faces are
 * filtered only when the list length differs from the instance's element count (:2087). */
static void surface_triangles_of(const inst_t* I, ivec* tri, ivec* tri_ele, ivec* nodes, const int64_t* contact,
                                 int64_t n_contact);
static void surface_triangles_of(const inst_t* I, ivec* tri, ivec* tri_ele, ivec* nodes, const int64_t* contact,
                                 int64_t n_contact) {
    const int64_t F = 6 * I->nE;
    char* dp = (char*)calloc((size_t)F + 1, 1);
    char* keep = NULL;
    if (I->order) {
        keep = (char*)calloc((size_t)F + 1, 1);
        exterior_marks_indexed(I, keep);
    }
    for (int64_t j = 0; j < F - 1; ++j) { /* j = 1 : nE*6-1 */
        if (dp[j]) continue;
        int u = 1;
        if (keep) {
            u = keep[j];
        } else {
            for (int64_t k = j + 1; k < F; ++k)
                if (same4(I->sorted + 4 * j, I->sorted + 4 * k)) {
                    u = 0;
                    dp[k] = 1;
                    break;
                }
        }
        if (u && n_contact >= 0 && n_contact != I->nE) { /* "pick up only contact element" */
            const int64_t local = I->face_ele[j] - I->e0;  /* 1-based instance-local */
            int in = 0;
            for (int64_t q = 0; q < n_contact; ++q) in |= (contact[q] == local);
            u = in;
        }
        if (u) {
            const int64_t* f = I->faces + 4 * j;
            iv_push(tri, f[0]); iv_push(tri, f[1]); iv_push(tri, f[2]);
            iv_push(tri, f[2]); iv_push(tri, f[3]); iv_push(tri, f[0]);
            iv_push(tri_ele, I->face_ele[j]);
            iv_push(tri_ele, I->face_ele[j]);
        }
    }
    free(dp);
    free(keep);
    /* sort!(unique!(c_nodes)) */
    const int64_t n0 = nodes->n;
    for (int64_t i = 0; i < tri->n; ++i) iv_push(nodes, tri->v[i]);
    qsort(nodes->v + n0, (size_t)(nodes->n - n0), sizeof(int64_t), cmp_i64);
    int64_t w = n0;
    for (int64_t i = n0; i < nodes->n; ++i)
        if (w == n0 || nodes->v[w - 1] != nodes->v[i]) nodes->v[w++] = nodes->v[i];
    nodes->n = w;
}

hko_contact* hko_contact_create(const hko_model_view* mv, int contact_flag, const int64_t* element_instance,
                                const double* mat_young) {
    return hko_contact_create_cp(mv, contact_flag, element_instance, mat_young, 0, NULL, NULL, NULL);
}

hko_contact* hko_contact_create_cp(const hko_model_view* mv, int contact_flag, const int64_t* element_instance,
                                   const double* mat_young, int32_t n_cp, const int32_t* cp_instance,
                                   const int64_t* cp_off, const int64_t* cp_elems) {
    return hko_contact_create_ex(mv, contact_flag, element_instance, mat_young, n_cp, cp_instance, cp_off, cp_elems,
                                 0);
}

hko_contact* hko_contact_create_ex(const hko_model_view* mv, int contact_flag, const int64_t* element_instance,
                                   const double* mat_young, int32_t n_cp, const int32_t* cp_instance,
                                   const int64_t* cp_off, const int64_t* cp_elems, int indexed) {
    if (contact_flag < 1) return NULL;
    hko_contact* C = (hko_contact*)calloc(1, sizeof(hko_contact));
    C->indexed = indexed;
    C->view = *mv;
    C->mv = &C->view;
    mv = C->mv;
    C->myu = 0.25 * 1.0; C->kc_o = 1.0; C->kc_s = 1.0; C->Cr_o = 0.0; C->Cr_s = 0.0; /* :2255-2259 */
    int n_inst = 0;
    for (int64_t e = 0; e < mv->nE; ++e)
        if (element_instance[e] > n_inst) n_inst = (int)element_instance[e];
    C->n_inst = n_inst;
    C->inst = (inst_t*)calloc((size_t)n_inst, sizeof(inst_t));
    for (int i = 0; i < n_inst; ++i) C->inst[i].e0 = -1;
    for (int64_t e = 0; e < mv->nE; ++e) {
        inst_t* I = &C->inst[element_instance[e] - 1];
        if (I->e0 < 0) {
            I->e0 = e;
            I->young = mat_young[mv->element_material[e] - 1];
        }
        I->nE++;
    }
    for (int i = 0; i < n_inst; ++i) {
        element_faces(mv, &C->inst[i]);
        if (indexed) face_order(&C->inst[i]);
    }
    /* pairs, :273-311 (all exterior) or the *Contact Pair list (:1063-1102) */
    int np = 0;
    int (*pi)[2] = (int (*)[2])malloc(sizeof(int[2]) * (size_t)(n_inst * (n_inst + 1) / 2 + 1 + n_cp));
    if (n_cp > 0) {
        for (int k = 0; k < n_cp; ++k) {
            pi[np][0] = cp_instance[2 * k] - 1;
            pi[np][1] = cp_instance[2 * k + 1] - 1;
            ++np;
        }
    } else if (n_inst > 1) {
        for (int i = 0; i < n_inst; ++i)
            for (int j = (contact_flag == 2 ? i : i + 1); j < n_inst; ++j) {
                pi[np][0] = i; pi[np][1] = j; ++np;
            }
    } else {
        pi[0][0] = 0; pi[0][1] = 0; np = 1;
    }
    /* instance_pair / cp_index, :332-345 */
    C->ct = (ct_t*)calloc((size_t)(2 * np), sizeof(ct_t));
    for (int cc = 0; cc < np; ++cc) {
        const int a = pi[cc][0], b = pi[cc][1];
        const int prs[2][2] = {{a, b}, {b, a}};
        for (int r = 0; r < (a == b ? 1 : 2); ++r) {
            ct_t* T = &C->ct[C->n_ct++];
            T->i_inst = prs[r][0];
            T->j_inst = prs[r][1];
            /* surface lists of this CT entry (:347-365): side 1 of the CP when i is its instance_1 */
            const int si = (r == 0) ? 0 : 1, sj = (r == 0) ? 1 : 0;
            const int64_t* li = n_cp ? cp_elems + cp_off[2 * cc + si] : NULL;
            const int64_t ni = n_cp ? cp_off[2 * cc + si + 1] - cp_off[2 * cc + si] : -1;
            const int64_t* lj = n_cp ? cp_elems + cp_off[2 * cc + sj] : NULL;
            const int64_t nj = n_cp ? cp_off[2 * cc + sj + 1] - cp_off[2 * cc + sj] : -1;
            ivec tri = {0}, te = {0};
            surface_triangles_of(&C->inst[T->i_inst], &tri, &te, &T->nodes_i, li, ni);
            free(tri.v); free(te.v);
            surface_triangles_of(&C->inst[T->j_inst], &T->tri, &T->tri_ele, &T->nodes_j, lj, nj);
            T->young = C->inst[T->j_inst].young;  /* :367 */
            if (indexed) {
                T->in_i = (char*)calloc((size_t)mv->nN + 1, 1);
                T->in_j = (char*)calloc((size_t)mv->nN + 1, 1);
                for (int64_t q = 0; q < T->nodes_i.n; ++q) T->in_i[T->nodes_i.v[q]] = 1;
                for (int64_t q = 0; q < T->nodes_j.n; ++q) T->in_j[T->nodes_j.v[q]] = 1;
            }
        }
    }
    free(pi);
    /* element sizes, :404-421 */
    double mn = INFINITY, mx = -INFINITY;
    for (int64_t e = 0; e < mv->nE; ++e) {
        const int64_t* el = mv->elementmat + 8 * e;
        const double* p1 = mv->coordmat + 3 * (el[0] - 1);
        const int oth[3] = {1, 3, 4};
        for (int q = 0; q < 3; ++q) {
            const double* p = mv->coordmat + 3 * (el[oth[q]] - 1);
            const double L = my3norm(p1[0] - p[0], p1[1] - p[1], p1[2] - p[2]);
            if (L < mn) mn = L;
            if (L > mx) mx = L;
        }
    }
    C->elementMinSize = mn;
    C->elementMaxSize = mx;
    return C;
}

void hko_contact_set_params(hko_contact* C, double myu, double kc_o, double kc_s, double Cr_o, double Cr_s) {
    C->myu = myu; C->kc_o = kc_o; C->kc_s = kc_s; C->Cr_o = Cr_o; C->Cr_s = Cr_s;
}

void hko_contact_destroy(hko_contact* C) {
    if (!C) return;
    for (int i = 0; i < C->n_inst; ++i) {
        free(C->inst[i].faces); free(C->inst[i].sorted); free(C->inst[i].face_ele); free(C->inst[i].order);
    }
    for (int c = 0; c < C->n_ct; ++c) {
        free(C->ct[c].nodes_i.v); free(C->ct[c].nodes_j.v); free(C->ct[c].tri.v); free(C->ct[c].tri_ele.v);
        free(C->ct[c].in_i); free(C->ct[c].in_j);
    }
    free(C->inst);
    free(C->ct);
    free(C);
}

/* add_surface_triangle + the CT update, v2/HAKAI_j.jl:2167-2245 and :766-804 */
void hko_contact_element_deleted(hko_contact* C, const int64_t* element_instance, int64_t e1) {
    const int ii = (int)element_instance[e1 - 1] - 1;
    const inst_t* I = &C->inst[ii];
    const int64_t ele = e1;  /* global id; the reference compares instance-local ids, same test */
    const int64_t F = 6 * I->nE;
    ivec add_tri = {0}, add_ele = {0}, add_nodes = {0};
    const int64_t j0 = (e1 - 1 - I->e0) * 6;
    for (int j = 0; j < 6; ++j) {
        const int64_t* sj = I->sorted + 4 * (j0 + j);
        if (I->order) { /* indexed: the first face (index order) with this key, not of ele */
            for (int64_t q = order_lower(I, sj); q < F && same4(sj, I->sorted + 4 * I->order[q]); ++q) {
                const int64_t k = I->order[q];
                if (I->face_ele[k] == ele) continue;
                const int64_t* f = I->faces + 4 * k;
                iv_push(&add_tri, f[0]); iv_push(&add_tri, f[1]); iv_push(&add_tri, f[2]);
                iv_push(&add_tri, f[2]); iv_push(&add_tri, f[3]); iv_push(&add_tri, f[0]);
                iv_push(&add_ele, I->face_ele[k]);
                iv_push(&add_ele, I->face_ele[k]);
                break;
            }
            continue;
        }
        for (int64_t k = 0; k < F; ++k) {
            if (I->face_ele[k] == ele) continue;
            if (same4(sj, I->sorted + 4 * k)) {
                const int64_t* f = I->faces + 4 * k;
                iv_push(&add_tri, f[0]); iv_push(&add_tri, f[1]); iv_push(&add_tri, f[2]);
                iv_push(&add_tri, f[2]); iv_push(&add_tri, f[3]); iv_push(&add_tri, f[0]);
                iv_push(&add_ele, I->face_ele[k]);
                iv_push(&add_ele, I->face_ele[k]);
                break;
            }
        }
    }
    for (int64_t i = 0; i < add_tri.n; ++i) iv_push(&add_nodes, add_tri.v[i]);
    iv_unique_inplace(&add_nodes);
    qsort(add_nodes.v, (size_t)add_nodes.n, sizeof(int64_t), cmp_i64);
    for (int c = 0; c < C->n_ct; ++c) {
        ct_t* T = &C->ct[c];
        if (T->i_inst == ii) {
            if (T->in_i) { /* unique! keeps first occurrences: append the nodes not yet listed */
                for (int64_t i = 0; i < add_nodes.n; ++i)
                    if (!T->in_i[add_nodes.v[i]]) {
                        T->in_i[add_nodes.v[i]] = 1;
                        iv_push(&T->nodes_i, add_nodes.v[i]);
                    }
            } else {
                for (int64_t i = 0; i < add_nodes.n; ++i) iv_push(&T->nodes_i, add_nodes.v[i]);
                iv_unique_inplace(&T->nodes_i);
            }
        } else if (T->j_inst == ii) {
            if (T->in_j) {
                for (int64_t i = 0; i < add_nodes.n; ++i)
                    if (!T->in_j[add_nodes.v[i]]) {
                        T->in_j[add_nodes.v[i]] = 1;
                        iv_push(&T->nodes_j, add_nodes.v[i]);
                    }
            } else {
                for (int64_t i = 0; i < add_nodes.n; ++i) iv_push(&T->nodes_j, add_nodes.v[i]);
                iv_unique_inplace(&T->nodes_j);
            }
            for (int64_t i = 0; i < add_ele.n; ++i) iv_push(&T->tri_ele, add_ele.v[i]);
            for (int64_t i = 0; i < add_tri.n; ++i) iv_push(&T->tri, add_tri.v[i]);
        }
    }
    free(add_tri.v); free(add_ele.v); free(add_nodes.v);
}

static int64_t map_of(double p, double mn, double ddiv) { return (int64_t)ceil((p - mn) / ddiv); }

typedef struct {
    int64_t key, k;
} cellk_t;

static int cmp_cellk(const void* x, const void* y) {
    const cellk_t *a = (const cellk_t*)x, *b = (const cellk_t*)y;
    if (a->key != b->key) return a->key < b->key ? -1 : 1;
    return a->k < b->k ? -1 : a->k > b->k;
}

static int64_t cell_lower(const cellk_t* c, int64_t n, int64_t key) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (c[mid].key < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/* cal_contact_force, v2/HAKAI_j.jl:2248-2706 (one thread => c_force3[:,1]), then
 * external_force[i] += c_force3[i] (:536-538): one rounding of the Float128 sum to Float64. */
int64_t hko_contact_force(const hko_contact* C, const double* position, const double* velo, const double* diag_M,
                          const int64_t* element_flag, double* external_force) {
    const hko_model_view* mv = C->mv;
    const int64_t fn = 3 * mv->nN;
    __float128* acc = (__float128*)calloc((size_t)fn, sizeof(__float128));
    const double d_lim = C->elementMinSize * 0.3;
    int64_t n_events = 0;
    for (int c = 0; c < C->n_ct; ++c) {
        const ct_t* T = &C->ct[c];
        const int self = T->i_inst == T->j_inst;
        const int64_t nn_i = T->nodes_i.n, nn_j = T->nodes_j.n;
        if (nn_i == 0 || nn_j == 0) continue;
        double mni[3] = {INFINITY, INFINITY, INFINITY}, mxi[3] = {-INFINITY, -INFINITY, -INFINITY};
        double mnj[3] = {INFINITY, INFINITY, INFINITY}, mxj[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int64_t k = 0; k < nn_i; ++k)
            for (int d = 0; d < 3; ++d) {
                const double p = position[3 * (T->nodes_i.v[k] - 1) + d];
                if (p < mni[d]) mni[d] = p;
                if (p > mxi[d]) mxi[d] = p;
            }
        for (int64_t k = 0; k < nn_j; ++k)
            for (int d = 0; d < 3; ++d) {
                const double p = position[3 * (T->nodes_j.v[k] - 1) + d];
                if (p < mnj[d]) mnj[d] = p;
                if (p > mxj[d]) mxj[d] = p;
            }
        double rmn[3], rmx[3], amn[3];
        for (int d = 0; d < 3; ++d) {
            rmn[d] = fmax(mni[d], mnj[d]);
            rmx[d] = fmin(mxi[d], mxj[d]);
            amn[d] = fmin(mni[d], mnj[d]);
        }
        if (rmn[0] > rmx[0] || rmn[1] > rmx[1] || rmn[2] > rmx[2]) continue;
        const double ddiv = self ? C->elementMaxSize * 0.6 : C->elementMaxSize * 1.1;
        int64_t* mapi = (int64_t*)malloc(sizeof(int64_t) * 3 * (size_t)nn_i);
        for (int64_t k = 0; k < nn_i; ++k)
            for (int d = 0; d < 3; ++d) mapi[3 * k + d] = map_of(position[3 * (T->nodes_i.v[k] - 1) + d], amn[d], ddiv);
        const double kc = self ? C->kc_s : C->kc_o, Cr = self ? C->Cr_s : C->Cr_o;
        /* indexed mode: i-nodes by cell, (cell key, k) ascending */
        cellk_t* cells = NULL;
        int64_t M1 = 0, M2 = 0, M0 = 0;
        int64_t* cand = NULL;
        if (C->indexed) {
            for (int64_t k = 0; k < nn_i; ++k) {
                if (mapi[3 * k] > M0) M0 = mapi[3 * k];
                if (mapi[3 * k + 1] > M1) M1 = mapi[3 * k + 1];
                if (mapi[3 * k + 2] > M2) M2 = mapi[3 * k + 2];
            }
            cells = (cellk_t*)malloc(sizeof(cellk_t) * (size_t)nn_i);
            for (int64_t k = 0; k < nn_i; ++k) {
                cells[k].key = (mapi[3 * k] * (M1 + 1) + mapi[3 * k + 1]) * (M2 + 1) + mapi[3 * k + 2];
                cells[k].k = k;
            }
            qsort(cells, (size_t)nn_i, sizeof(cellk_t), cmp_cellk);
            cand = (int64_t*)malloc(sizeof(int64_t) * (size_t)nn_i);
        }
        const int64_t ntri = T->tri_ele.n;
        for (int64_t j = 0; j < ntri; ++j) {
            const int64_t eleid = T->tri_ele.v[j];
            if (element_flag[eleid - 1] == 0) continue;
            const int64_t j0 = T->tri.v[3 * j], j1 = T->tri.v[3 * j + 1], j2 = T->tri.v[3 * j + 2];
            const double* q0 = position + 3 * (j0 - 1);
            const double* q1 = position + 3 * (j1 - 1);
            const double* q2 = position + 3 * (j2 - 1);
            const double q0x = q0[0], q0y = q0[1], q0z = q0[2];
            const double q1x = q1[0], q1y = q1[1], q1z = q1[2];
            const double q2x = q2[0], q2y = q2[1], q2z = q2[2];
            if (q0x < rmn[0] && q1x < rmn[0] && q2x < rmn[0]) continue;
            if (q0y < rmn[1] && q1y < rmn[1] && q2y < rmn[1]) continue;
            if (q0z < rmn[2] && q1z < rmn[2] && q2z < rmn[2]) continue;
            if (q0x > rmx[0] && q1x > rmx[0] && q2x > rmx[0]) continue;
            if (q0y > rmx[1] && q1y > rmx[1] && q2y > rmx[1]) continue;
            if (q0z > rmx[2] && q1z > rmx[2] && q2z > rmx[2]) continue;
            const double cx = (q0x + q1x + q2x) / 3.0, cy = (q0y + q1y + q2y) / 3.0, cz = (q0z + q1z + q2z) / 3.0;
            const double R0 = my3norm(q0x - cx, q0y - cy, q0z - cz);
            const double R1 = my3norm(q1x - cx, q1y - cy, q1z - cz);
            const double R2 = my3norm(q2x - cx, q2y - cy, q2z - cz);
            const double Rmax = fmax(fmax(R0, R1), R2);
            const double v1x = q1x - q0x, v1y = q1y - q0y, v1z = q1z - q0z;
            const double v2x = q2x - q0x, v2y = q2y - q0y, v2z = q2z - q0z;
            const double L1 = my3norm(v1x, v1y, v1z), L2 = my3norm(v2x, v2y, v2z);
            const double Lmax = fmax(L1, L2);
            double nx = v1y * v2z - v1z * v2y, ny = v1z * v2x - v1x * v2z, nz = v1x * v2y - v1y * v2x;
            const double mag_n = sqrt(nx * nx + ny * ny + nz * nz);
            nx = nx / mag_n; ny = ny / mag_n; nz = nz / mag_n;
            const double d12 = v1x * v2x + v1y * v2y + v1z * v2z;
            const double S = 0.5 * sqrt(L1 * L1 * L2 * L2 - d12 * d12);
            const double A11 = v1x, A21 = v1y, A31 = v1z, A12 = v2x, A22 = v2y, A32 = v2z;
            const double A13 = -nx, A23 = -ny, A33 = -nz;
            const int64_t mj0[3] = {map_of(q0x, amn[0], ddiv), map_of(q0y, amn[1], ddiv), map_of(q0z, amn[2], ddiv)};
            const int64_t* el = mv->elementmat + 8 * (eleid - 1);
            int64_t ncand = nn_i;
            if (C->indexed) { /* the nodes of the 27 cells around mj0, in ascending k like the loop */
                ncand = 0;
                for (int64_t dx = -1; dx <= 1; ++dx)
                    for (int64_t dy = -1; dy <= 1; ++dy)
                        for (int64_t dz = -1; dz <= 1; ++dz) {
                            const int64_t x = mj0[0] + dx, y = mj0[1] + dy, z = mj0[2] + dz;
                            if (x < 0 || y < 0 || z < 0 || x > M0 || y > M1 || z > M2) continue;
                            const int64_t key = (x * (M1 + 1) + y) * (M2 + 1) + z;
                            for (int64_t q = cell_lower(cells, nn_i, key); q < nn_i && cells[q].key == key; ++q)
                                cand[ncand++] = cells[q].k;
                        }
                qsort(cand, (size_t)ncand, sizeof(int64_t), cmp_i64);
            }
            for (int64_t kq = 0; kq < ncand; ++kq) {
                const int64_t k = C->indexed ? cand[kq] : kq;
                if (llabs(mj0[0] - mapi[3 * k]) > 1 || llabs(mj0[1] - mapi[3 * k + 1]) > 1 ||
                    llabs(mj0[2] - mapi[3 * k + 2]) > 1)
                    continue;
                const int64_t i = T->nodes_i.v[k];
                if (self && (i == el[0] || i == el[1] || i == el[2] || i == el[3] || i == el[4] || i == el[5] ||
                             i == el[6] || i == el[7]))
                    continue;
                const double px = position[3 * (i - 1)], py = position[3 * (i - 1) + 1], pz = position[3 * (i - 1) + 2];
                if (px < rmn[0] || py < rmn[1] || pz < rmn[2]) continue;
                if (px > rmx[0] || py > rmx[1] || pz > rmx[2]) continue;
                const double dpc = my3norm(px - cx, py - cy, pz - cz);
                if (dpc >= Rmax) continue;
                const double bx = px - q0x, by = py - q0y, bz = pz - q0z;
                /* my3SolveAb, v2/HAKAI_j.jl:3342-3373 */
                const double v = (A11 * A22 * A33 + A12 * A23 * A31 + A13 * A21 * A32 - A11 * A23 * A32 -
                                  A12 * A21 * A33 - A13 * A22 * A31);
                const double im11 = A22 * A33 - A23 * A32, im21 = A23 * A31 - A21 * A33, im31 = A21 * A32 - A22 * A31;
                const double im12 = A13 * A32 - A12 * A33, im22 = A11 * A33 - A13 * A31, im32 = A12 * A31 - A11 * A32;
                const double im13 = A12 * A23 - A13 * A22, im23 = A13 * A21 - A11 * A23, im33 = A11 * A22 - A12 * A21;
                const double x1 = (im11 * bx + im12 * by + im13 * bz) / v;
                const double x2 = (im21 * bx + im22 * by + im23 * bz) / v;
                const double d = (im31 * bx + im32 * by + im33 * bz) / v;
                if (!(0.0 <= x1 && 0.0 <= x2 && x1 + x2 <= 1.0 && d > 0.0 && d <= d_lim)) continue;
                const double vx = velo[i * 3 - 3] - velo[j0 * 3 - 3];
                const double vy = velo[i * 3 - 2] - velo[j0 * 3 - 2];
                const double vz = velo[i * 3 - 1] - velo[j0 * 3 - 1];
                const double mag_v = my3norm(vx, vy, vz);
                double vex = 0.0, vey = 0.0, vez = 0.0;
                if (mag_v > 0.0) {
                    vex = vx / mag_v; vey = vy / mag_v; vez = vz / mag_v;
                }
                const double kk = T->young * S / Lmax * kc;
                const double F = kk * d;
                double fx = F * nx, fy = F * ny, fz = F * nz;
                const double Cd = 2 * sqrt(diag_M[i - 1] * kk) * Cr; /* diag_M[i]: the reference indexes dof i with a node id */
                const double fc_x = -Cd * vx, fc_y = -Cd * vy, fc_z = -Cd * vz;
                const double dot_ve_n = vex * nx + vey * ny + vez * nz;
                const double vsx = vex - dot_ve_n * nx, vsy = vey - dot_ve_n * ny, vsz = vez - dot_ve_n * nz;
                const double fric_x = -C->myu * F * vsx, fric_y = -C->myu * F * vsy, fric_z = -C->myu * F * vsz;
                fx += fric_x + fc_x;
                fy += fric_y + fc_y;
                fz += fric_z + fc_z;
                acc[3 * (i - 1) + 0] += fx;
                acc[3 * (i - 1) + 1] += fy;
                acc[3 * (i - 1) + 2] += fz;
                const int64_t tn[3] = {j0, j1, j2};
                for (int q = 0; q < 3; ++q) {
                    acc[3 * (tn[q] - 1) + 0] += -fx / 3.0;
                    acc[3 * (tn[q] - 1) + 1] += -fy / 3.0;
                    acc[3 * (tn[q] - 1) + 2] += -fz / 3.0;
                }
                ++n_events;
            }
        }
        free(mapi);
        free(cells);
        free(cand);
    }
    for (int64_t i = 0; i < fn; ++i) external_force[i] = (double)((__float128)external_force[i] + acc[i]);
    free(acc);
    return n_events;
}

double hko_contact_min_size(const hko_contact* C) { return C->elementMinSize; }
double hko_contact_max_size(const hko_contact* C) { return C->elementMaxSize; }
int hko_contact_n_pairs(const hko_contact* C) { return C->n_ct; }

int64_t hko_contact_pair_info(const hko_contact* C, int c, int64_t* out4) {
    if (c < 0 || c >= C->n_ct) return -1;
    out4[0] = C->ct[c].i_inst + 1;
    out4[1] = C->ct[c].j_inst + 1;
    out4[2] = C->ct[c].nodes_i.n;
    out4[3] = C->ct[c].tri_ele.n;
    return C->ct[c].nodes_j.n;
}
