/*
 * hakai_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, FP64, serial by default) of the per-time-step body of the
 * reference solver HAKAI v0.0.2 (/root/reference/HAKAI-v0.0.2/Julia/HAKAI_j.jl, "v2/HAKAI_j.jl"
 * below). It exists to CHECK the MI355X product (hakai-fem_amd/); only tests/, the smoke()
 * entry point and bench.py's cpu_baseline leg may load it. The product never links it.
 *
 * Data layout mirrors the reference exactly (Julia column-major, 1-based Int64 indices):
 *   coordmat/position 3 x nN, elementmat 8 x nE (1-based), integ_stress/strain 6 x 8nE,
 *   integ_* scalars 8nE, Qe 24 x nE, nodal vectors 3nN with dof = 3(n-1)+c.
 *
 * Parity status: the reference (Julia + StaticArrays/FLoops/Quadmath) cannot run in this image
 * and ships no golden outputs, so this oracle is "parity unpinned" against
 * the reference itself. It is pinned instead by (1) analytic known-answer tests, (2) an
 * independent NumPy restatement (tests/numpy_ref.py) and (3) committed fixtures it generated
 * (tests/golden/). Arithmetic follows the reference's expression order; the three StaticArrays
 * products (B*du, D*de, B'*sigma; v2/HAKAI_j.jl:1204-1205, :1330) use fma chains because
 * StaticArrays lowers them to muladd, which fuses on FMA-capable hosts.
 */
#ifndef HAKAI_ORACLE_H
#define HAKAI_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Material as read by readInpFile (v2/readInpFile_j.jl:84-96, :684-793). */
typedef struct {
    double density, young, poisson;
    int32_t n_plastic;        /* rows of *Plastic: (yield stress, plastic strain) */
    const double* plastic;    /* row-major [n_plastic][2] */
    int32_t n_ductile;        /* rows of *Damage Initiation, criterion=DUCTILE */
    const double* ductile;    /* row-major [n_ductile][3] (strain, triaxiality, rate) */
} hko_material_in;

/* Boundary conditions (v2/readInpFile_j.jl:843-957), flattened. Group g = one *Boundary block. */
typedef struct {
    int32_t n_groups;
    const int32_t* amp_n;      /* [n_groups] amplitude points, 0 => amp = 1.0 */
    const int64_t* amp_off;    /* [n_groups] offset into amp_time/amp_value */
    const double* amp_time;
    const double* amp_value;
    const int64_t* entry_off;  /* [n_groups+1] entries of group g */
    const double* entry_value; /* [n_entries] prescribed value (times amp) */
    const int64_t* dof_off;    /* [n_entries+1] */
    const int64_t* dofs;       /* 1-based dofs */
} hko_bc;

typedef struct hko_model hko_model;

/* State arrays, all owned by the caller, reference layout. */
typedef struct {
    double* disp;      /* 3nN */
    double* disp_pre;  /* 3nN */
    double* disp_new;  /* 3nN scratch */
    double* d_disp;    /* 3nN */
    double* velo;      /* 3nN */
    double* position;  /* 3 x nN */
    double* Q;         /* 3nN */
    double* Qe;        /* 24 x nE */
    double* external_force; /* 3nN */
    double* integ_stress;   /* 6 x 8nE */
    double* integ_strain;   /* 6 x 8nE */
    double* integ_yield_stress;      /* 8nE */
    double* integ_eq_plastic_strain; /* 8nE */
    double* integ_triax_stress;      /* 8nE */
    double* elementVolume;  /* nE */
    int64_t* element_flag;  /* nE */
} hko_state;

/* Model setup: Dmat/G (v2/HAKAI_j.jl:143-172), Hd (v2/readInpFile_j.jl:763-768), Pusai
 * (v2/HAKAI_j.jl:1895-1943). d_time is the step AFTER mass scaling (v2/HAKAI_j.jl:114). */
hko_model* hko_model_create(int64_t nN, const double* coordmat, int64_t nE,
                            const int64_t* elementmat, const int64_t* element_material,
                            int32_t nmat, const hko_material_in* mats, double d_time);
void hko_model_destroy(hko_model* m);
int hko_model_set_bc(hko_model* m, const hko_bc* bc);

/* Lumped mass (v2/HAKAI_j.jl:183-218): diag_M[3nN], elementVolume[nE]. */
void hko_lumped_mass(const hko_model* m, double mass_scaling, double* diag_M, double* elementVolume);
/* Initial yield stress (v2/HAKAI_j.jl:456-465). */
void hko_init_yield(const hko_model* m, double* integ_yield_stress);
/* Shape-function derivatives at the 8 Gauss points: out[k][a][i] (k GP, a=dxi/deta/dzeta, i node). */
void hko_pusai(double out[8][3][8]);

/* Literal restatement of cal_stress_hexa (v2/HAKAI_j.jl:1033-1371). Qe must be zeroed by the
 * caller like the reference does at :662. nthreads>1 parallelises the element loop (@floop). */
void hko_cal_stress_hexa(const hko_model* m, double* Qe, double* integ_stress, double* integ_strain,
                         double* integ_yield_stress, double* integ_eq_plastic_strain,
                         const double* position, const double* d_disp, const int64_t* element_flag,
                         double* elementVolume, int nthreads);
/* cal_triax_stress (v2/HAKAI_j.jl:982-1022), StaticArrays closed-form symmetric eigvals. */
void hko_cal_triax_stress(int64_t nGP, const double* integ_stress, double* integ_triax_stress);
/* Eigenvalues of the symmetric stress tensor, StaticArrays order (eig1, eig2, eig3). */
void hko_eigvals_sym3(const double s[6], double out[3]);

/* n_steps iterations of the time loop body v2/HAKAI_j.jl:487-951 (contact-free decks),
 * t = t_first .. t_first+n_steps-1 (Float64, like `for t = 1:time_num`). Deleted elements are
 * appended to del_log as (t, element 1-based) pairs while *del_n < del_cap.
 * diag_M is per dof (3nN). Returns 0, or <0 on error. */
int hko_run(const hko_model* m, hko_state* s, const double* diag_M, double t_first, int64_t n_steps,
            int nthreads, int64_t* del_log, int64_t del_cap, int64_t* del_n);

/* ---- contact (hakai_oracle_contact.c): all-exterior instance-vs-instance contact ---------- */
typedef struct {
    int64_t nN, nE;
    const double* coordmat;          /* 3 x nN, kept by reference: must outlive the contact object */
    const int64_t* elementmat;       /* 8 x nE, 1-based */
    const int64_t* element_material; /* nE, 1-based */
} hko_model_view;
typedef struct hko_contact hko_contact;
/* Setup v2/HAKAI_j.jl:244-421 for contact_flag >= 1 (no *Contact Pair: all exterior).
 * element_instance: nE, 1-based, contiguous blocks; mat_young[mat] = Young's modulus. */
hko_contact* hko_contact_create(const hko_model_view* mv, int contact_flag, const int64_t* element_instance,
                                const double* mat_young);
/* With *Contact Pair surfaces: pair k = instances cp_instance[2k], cp_instance[2k+1] (1-based),
 * side s elements cp_elems[cp_off[2k+s] .. cp_off[2k+s+1]) (instance-local, 1-based). */
hko_contact* hko_contact_create_cp(const hko_model_view* mv, int contact_flag, const int64_t* element_instance,
                                   const double* mat_young, int32_t n_cp, const int32_t* cp_instance,
                                   const int64_t* cp_off, const int64_t* cp_elems);
/* Same, indexed = 1: identical results through sorted face keys / cell index (large models). */
hko_contact* hko_contact_create_ex(const hko_model_view* mv, int contact_flag, const int64_t* element_instance,
                                   const double* mat_young, int32_t n_cp, const int32_t* cp_instance,
                                   const int64_t* cp_off, const int64_t* cp_elems, int indexed);
void hko_contact_destroy(hko_contact* c);
/* The constants of cal_contact_force (v2/HAKAI_j.jl:2255-2259); defaults 0.25, 1, 1, 0, 0. */
void hko_contact_set_params(hko_contact* c, double myu, double kc_o, double kc_s, double Cr_o, double Cr_s);
/* external_force += contact force (Float128 accumulation, one rounding). Returns #contact events. */
int64_t hko_contact_force(const hko_contact* c, const double* position, const double* velo, const double* diag_M,
                          const int64_t* element_flag, double* external_force);
/* Surface update after element e (1-based) was deleted (v2/HAKAI_j.jl:766-804). */
void hko_contact_element_deleted(hko_contact* c, const int64_t* element_instance, int64_t e);
double hko_contact_min_size(const hko_contact* c);
double hko_contact_max_size(const hko_contact* c);
int hko_contact_n_pairs(const hko_contact* c);
/* out4 = (i_instance, j_instance, #nodes_i, #triangles); returns #nodes_j. */
int64_t hko_contact_pair_info(const hko_contact* c, int pair, int64_t* out4);

/* hko_run with contact (c may be NULL): contact force at the top of each step (:500-560) and the
 * surface update after deletions (:766-804). element_instance is needed only with contact. */
int hko_run_contact(const hko_model* m, hko_state* s, const double* diag_M, double t_first, int64_t n_steps,
                    int nthreads, int64_t* del_log, int64_t del_cap, int64_t* del_n, hko_contact* c,
                    const int64_t* element_instance);

/* cal_node_stress_strain (v2/HAKAI_j.jl:3408-3486). node_stress/strain are nN x 6 row-major
 * like the reference's (nNode,6) Julia arrays read row-wise. */
void hko_node_stress_strain(int64_t nN, int64_t nE, const int64_t* elementmat,
                            const double* integ_stress, const double* integ_strain,
                            const double* integ_eq_plastic_strain, const double* integ_triax_stress,
                            double* node_stress, double* node_strain, double* node_eq_plastic_strain,
                            double* node_mises_stress, double* node_triax_stress);

#ifdef __cplusplus
}
#endif
#endif
