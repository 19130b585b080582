/*
 * hakai_hip.h -- C ABI of libhakai_hip.so: the MI355X (gfx950) explicit-dynamics inner loop of
 * HAKAI (yozoyugen/HAKAI-fem v0.0.2), behind HAKAI's own driver surface
 * (HAKAI("*.inp") -> temp/fileNNN.vtk).
 *
 * Reference files (read-only, /root/reference):  "v2/" = HAKAI-v0.0.2/Julia/
 *   v2/HAKAI_j.jl        solver; time loop :487-951
 *   v2/readInpFile_j.jl  .inp reader, :152-1113
 *
 * Conventions (identical to the reference's Julia arrays):
 *   - reals are FP64; index arrays are int64 and 1-BASED (elementmat, element_material, dofs);
 *   - coordmat/position are 3 x nNode column-major (x of node n at [3(n-1)]);
 *   - nodal vectors are 3nNode with dof = 3(n-1)+c;
 *   - integ_stress/integ_strain are 6 x 8nElement column-major, Voigt (xx,yy,zz,xy,yz,xz),
 *     Gauss point index 8(e-1)+i;  integ_* scalars are 8nElement;  Qe is 24 x nElement.
 * The library owns all device memory and converts layout (Julia AoS <-> device SoA, int64 1-based
 * <-> int32 0-based) at upload/download; it never frees caller memory.
 * Errors: every int-returning call returns 0 on success and a negative code on failure;
 * hakai_last_error() gives the message (thread-local). A context is used by one host thread.
 * There is no CPU fallback: compute entry points fail with HAKAI_ERR_DEVICE when no gfx950 device
 * is present.
 */
#ifndef HAKAI_HIP_H
#define HAKAI_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HAKAI_ABI_VERSION 1

enum {
    HAKAI_OK = 0,
    HAKAI_ERR_ARG = -1,      /* bad argument / shape */
    HAKAI_ERR_DEVICE = -2,   /* no device, HIP failure */
    HAKAI_ERR_IO = -3,       /* file open / parse */
    HAKAI_ERR_STATE = -4,    /* call order (e.g. step before upload_model) */
    HAKAI_ERR_MODEL = -5,    /* a case the reference itself rejects (e.g. 1-row *Plastic -> BoundsError) */
    HAKAI_ERR_COMM = -6      /* RCCL */
};

typedef struct hakai_ctx hakai_ctx;

/* One material as readInpFile builds it (MaterialType, v2/readInpFile_j.jl:84-96). G, Dmat
 * (v2/HAKAI_j.jl:143-160) and Hd (v2/readInpFile_j.jl:763-768) are derived inside. */
typedef struct {
    double density, young, poisson;
    int32_t n_plastic;      /* rows of *Plastic (yield stress, eq. plastic strain); 0 = elastic */
    const double* plastic;  /* row-major [n_plastic][2] */
    int32_t n_ductile;      /* rows of *Damage Initiation, criterion=DUCTILE; 0 = no deletion */
    const double* ductile;  /* row-major [n_ductile][3] (fracture strain, triaxiality, rate) */
} hakai_material_t;

/* Boundary conditions, flattened BCType list (v2/readInpFile_j.jl:98-104, :843-957).
 * Group g is one *Boundary block; its entries are (dof list, value) lines applied in order, later
 * groups overwrite earlier ones (v2/HAKAI_j.jl:585-617). amp_n[g] == 0 means no amplitude. */
typedef struct {
    int32_t n_groups;
    const int32_t* amp_n;      /* [n_groups] */
    const int64_t* amp_off;    /* [n_groups] into amp_time / amp_value */
    const double* amp_time;
    const double* amp_value;
    const int64_t* entry_off;  /* [n_groups+1] */
    const double* entry_value; /* [n_entries] */
    const int64_t* dof_off;    /* [n_entries+1] into dofs */
    const int64_t* dofs;       /* 1-based dofs */
} hakai_bc_t;

/* Per-step state in the reference layout (v2/HAKAI_j.jl:225-230, :430-456). Any pointer may be
 * NULL to skip that array. velo is derived (d_disp/d_time, :628) on download. */
typedef struct {
    double* disp;                    /* 3nN */
    double* disp_pre;                /* 3nN */
    double* velo;                    /* 3nN */
    double* Q;                       /* 3nN, internal force of the last step (used by the next) */
    double* integ_stress;            /* 6 x 8nE */
    double* integ_strain;            /* 6 x 8nE */
    double* integ_yield_stress;      /* 8nE */
    double* integ_eq_plastic_strain; /* 8nE */
    double* integ_triax_stress;      /* 8nE */
    int64_t* element_flag;           /* nE (1 = active, 0 = deleted) */
    double* Qe;                      /* 24 x nE element internal forces of the last step (:1330-1340) */
} hakai_state_t;

/* ---- library / device --------------------------------------------------------------------- */
int hakai_abi_version(void);
const char* hakai_last_error(void);
/* Number of visible HIP devices (0 on a host without GPU). */
int hakai_device_count(int* n);

/* ---- persistent device context (replaces the Julia-side state of hakai(), v2/HAKAI_j.jl:81-480) */
int hakai_create(hakai_ctx** ctx, int device);
int hakai_destroy(hakai_ctx* ctx);

/* Model: mesh, materials, lumped mass (diag_M is per dof, 3nN, as v2/HAKAI_j.jl:202-215 builds
 * it; the three dofs of a node must carry the same mass, as the reference always produces). */
int hakai_upload_model(hakai_ctx* ctx, int64_t nNode, const double* coordmat, int64_t nElement,
                       const int64_t* elementmat, const int64_t* element_material, int32_t nMat,
                       const hakai_material_t* mats, const double* diag_M);
int hakai_set_bc(hakai_ctx* ctx, const hakai_bc_t* bc);

/* Fresh state on device: disp = disp_pre = Q = 0, stress/strain/eqps/triax = 0, element_flag = 1,
 * yield = first *Plastic row (v2/HAKAI_j.jl:225-239, :430-465), then the initial velocity field
 * (ic_dofs 1-based, one value per dof): disp_pre[dof] = -v*d_time, velo[dof] = v (:233-239). */
int hakai_reset_state(hakai_ctx* ctx, int64_t n_ic, const int64_t* ic_dofs, const double* ic_values,
                      double d_time);
int hakai_upload_state(hakai_ctx* ctx, const hakai_state_t* st);
int hakai_download_state(hakai_ctx* ctx, hakai_state_t* st);

/* n_steps iterations of the time-loop body v2/HAKAI_j.jl:497-764 (with contact if enabled) for
 * t = t_first .. t_first+n_steps-1 (t is Float64 like `for t = 1:time_num`). Asynchronous with
 * respect to the host until hakai_sync / a download. */
int hakai_step(hakai_ctx* ctx, double t_first, int64_t n_steps, double d_time);
/* Launch-bound step loops run from hipGraphs: hakai_step captures `graph` steps per graph
 * (default 16, an even count; tuning key "graph" or env HAKAI_GRAPH, 0 = no capture), one graph per
 * starting parity, reused for the whole run, plus 2-step graphs for a run's tail. A step is captured
 * whenever it is the same launch sequence every time -- no multi-GPU exchange, no profiling, no
 * uploaded Q, contact in its steady state -- and the call's last step always runs in stream mode.
 * Results are bit-identical to stream mode. hakai_graph_steps returns the steps run from graphs. */
int hakai_graph_steps(hakai_ctx* ctx, int64_t* n_steps);
/* Step-loop counters (tests, tools; no reference counterpart): "graph_steps", "own_steps" (element
 * steps with owner-computed assembly), "own_rows" / "own_entries" (its exported rows / per-batch
 * entries for this mesh), "own_superbatch" (batches of 32 elements per LDS summing pass: 2, or 1
 * for wide meshes), "own_slots" (LDS running sums a block keeps open at most), "own_banded" (1: the
 * blocks walk row bands of a structured wide cross-section), "own_grid" (blocks of that schedule),
 * "own_round2" (summing passes that take a second entry per thread), "exchange_retries" (steps run
 * again after a multi-GPU contact exchange block overflowed). */
int hakai_stat(hakai_ctx* ctx, const char* key, int64_t* value);
int hakai_sync(hakai_ctx* ctx);
/* Deletions so far (v2/HAKAI_j.jl:733-736): count, and up to cap (step, element 1-based) pairs. */
int hakai_deleted(hakai_ctx* ctx, int64_t* n_deleted, int64_t* log, int64_t cap);
/* Gauss points of active elements with det J < 0 in the current configuration (the reference
 * prints a warning and takes |det J|, :1736-1739). Diagnostic, runs a separate kernel. */
int hakai_negative_jacobians(hakai_ctx* ctx, int64_t* n);

/* GP -> node averages for output, on device (cal_node_stress_strain, v2/HAKAI_j.jl:3408-3486).
 * node_stress/node_strain are nN x 6 row-major; any pointer may be NULL. */
int hakai_node_stress_strain(hakai_ctx* ctx, double* node_stress, double* node_strain,
                             double* node_eq_plastic_strain, double* node_mises_stress,
                             double* node_triax_stress);

/* ---- stateless literal drop-ins (host arrays, reference layout, in place; PCIe-bound, for parity) */
/* cal_stress_hexa(Qe, integ_stress, integ_strain, integ_yield_stress, integ_eq_plastic_strain,
 *   position, d_disp, elementmat, element_flag, integ_num, Pusai_mat, MATERIAL, element_material,
 *   elementMinSize, elementVolume)  -- v2/HAKAI_j.jl:1033-1036 (called at :664-667).
 * Qe is accumulated into (the reference zeroes it first at :662); integ_num must be 8;
 * Pusai_mat and elementMinSize are implied (the kernel builds Pusai in registers). */
int hakai_stress_hexa(int device, int64_t nNode, int64_t nElement, double* Qe, double* integ_stress,
                      double* integ_strain, double* integ_yield_stress, double* integ_eq_plastic_strain,
                      const double* position, const double* d_disp, const int64_t* elementmat,
                      const int64_t* element_flag, int32_t integ_num, int32_t nMat,
                      const hakai_material_t* mats, const int64_t* element_material, double* elementVolume);
/* cal_triax_stress(integ_stress, integ_triax_stress) -- v2/HAKAI_j.jl:982 (called at :677). */
int hakai_triax_stress(int device, int64_t nGP, const double* integ_stress, double* integ_triax_stress);

/* ---- host-side setup helpers (no GPU) ------------------------------------------------------ */
/* Element volumes and lumped mass, v2/HAKAI_j.jl:183-218 (diag_M per dof, 3nN). */
int hakai_lumped_mass(int64_t nNode, const double* coordmat, int64_t nElement, const int64_t* elementmat,
                      const int64_t* element_material, int32_t nMat, const hakai_material_t* mats,
                      double mass_scaling, double* diag_M, double* elementVolume);

/* ---- profiling: per-kernel device time measured with HIP events on the context's stream ---- */
/* HAKAI_K_CONTACT: the contact step (multi-GPU contact: phases A1-A3, the search); HAKAI_K_CONTACT_SUM:
 * multi-GPU contact phase B (the gathered events' force sums of the rank's nodes). */
enum { HAKAI_K_ELEMENT = 0, HAKAI_K_NODAL = 1, HAKAI_K_BC = 2, HAKAI_K_EXCHANGE = 3, HAKAI_K_CONTACT = 4,
       HAKAI_K_CONTACT_SUM = 5, HAKAI_K_COUNT = 6 };
int hakai_profile_enable(hakai_ctx* ctx, int on);  /* all kernels on / off; resets the totals */
/* Time only the kernels whose bit (1 << HAKAI_K_*) is set (fewer events in a timed loop). */
int hakai_profile_mask(hakai_ctx* ctx, uint32_t mask);
int hakai_profile_read(hakai_ctx* ctx, int kernel, double* total_ms, int64_t* launches);
/* Tuning knobs (results are bit-identical across every setting except elem_exact, which selects
 * the arithmetic):
 *   "elem_exact"        1: reference-order element arithmetic (cal_stress_hexa op for op; GPU
 *                       trajectories bit-identical to the reference's expression order; the mode
 *                       hakai_run_inp uses), 0 (default for hakai_step): fused single-pass element
 *                       kernel (rounding-level differences); env HAKAI_ELEM_EXACT sets the default;
 *   "elem_pipe_blocks"  >0: persistent software-pipelined element kernel on that many blocks
 *                       (default 512); 0: one batch of 32 elements per block;
 *   "elem_pipe_min"     persistent kernel only with >= this many batches per block (default 2);
 *   "elem_gp_nt"        1 (default): Gauss-point state streamed with nontemporal loads and stores;
 *   "own_assembly"      1 (default; env HAKAI_OWN_ASSEMBLY): the persistent element kernel sums node
 *                       forces in LDS in element order and hands the nodal update Q (+ the rows of
 *                       nodes shared between blocks) instead of the per-element force array; meshes
 *                       it does not fit use that array (hakai_stat "own_steps"), and so does the
 *                       reference-order kernel where the lists need two entries per thread in some
 *                       pass (wide sections, hakai_stat "own_round2": the array is faster there);
 *                       2: the owner sums wherever they fit;
 *   "own_band_rows"     0 (default): the banded owner schedule plans its row-band height; >0: that
 *                       height (capped by the block's LDS slots), re-planned at the next step;
 *   "own_pass_batches"  0 (default): owner summing passes over 2 batches where the lists fit, else 1;
 *                       1 or 2: that many (re-planned at the next step);
 *   "nodal_padded"      0: CSR force gather instead of the padded [nN][8] table;
 *   "fuse_bc"           1 (default): one GPU, <= 2^18 nodes: the nodal kernel applies the BCs;
 *   "graph"             steps per captured hipGraph (even, default 16; 0 = stream mode);
 *   "contact_event_cap", "contact_candidate_cap", "contact_full_rebuild": contact buffers and
 *                       rebuild policy;
 *   "contact_exchange_deletions", "contact_exchange_bins", "contact_exchange_events": multi-GPU
 *                       contact, records per rank block of each per-step exchange (they also grow
 *                       on their own; call on every rank between steps);
 *   "contact_fuse_small" 1 (default): decks of <= 2^16 elements run fused single-workgroup phases;
 *   "contact_fuse_binfilter" 1 (default): the binning (multi-GPU: the bucket insert) and the
 *                       triangle prefilter run in one launch, side by side;
 *   "group_serial"      1 on rank 0 of a hakai_step_group: each rank's phase is drained before the
 *                       next rank's (uncontended per-rank timings on one GPU; default 0); 2: the
 *                       same, each phase enqueued behind a fixed ≈0.3 ms sleep kernel so it runs
 *                       back to back on the GPU instead of at the host's enqueue pace. */
int hakai_set_tuning(hakai_ctx* ctx, const char* key, int64_t value);

/* ---- contact: all-exterior instance-vs-instance penalty contact --------- */
/* Enables contact for the uploaded model: contact_flag as readInpFile sets it (1 = *Contact,
 * 2 = HAKAIoption=self-contact; v2/readInpFile_j.jl:1046-1060), element_instance = instance
 * (1-based, contiguous element blocks) of each element. Builds the exterior surfaces and pairs
 * (v2/HAKAI_j.jl:244-421, :1944-2164) and, once, every face an element deletion can expose
 * (:2167-2245, :766-804). Then every hakai_step
 * computes cal_contact_force (:2248-2706) into the external force before the nodal update. */
int hakai_set_contact(hakai_ctx* ctx, int32_t contact_flag, const int64_t* element_instance);
/* Same with explicit *Contact Pair surfaces (v2/readInpFile_j.jl:517-564, :1063-1102; pairs
 * v2/HAKAI_j.jl:273-345): pair k couples instances cp_instance[2k], cp_instance[2k+1] (1-based);
 * side s of pair k holds the surface's elements cp_elems[cp_elem_off[2k+s] .. cp_elem_off[2k+s+1])
 * (instance-local, 1-based). n_cp = 0 is the all-exterior case of hakai_set_contact. */
int hakai_set_contact_cp(hakai_ctx* ctx, int32_t contact_flag, const int64_t* element_instance, int32_t n_cp,
                         const int32_t* cp_instance, const int64_t* cp_elem_off, const int64_t* cp_elems);
/* Multi-GPU contact (same reference seams as hakai_set_contact_cp). Call on every
 * rank after hakai_comm_init[_local], hakai_set_element_offset and hakai_set_interface, with the
 * GLOBAL model (the arrays of hakai_upload_model / hakai_set_contact_cp for the whole mesh, and
 * its global diag_M), local_node_global[l] = global 1-based id of this rank's local node l, and
 * rank_elem_off[0..nranks] = the ranks' contiguous global element ranges (0-based, rank r holds
 * [rank_elem_off[r], rank_elem_off[r+1])). Owner-computed search: each rank keeps the triangles
 * of its elements and the contact nodes it owns (the rank of the node's lowest incident element);
 * per step the deletions are all-gathered, the pair boxes all-reduced (exact min/max), the own
 * contact-zone nodes binned and all-gathered, each rank searches its own triangles, and the events
 * are all-gathered; each rank sums the forces of its own nodes. The contact force is
 * bit-identical to one GPU. hakai_set_contact[_cp] on a rank with a communicator returns
 * HAKAI_ERR_STATE. hakai_step, hakai_reset_state, hakai_upload_state and
 * hakai_set_tuning("contact_exchange_*") are collective: every rank calls them in the same order.
 * An exchange capacity overflow grows the capacity and the step runs again (up to 8 times);
 * hakai_contact_force is refused on such a rank (step the group instead). */
int hakai_set_contact_global(hakai_ctx* ctx, int32_t contact_flag, int64_t nNode, const double* coordmat,
                             int64_t nElement, const int64_t* elementmat, const int64_t* element_material,
                             const int64_t* element_instance, const double* diag_M, const int64_t* local_node_global,
                             const int64_t* rank_elem_off, int32_t n_cp, const int32_t* cp_instance,
                             const int64_t* cp_elem_off, const int64_t* cp_elems);
/* The constants hard-coded at v2/HAKAI_j.jl:2255-2259 (defaults myu 0.25, kc_o 1, kc_s 1,
 * Cr_o 0, Cr_s 0). BASELINE's C4 runs frictionless: myu = 0. */
int hakai_set_contact_params(hakai_ctx* ctx, double myu, double kc_o, double kc_s, double Cr_o, double Cr_s);
/* Pairs (CT entries): info[5p..5p+4] = (i_instance, j_instance, #nodes_i, #triangles, #nodes_j)
 * at setup; sizes = (elementMinSize, elementMaxSize). */
int hakai_contact_info(hakai_ctx* ctx, int32_t* n_pairs, int64_t* info, int32_t cap, double* sizes);
/* Counters of the last contact step (diagnostics; syncs the stream): stats[0..cap) = events,
 * max events in any step, prefiltered triangles, nodes with contact force, live triangles, live
 * i-node entries, live j-node entries (the last three = the lengths of the reference's c_triangles,
 * c_nodes_i, c_nodes_j summed over pairs, deleted elements' triangles included); multi-GPU only:
 * [7] contact-zone nodes all ranks binned in the last step, [8] bytes this rank's exchanges receive
 * per step (the other ranks' deletion, bin and event blocks, each at its rank's capacity;
 * hakai_set_contact_global); [9] hash-grid buckets of all pairs; [10] live triangles the prefilter
 * tested in full in the last step (those whose pair has a non-empty range box; multi-GPU: this
 * rank's); [11] multi-GPU: bytes of the records in those blocks in the last step (headers + the
 * gathered counts), what [8] would be with blocks sized exactly. */
int hakai_contact_stats(hakai_ctx* ctx, int64_t* stats, int32_t cap);
/* Probe: the contact force (3nN, = external_force of step t) at the current state, no step. */
int hakai_contact_force(hakai_ctx* ctx, double t, double d_time, double* external_force);

/* ---- multi-GPU: one process per GPU, contiguous element ranges, RCCL over xGMI -------------- */
int hakai_comm_unique_id(uint8_t id[128]);
/* Attach a communicator (ncclCommInitRank) to a context created on this rank's device. */
int hakai_comm_init(hakai_ctx* ctx, int rank, int nranks, const uint8_t id[128]);
/* In-process group: contexts in one process that pass the same group_key exchange interface
 * forces with device copies instead of RCCL (several subdomains on one device; the same pack /
 * sum / fix kernels as the RCCL path). The host must step all ranks in lockstep (rank 0..n-1,
 * one hakai_step call of equal length each) on the same device: a context on another device than
 * the group's members is rejected with HAKAI_ERR_ARG (the group's kernels read the peers' buffers
 * directly; across devices use hakai_comm_init). */
int hakai_comm_init_local(hakai_ctx* ctx, int rank, int nranks, int64_t group_key);
/* Steps an in-process group (the n contexts of hakai_comm_init_local, ctxs[r] = rank r) in lockstep,
 * n_steps steps from t_first: per step every rank's contact phase A1 (deletions, live lists, boxes),
 * then every rank's A2 (box combine, binning), A3 (hash grid, triangle search), then every rank's
 * phase B (event sums), nodal and element update, so the multi-GPU contact search works in one
 * process. A contact rank of an in-process group cannot step alone (HAKAI_ERR_STATE). */
int hakai_step_group(hakai_ctx** ctxs, int32_t n, double t_first, int64_t n_steps, double d_time);
/* Interface description for this rank's local model ("multi-GPU"):
 * shared nodes (local 0-based ids, sorted by global id) with the rank range [lo, hi] of ranks
 * whose elements touch each node (hi == lo+1 for slab partitions). */
int hakai_set_interface(hakai_ctx* ctx, int64_t n_shared, const int64_t* local_node, const int32_t* rank_lo,
                        const int32_t* rank_hi);
/* Global id offset of this rank's element 0 (deletion log reports global 1-based ids). */
int hakai_set_element_offset(hakai_ctx* ctx, int64_t element_offset);

/* ---- driver surface: .inp reader, VTK writer, HAKAI(fname) ---------------------------------- */
/* Flattened ModelType (v2/readInpFile_j.jl:129-150) as the solver consumes it. Owned by the
 * library; free with hakai_inp_free. */
typedef struct {
    int64_t nNode;
    const double* coordmat;           /* 3 x nNode */
    int64_t nElement;
    const int64_t* elementmat;        /* 8 x nElement, 1-based */
    const int64_t* element_material;  /* nElement, 1-based */
    const int64_t* element_instance;  /* nElement, 1-based */
    int32_t nMat;
    const hakai_material_t* materials;
    double d_time, end_time, mass_scaling;
    int32_t contact_flag;             /* 0 none, 1 *Contact, 2 self-contact option */
    hakai_bc_t bc;
    int64_t n_ic_dofs;                /* initial velocity: dofs (1-based) and values, in IC order */
    const int64_t* ic_dofs;
    const double* ic_values;
    int32_t n_instance;
    const int64_t* instance_node_offset;    /* [n_instance] */
    const int64_t* instance_element_offset; /* [n_instance] */
    const int64_t* instance_nElement;       /* [n_instance] */
    int32_t n_cp;                           /* *Contact Pair blocks (0: all-exterior contact) */
    const int32_t* cp_instance;             /* [2 n_cp] instances (1-based) of the two surfaces */
    const int64_t* cp_elem_off;             /* [2 n_cp + 1] into cp_elems */
    const int64_t* cp_elems;                /* surface elements, instance-local 1-based */
} hakai_inp_model_t;

int hakai_inp_read(const char* path, hakai_inp_model_t** out);
void hakai_inp_free(hakai_inp_model_t* m);

/* Legacy-ASCII VTK writer with the reference's content (write_vtk, v2/HAKAI_j.jl:3517-3717):
 * writes <dir>/file%03d.vtk. node arrays as produced by hakai_node_stress_strain. */
int hakai_write_vtk(const char* dir, int index, int64_t nNode, const double* coordmat, int64_t nElement,
                    const int64_t* elementmat, const int64_t* element_flag, const double* disp,
                    const double* velo, const double* node_stress, const double* node_strain,
                    const double* node_eq_plastic_strain, const double* node_mises_stress,
                    const double* node_triax_stress);

/* Asynchronous, multi-threaded VTK writer (same bytes as hakai_write_vtk). A writer holds the
 * mesh (initial coordinates are formatted once, elementmat is copied) and writes one file at a
 * time on a background thread, so the device keeps stepping while the previous output is
 * formatted (the reference writes synchronously, v2/HAKAI_j.jl:932-942). n_threads <= 0: env
 * HAKAI_VTK_THREADS, else OMP_NUM_THREADS, else all hardware threads (at most 64).
 *   submit: copies the arrays, waits for the file in flight, starts <dir>/file%03d.vtk.
 *   acquire/commit: zero-copy variant; acquire returns the writer's fill buffers (valid until
 *   commit), commit waits for the file in flight and starts writing the filled buffers.
 *   wait: blocks until the file in flight is written; returns its status (write errors of an
 *   earlier file also surface at the next submit/commit). destroy waits, then frees. */
typedef struct hakai_vtk_writer hakai_vtk_writer;
typedef struct {
    int64_t* element_flag;           /* nElement */
    double* disp;                    /* 3 x nNode */
    double* velo;                    /* 3 x nNode */
    double* node_stress;             /* 6 x nNode */
    double* node_strain;             /* 6 x nNode */
    double* node_eq_plastic_strain;  /* nNode */
    double* node_mises_stress;       /* nNode */
    double* node_triax_stress;       /* nNode */
} hakai_vtk_arrays_t;
int hakai_vtk_writer_create(hakai_vtk_writer** w, const char* dir, int64_t nNode, const double* coordmat,
                            int64_t nElement, const int64_t* elementmat, int n_threads);
int hakai_vtk_writer_submit(hakai_vtk_writer* w, int index, const int64_t* element_flag, const double* disp,
                            const double* velo, const double* node_stress, const double* node_strain,
                            const double* node_eq_plastic_strain, const double* node_mises_stress,
                            const double* node_triax_stress);
int hakai_vtk_writer_acquire(hakai_vtk_writer* w, hakai_vtk_arrays_t* arrays);
int hakai_vtk_writer_commit(hakai_vtk_writer* w, int index);
int hakai_vtk_writer_wait(hakai_vtk_writer* w);
void hakai_vtk_writer_destroy(hakai_vtk_writer* w);

/* HAKAI(fname) (v2/HAKAI_j.jl:81-978): read, set up, run the whole step loop on `device`, write
 * out_dir/file000.vtk .. file100.vtk every floor(time_num/100) steps. verbose=1 prints the
 * reference's progress lines. Returns 0 or <0. */
int hakai_run_inp(const char* fname, const char* out_dir, int device, int verbose);

#ifdef __cplusplus
}
#endif
#endif
