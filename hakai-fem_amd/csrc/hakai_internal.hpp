// hakai_internal.hpp -- context definition shared by the translation units of libhakai_hip.so.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/hakai_hip.h"
#include "hakai_device.hpp"

namespace hkc {
struct Comm;     // multi-GPU state (hakai_comm.cpp)
struct Contact;  // contact search state (hakai_contact.hip)
int fail(int code, const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);
}  // namespace hkc

struct EventPair {
    hipEvent_t a, b;
    int kernel;
};


// BCs fused into k_nodal up to this many nodes: the per-node lookup (4 B/node, one dependent load)
// costs more than the k_bc launch it saves on large meshes (C3: nodal 0.165 -> 0.180 ms, measured
// profiles/r02_assembly_bound_sweep.log), and wins on launch-bound small decks. With owner-computed
// assembly it neither wins nor loses on C3 / the C5 slab (profiles/r03_fuse_bc_sweep.log).
constexpr long long kFuseBcMaxNodes = 1 << 18;

struct hakai_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // model
    long long nN = 0, nE = 0, nEp = 0, ld = 0;
    double* d_coord = nullptr;
    double* d_u[2] = {nullptr, nullptr};
    int cur = 0;  // d_u[cur] = disp, d_u[1-cur] = disp_pre
    double* d_mass = nullptr;
    int* d_conn = nullptr;
    int* d_flag = nullptr;
    int* d_mat = nullptr;
    hk::DevMat* d_mats = nullptr;
    std::vector<hk::DevMat> h_mats;
    bool has_ductile = false;
    double* d_stress = nullptr;
    double* d_strain = nullptr;
    double* d_eqps = nullptr;
    double* d_yield = nullptr;
    double* d_triax = nullptr;
    double* d_fe = nullptr;
    int* d_inc_ptr = nullptr;
    int* d_inc = nullptr;        // CSR incidences as force base offsets of the active layout
    int* d_inc_row = nullptr;    // the same incidences as (8e+k), for element-indexed data
    int* d_inc8 = nullptr;       // padded incidence table, null if a node has > 8 incidences
    // Element forces [nEp][8][3] (= the reference's Qe column order), row (e, k) at base 24e + 3k;
    // d_inc / d_inc8 hold the bases, and base 24nEp is an all-zero row (padding).
    long long fe_len = 0;        // doubles allocated for fe
    int max_inc = 0;
    std::vector<int> h_ptr, h_inc0;  // CSR node -> (8e+k), ascending element order
    int pipe_blocks = 512;       // persistent pipelined element kernel grid (0 = simple kernel)
    int pipe_min = 2;            // persistent kernel only with >= pipe_min batches per block (small
                                 // meshes: one batch per block, the pipeline only adds latency)
    int gp_nt = 1;               // element kernel: Gauss-point state nontemporal (loads and stores)
    int elem_exact = 0;          // tuning "elem_exact": reference-order element arithmetic
    int group_serial = 0;        // tuning "group_serial" (rank 0 of a hakai_step_group): drain every rank's
                                 // phase before the next rank's (per-rank timings without the ranks
                                 // sharing the one GPU)
    double* d_pusai = nullptr;   // cal_Pusai_hexa table for the exact element kernel (192 doubles)
    int nmat = 0;
    long long elem_offset = 0;   // global id of local element 0
    // bc
    int nbc = 0;
    int* d_bc_dof = nullptr;
    int* d_bc_grp = nullptr;
    double* d_bc_val = nullptr;
    int* d_amp_n = nullptr;
    int* d_amp_off = nullptr;
    double* d_amp_t = nullptr;
    double* d_amp_v = nullptr;
    int* d_bc_of_node = nullptr; // [nN] first resolved BC entry of each node (-1 none)
    int fuse_bc = 1;             // tuning "fuse_bc": the nodal kernel applies the BCs (one GPU)
    // state extras
    double* d_qbuf = nullptr;
    bool q_from_buf = false;
    // fe / triax hold the current state's element forces / triaxiality. With owner-computed assembly
    // the element kernel stores fe (and, in both modes, triax) only on a call's last step, so after
    // a call whose later steps a contact overflow turned into no-ops they are stale: the Qe and
    // triaxiality downloads then fail (HAKAI_ERR_STATE) until a step has run (Q stays available).
    bool fe_ok = true, triax_ok = true;
    std::vector<double> h_velo0;  // velo as uploaded / set by IC, valid until the first step
    long long steps_done = 0;
    double last_dt = 0.0;
    int* d_del_step = nullptr;   // [nEp+2] deletion step per element (0 = never), [nEp] dump slot,
                                 // [nEp+1] last step in which any element was deleted
    unsigned long long* d_negjac = nullptr;
    int* d_poison = nullptr;     // [2]: contact buffer overflow in this call (flag, step); see ElemArgs
    long long poison_step = -1;  // the step a contact overflow poisoned in the last failed call
    long long exchange_retries = 0;  // steps run again after a multi-GPU contact exchange overflow
    bool any_plastic = false;
    bool model_ok = false;
    bool state_ok = false;
    // host copies kept for setup work that needs the mesh (contact surfaces)
    std::vector<double> h_coord;  // 3nN
    std::vector<int> h_conn;      // 8nE, 0-based
    std::vector<int> h_mat;       // nE, 0-based
    std::vector<double> h_young;  // per material
    // external force (contact) -- null until contact is enabled
    double* d_fext = nullptr;
    hkc::Contact* contact = nullptr;
    // profiling
    bool prof = false;
    uint32_t prof_mask = 0;      // bit k: time kernel k (HAKAI_K_*)
    std::vector<hipEvent_t> ev_pool;
    std::vector<EventPair> ev_pending;
    double k_ms[HAKAI_K_COUNT] = {0, 0, 0, 0};
    long long k_n[HAKAI_K_COUNT] = {0, 0, 0, 0};
    // graph mode (hakai_step): `graph` steps (even) captured in one hipGraph per starting parity
    // (cur), plus a 2-step graph for the tail; the step number is read from a device counter
    // instead of kernel arguments. Slot [g][p]: g 0 = `graph` steps, 1 = 2 steps; p = parity.
    double* d_tstep = nullptr;         // [2] counter slots (slot 1-cur: previous step's number)
    const double* g_trd = nullptr;     // non-null while a step is captured: its counter slot
    hipGraphExec_t g_exec[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
    double g_dt[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
    long long g_epoch[2][2] = {{-1, -1}, {-1, -1}};
    int g_len[2][2] = {{0, 0}, {0, 0}};
    long long epoch = 0;               // bumped by every call that may change buffers or settings
    long long tdev_next = -1;          // the step the device counter is valid for (-1: unknown)
    int graph = 16;                    // tuning "graph": steps per graph (even), 0 = no capture
    long long graph_steps = 0;         // steps run from graphs (tests, stats)
    // Owner-computed assembly (tuning "own_assembly", hakai_capi.cpp own_build): the persistent
    // element kernel sums node forces in LDS in element order and stores Q (or a prefix partial plus
    // the later contributions as rows) instead of the per-element fe array.
    int own_assembly = 1;              // tuning value (1 = use when eligible; env HAKAI_OWN_ASSEMBLY)
    long long own_built_g = -1;        // grid the lists were built for (-1 none, -2 mesh not suitable)
    long long own_for_g0 = -1;         // persistent-kernel grid that build was for (a change rebuilds)
    int own_band_rows = 0;             // tuning: row-band height of the banded schedule (0: planned)
    int own_pass_batches = 0;          // tuning: batches per summing pass (0: 2 where they fit, else 1)
    bool own_valid = false;            // d_own_q/d_own_rows hold the last element step's sums
    int* d_own_off = nullptr;          // [nb+1] entry offsets per schedule position (super-batch starts)
    int* d_own_seq = nullptr;          // [nb] batch at each schedule position (ascending within a block)
    int* d_own_bstart = nullptr;       // [grid+1] first schedule position of each block
    int own_banded = 0;                // the schedule walks row bands of a structured cross-section
    long long own_round2 = 0;          // summing passes of the built lists that take a second entry per thread
    int* d_own_list = nullptr;         // 4 ints per entry (+ one no-op entry at own_nop)
    int own_nop = 0;
    int own_slots = 0;                 // LDS running-sum slots the lists use (the kernel's dynamic LDS)
    double* d_own_q = nullptr;         // [nN][3]
    int* d_own_rp = nullptr;           // [nN+1]
    double* d_own_rows = nullptr;      // [rows][3], numbered by super-batch
    int* d_own_ridx = nullptr;         // rows of node n: own_ridx[own_rp[n] .. own_rp[n+1]), element order
    double* d_own_dump = nullptr;      // [grid][8]
    long long own_rows = 0, own_entries = 0;
    long long own_steps = 0;           // element steps run with owner-computed assembly
    int own_s = 2;                     // batches per super-batch of the built lists (2, or 1)
    // multi-GPU
    hkc::Comm* comm = nullptr;
};


namespace hkc {
void prof_begin(hakai_ctx* c, int kernel, EventPair* p);
void prof_end(hakai_ctx* c, EventPair* p);
void comm_destroy(hakai_ctx* c);
int comm_reset(hakai_ctx* c);
void comm_pending_get(const hakai_ctx* c, bool* pending, int* par);
void comm_rollback(hakai_ctx* c, bool had_good, long long last_good, bool pending, int par);
// Multi-GPU hooks used by hakai_step (no-ops without a communicator).
int comm_pre_nodal(hakai_ctx* c);                    // save u_pre of interface nodes
int comm_post_nodal(hakai_ctx* c, double d_time);    // wait exchange, fix interface nodes
int comm_post_element(hakai_ctx* c, long long step); // pack interface forces, start exchange
bool comm_is_local(const hakai_ctx* c);              // in-process group stepped in lockstep
const std::vector<int>* comm_dn_nodes(const hakai_ctx* c);  // nodes shared with rank-1 (or null)
int comm_rank(const hakai_ctx* c);
int comm_size(const hakai_ctx* c);
// in-process group: dst + off[q] <- src[q] (bytes[q], 8-byte aligned), all ranks in one launch on
// c->stream (the caller orders it after the peers' producers)
constexpr int kMaxLocalGather = 64;
struct LocalGather {
    const char* src[kMaxLocalGather];
    long long bytes[kMaxLocalGather];
    long long off[kMaxLocalGather];
};
int gather_local(hakai_ctx* c, const LocalGather& g, int n, void* dst);
// RCCL only, ordered on c->stream: recv[q*bytes ..] = rank q's send; recv = MIN over ranks (uint64)
int comm_allgather_raw(hakai_ctx* c, const void* send, void* recv, size_t bytes);
int comm_allgatherv_raw(hakai_ctx* c, const void* send, void* recv, const size_t* bytes, const size_t* off);
int comm_allreduce_min_u64(hakai_ctx* c, const void* send, void* recv, size_t count);
bool comm_is_rccl(const hakai_ctx* c);
hakai_ctx* comm_peer_ctx(hakai_ctx* c, int q);                          // in-process group member q
// Contact (no-ops without hakai_set_contact).
void contact_destroy(hakai_ctx* c);
int contact_state_reset(hakai_ctx* c, const double* velo0_host);
int contact_step(hakai_ctx* c, double t, double d_time);  // one GPU: contact force of step t -> d_fext
// The contact work of a step in phases (step_once's phase bits kPhaseA1 / A2 / A3): one GPU runs it
// all in part 1. Multi-GPU (hakai_set_contact_global): part 1 = deletions of the previous step,
// live lists, this rank's pair boxes; 2 = boxes combined, this rank's contact-zone nodes binned;
// 3 = every rank's binned nodes hashed, this rank's triangles searched, its events packed;
// contact_step_b = every rank's events gathered and summed. An in-process group runs each part on
// every rank before the next part on any (hakai_step_group).
int contact_phase(hakai_ctx* c, int part, double t, double d_time);
int contact_step_b(hakai_ctx* c);
bool contact_multi(const hakai_ctx* c);                   // multi-GPU contact (phase B runs)
int contact_post_step(hakai_ctx* c);                      // multi-GPU: pack this step's deletions
int contact_check(hakai_ctx* c);                          // buffer overflow check (syncs)
void contact_after_overflow(hakai_ctx* c, long long steps_since_reset);  // host state after a poisoned call
bool contact_exchange_retry(hakai_ctx* c);                // that call overflowed a multi-GPU exchange,
                                                          // now grown: the step may run again
void graph_invalidate(hakai_ctx* c);                      // drop captured step graphs (hakai_step)
bool contact_graph_ok(const hakai_ctx* c, double t);       // step t's contact work can be captured
void contact_graph_advance(hakai_ctx* c, double t_last);   // host state after a cached graph's steps
int contact_tuning(hakai_ctx* c, const char* key, long long value);  // "contact_*" tuning keys
}  // namespace hkc
