// hakai_kernels.hpp -- host-side launch interface of the gfx950 kernels (internal to the library).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hakai_device.hpp"

namespace hk {

struct ElemArgs {
    const double* coord;   // 3nN reference position
    const double* u;       // disp  (after this step's update)
    const double* u_pre;   // disp_pre (= disp of the previous step) -> d_disp = u - u_pre
    const int* conn;       // 8nE, 0-based
    int* flag;             // nE: 1 active, 2 deleted in the previous step (fe still live), 0 deleted
    const int* mat;        // nE, 0-based
    const DevMat* mats;
    double* stress;        // SoA [6][ld]
    double* strain;        // SoA [6][ld]
    double* sc[6];         // stress + c*ld, strain + c*ld: one uniform base per component, so the
    double* ec[6];         // element kernel addresses each with an SGPR base + a 32-bit lane offset
    double* eqps;          // [ld]
    double* yield;         // [ld]
    double* triax;         // [ld]
    double* fe;            // element nodal forces [nEp][8][3] (the reference's Qe column order)
    double* vol;           // optional current volume per element (elementVolume, :1169)
    long long nE;          // elements
    long long nEp;         // elements padded to whole 32-element batches (padding: flag 0)
    long long ld;          // Gauss-point stride of the SoA arrays (8 nEp)
    int* del_step;         // [nEp+1] step at which each element was deleted (0 = never); [nEp] = dump
    int step_i;            // current step number
    const double* t_rd;    // graph mode: step number = *t_rd + 1 (read on device), else step_i
    double* t_wr;          // graph mode: block 0 stores *t_rd + 1 here (the next step's t_rd)
    int any_plastic;       // some material has a *Plastic table (eqps/yield are live)
    int pipe_blocks;        // > 0: persistent pipelined kernel with this many blocks
    int nmat;               // materials (staged in LDS when <= kMaxLdsMats)
    int gp_nt;              // 1: Gauss-point state streamed with nontemporal loads and stores
    int exact;              // 1: reference-order arithmetic (elem_step_exact), bit-identical to
                            //    cal_stress_hexa; 0: fused single-pass form (elem_step)
    const double* pusai;    // [8 GP][3][8 nodes] cal_Pusai_hexa table (exact mode)
    const int* poison;      // [0] != 0: a contact buffer overflowed in this call; every state-writing
                            // kernel is a no-op from then on (the state stays the last good step's)
    // Owner-computed assembly (tuning "own_assembly", hakai_capi.cpp own_build): block lb of the
    // persistent kernel walks its schedule positions (own_seq, own_bstart) in order and sums every node force
    // it holds in LDS, in element order, from a per-batch list of 16-B entries
    // (own_list[own_off[b] .. own_off[b+1]), see OwnEntry in hakai_kernels.hip). It stores each
    // node's complete Q, or the prefix partial P of a node whose later incidences belong to later
    // blocks, into own_q, and those later contributions one by one into own_rows. No fe traffic
    // except on a call's last step (STORE_TRIAX), which also stores fe so Q/Qe downloads stay valid.
    int own;                // 0 off; 1 or 2: batches of 32 elements per summing pass (behind a block
                            // barrier, k_element_pipe)
    int own_grid;           // blocks of the owner-assembly launch (the lists' partition)
    const int* own_seq;     // [nb] batch at each schedule position; block lb walks positions
    const int* own_bstart;  // [own_bstart[lb], own_bstart[lb+1]) (batches ascending within a block)
    const int* own_off;     // [nb+1] entry offsets, indexed by the position of a super-batch's first batch
    const int4* own_list;
    int own_nop;            // index of a no-op entry (list padding)
    int own_slots;          // LDS running-sum slots the lists use (1..1024)
    double* own_q;          // [nN][3]
    double* own_rows;       // [rows][3]
    double* own_dump;       // [grid][8] target of the no-op entries' stores
};

struct BCArgs {
    const int* dof;        // 0-based dof
    const int* grp;
    const double* val;
    int n;
    const int* amp_n;
    const int* amp_off;
    const double* amp_t;
    const double* amp_v;
    double* out;           // disp_new
    double ct;             // current time t*d_time
    const double* t_rd;    // graph mode: ct = (*t_rd + 1) * dt (read on device), else ct
    double dt;
    const int* poison;     // see ElemArgs::poison
};

struct NodalArgs {
    const double* u;       // disp
    double* u_pre_out;     // in: disp_pre, out: disp_new (ping-pong buffers, no copies)
    const double* mass;    // per node lumped mass (diag_M of each dof)
    const int* inc_ptr;    // CSR node -> incidences (fe base offsets), ascending element order
    const int* inc;
    const int* inc8;       // padded [nN][8] table of bases (pad -> zero base 24nEp) or null (CSR)
    const double* fe;
    const double* qbuf;    // if non-null: Q taken from this 3nN buffer (uploaded state), not from fe
    const double* fext;    // external force 3nN or null (= 0)
    long long nN;
    double dt;
    const int* bc_of_node; // one GPU: [nN] first entry of `bc` of each node (-1 none); the nodal
    BCArgs bc;             // kernel then applies the BCs itself (no k_bc launch)
    const int* poison;     // see ElemArgs::poison
    // Owner-computed assembly (ElemArgs::own): Q = own_q[n] + own_rows[own_ridx[own_rp[n]]] + ...
    // in element order
    const double* own_q;
    const int* own_rp;
    const int* own_ridx;
    const double* own_rows;
};


// LDS running-sum slots one block of the owner-assembly element kernel may hold: what two blocks
// per CU (80 KB each) leave next to the kernel's static arrays (node area 12.8 KB, force staging
// 12 KB per batch of a pass, double-buffered, and in reference-order mode the exchange area and
// the Pusai table, 20 KB; hakai_kernels.hip checks these sizes) and the staged materials; at most
// 2048 (11-bit slot ids in the entry lists).
constexpr int kOwnSlotsMax = 2048;
inline int own_slot_cap(bool exact, int batches_per_pass, int nmat) {
    // (force staging: 6400 B per batch -- 32 elements x 25 doubles, padded -- two buffers)
    const int stat = 12800 + 6400 * batches_per_pass * 2 + (exact ? 20608 : 0) + 64;
    const int left = 81920 - 256 - stat - nmat * (int)sizeof(DevMat);
    return left < 24 ? 0 : (left / 24 > kOwnSlotsMax ? kOwnSlotsMax : left / 24);
}

hipError_t launch_element(const ElemArgs& a, bool do_delete, bool store_triax, hipStream_t s);
hipError_t launch_negjac(const ElemArgs& a, unsigned long long* count, hipStream_t s);
hipError_t launch_nodal(const NodalArgs& a, hipStream_t s);
hipError_t launch_bc(const BCArgs& a, hipStream_t s);
// graph mode: the step counter slot read by the first step of a captured graph
hipError_t launch_set_step(double* slot, double t_prev, hipStream_t s);
hipError_t launch_hold(int rounds, hipStream_t s);  // a fixed sleep on the stream (timing aid)

// Q of every dof from fe (for downloads): Q[3n+c] = sum over incidences in element order.
hipError_t launch_gather_q(const int* inc_ptr, const int* inc, const double* fe, double* Q, long long nN,
                           hipStream_t s);
// Q from the owner-computed sums: own_q[n] + the node's rows in element order (= k_nodal MODE 3).
hipError_t launch_own_q(const double* own_q, const int* rp, const int* ridx, const double* rows, double* Q,
                        long long nN, hipStream_t s);
// AoS [gp][6] <-> SoA [6][ld] conversions used at upload/download.
hipError_t launch_aos_to_soa6(const double* aos, double* soa, long long nGP, long long ld, hipStream_t s);
hipError_t launch_soa_to_aos6(const double* soa, double* aos, long long nGP, long long ld, hipStream_t s);
// Fresh state: stress/strain/eqps/triax 0, yield from material, flags 1.
hipError_t launch_reset_gp(double* stress, double* strain, double* eqps, double* yield, double* triax, int* flag,
                           const int* mat, const DevMat* mats, long long nE, long long nEp, long long ld, hipStream_t s);
// Stand-alone triaxiality (cal_triax_stress) on an AoS [gp][6] stress array.
hipError_t launch_triax_aos(const double* stress_aos, double* triax, long long nGP, hipStream_t s);
// Output: node averages of GP quantities (cal_node_stress_strain).
hipError_t launch_node_average(const int* inc_ptr, const int* inc, const double* stress, const double* strain,
                               const double* eqps, const double* triax, long long ld, long long nN,
                               double* node_stress, double* node_strain, double* node_eqps, double* node_mises,
                               double* node_triax, hipStream_t s);

}  // namespace hk
