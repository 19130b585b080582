// hakai_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the HAKAI explicit time step.
//
// Per step the device runs (DESIGN.md "Kernels"):
//   k_nodal    central difference u_new = f(u, u_pre, Q) per node, Q gathered from the previous
//              step's element forces in ascending element order (= the reference's serial assembly,
//              v2/HAKAI_j.jl:668-675, bit-for-bit) -- replaces :562-567 and :668-675;
//   k_bc       prescribed displacements with amplitude (v2/HAKAI_j.jl:585-617);
//   k_element  fused hex8 B-bar + J2 radial return + internal force + triaxiality + ductile
//              deletion (v2/HAKAI_j.jl:1033-1371, :982-1022, :682-764).
// d_disp (:625), disp_pre/disp shift (:626-627) and position (:650-652) are never materialised:
// disp/disp_pre are ping-pong buffers and the element kernel forms coord+u and u-u_pre on the fly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "hakai_kernels.hpp"

namespace hk {

constexpr int kBlock = 256;
constexpr int kEPB = kBlock / 8;     // elements per block
constexpr int kLdsStride = 50;       // doubles per element slot: 8 nodes x (X,du) + pad (bank spread)
// Owner-assembly force staging: [element][local node][3] with one pad double per element, so a
// pass's entries reading the same local node of consecutive elements (lane stride 8) hit spread
// banks (stride 24 doubles = 48 dwords put a 32-lane read on 4 banks: 8-way conflicts)
constexpr int kFeStride = 25;
__device__ __forceinline__ int fe_at(int l, int c) { return (l >> 3) * kFeStride + 3 * (l & 7) + c; }
// Pusai table in LDS: 24 doubles per Gauss point padded to 26 (lanes k and k+4 of an element read
// rows 4 x 24 doubles apart: the same bank; 26 keeps the rows 16-byte aligned for 128-bit reads)
constexpr int kPusStride = 26;

// Reference node index (C3D8 order) of the node with sign bits s = (x>0)<<2 | (y>0)<<1 | (z>0).
__device__ __forceinline__ int ref_of_sign(int s) {
    constexpr unsigned kTab = 0u | 4u << 3 | 3u << 6 | 7u << 9 | 1u << 12 | 5u << 15 | 2u << 18 | 6u << 21;
    return (int)((kTab >> (3 * s)) & 7u);
}

// Node sign table delta_mat (v2/HAKAI_j.jl:1900-1907).
__device__ constexpr double kSx[8] = {-1., 1., 1., -1., -1., 1., 1., -1.};
__device__ constexpr double kSy[8] = {-1., -1., 1., 1., -1., -1., 1., 1.};
__device__ constexpr double kSz[8] = {-1., -1., -1., -1., 1., 1., 1., 1.};

// ---------------------------------------------------------------------------------------------
// Element update: one 8-lane group per hex8 element, lane k = Gauss point k (gc order of
// v2/HAKAI_j.jl:1913-1920: k bits = (xi, eta, zeta) signs).
//
// Math (identical to the reference's Bfinal algebra, reorganised so no 6x24 matrix is formed):
//   P_k   = J_k^{-1} Pusai_k                    (dN_i/dx at GP k, signed det_k)
//   bbar_i = sum_k det_k P_k[:,i] / (3V),  V = sum_k |det_k|      (= BVbar rows 1-3, :1766-1780)
//   de    = sym(grad du) + (sum_i bbar_i.du_i - div_k(du)/3) (1,1,1,0,0,0)     (= Bfinal*d_u)
//   f_i  += det_k (sigma_k - tr_k/3 I) P_k[:,i] ;  f_i += (sum_k det_k tr sigma_k) bbar_i
//                                                                            (= sum_k det_k Bfinal' sigma)
// ---------------------------------------------------------------------------------------------

// Everything one lane needs from HBM for one element, gathered ahead of the compute.
struct ElemIn {
    int n, fl, mt, fb;   // stage A: local node, element flag, material, force base offset
    double x[3], du[3];  // stage B: this lane's node: position = coord + u, d_disp = u - u_pre
    double cx[3], uu[3], up[3];  // reference-order mode: the node's raw coord, u, u_pre (formed at use)
    double sig[6], eps[6], eqp, ys;
};

// Element arrays are padded to whole 32-element batches; padding elements carry flag 0 (they
// behave like deleted elements), so every load and store below is unconditional: the compiler can
// then count outstanding memory operations exactly and keep prefetches in flight across the
// stores of the previous batch (a conditional store makes its vmcnt accounting fall back to 0).
// EXACT: lane k stores the force of local node k (elem_step_exact); otherwise that of node
// ref_of_sign(k) (elem_step's relative slots).
// Addressing: a wave-uniform base (SGPRs) plus a 32-bit per-lane byte offset, so every access is a
// global_load/store with an SGPR base and one VGPR offset instead of a 64-bit VGPR address per
// array and component (12 Gauss-point components, 3 node arrays: ~60 VGPRs of addresses in the
// element kernel otherwise). The host keeps every element-kernel array below 4 GB
// (hakai_upload_model: nEp <= kMaxElemPerCtx).
template <class T>
__device__ __forceinline__ T* at32(T* base, unsigned bytes) {
    using C = typename std::conditional<std::is_const<T>::value, const char, char>::type;
    return reinterpret_cast<T*>(reinterpret_cast<C*>(base) + bytes);
}

// Orders this wave's LDS accesses around a cross-lane exchange (the 8 lanes of an element write,
// then read each other's values). A wave's LDS operations execute in order, so this only stops the
// compiler from moving LDS accesses across it; restricted to the local address space, it leaves
// the global loads and stores (the pipeline's prefetches, the write-back) free to be scheduled
// across the exchanges.
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

template <bool EXACT = false>
__device__ __forceinline__ void load_stage_a(const ElemArgs& a, long long e, int k, ElemIn& in) {
    const unsigned ue = (unsigned)e;
    in.fl = *at32(a.flag, 4u * ue);
    in.n = *at32(a.conn, 32u * ue + 4u * (unsigned)k);
    in.mt = *at32(a.mat, 4u * ue);
    const int kn = EXACT ? k : ref_of_sign(k);  // the node whose force lane k ends up with
    in.fb = (int)(24 * e + 3 * kn);
}

// Gauss-point state accesses: plain, or nontemporal (streamed once per step; keeps the caches for
// the node data and the element forces the nodal kernel reads next)
// (NT bit 0: loads, bit 1: stores)
template <int NT>
__device__ __forceinline__ double gp_ld(const double* p) {
    if (NT & 1) return __builtin_nontemporal_load(p);
    return *p;
}
template <int NT>
__device__ __forceinline__ void gp_st(double* p, double v) {
    if (NT & 2)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// stage B: the lane's node (position = coord + u, d_disp = u - u_pre) and its Gauss-point state
__device__ __forceinline__ unsigned gp_off(long long e, int k) { return 64u * (unsigned)e + 8u * (unsigned)k; }

template <bool ANY_PLASTIC, int NT = 0>
__device__ __forceinline__ void load_gp(const ElemArgs& a, long long e, int k, ElemIn& in) {
    const unsigned go = gp_off(e, k);
#pragma unroll
    for (int c = 0; c < 6; ++c) in.sig[c] = gp_ld<NT>(at32(a.sc[c], go));
#pragma unroll
    for (int c = 0; c < 6; ++c) in.eps[c] = gp_ld<NT>(at32(a.ec[c], go));
    in.eqp = 0.0;
    in.ys = 0.0;
    if (ANY_PLASTIC) {
        in.eqp = gp_ld<NT>(at32(a.eqps, go));
        in.ys = gp_ld<NT>(at32(a.yield, go));
    }
}

__device__ __forceinline__ void load_node(const ElemArgs& a, ElemIn& in) {
    const unsigned no = 24u * (unsigned)in.n;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double uc = at32(a.u, no)[c];
        in.x[c] = at32(a.coord, no)[c] + uc;
        in.du[c] = uc - at32(a.u_pre, no)[c];
    }
}

// The same node, raw: the reference-order kernel issues these loads before the previous batch's
// summing pass and forms x and du only where it stores them to LDS.
__device__ __forceinline__ void load_node_raw(const ElemArgs& a, ElemIn& in) {
    const unsigned no = 24u * (unsigned)in.n;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        in.cx[c] = at32(a.coord, no)[c];
        in.uu[c] = at32(a.u, no)[c];
        in.up[c] = at32(a.u_pre, no)[c];
    }
}

template <bool ANY_PLASTIC, int NT = 0>
__device__ __forceinline__ void load_stage_b(const ElemArgs& a, long long e, int k, ElemIn& in) {
    load_node(a, in);
    load_gp<ANY_PLASTIC, NT>(a, e, k, in);
}

// Unconditional write-back of one lane (selects, no branches): its node's force fk, its Gauss
// point's state, the element flag and the deletion log.
// PRESEL: fin/eps/eqp/ys already hold the values to store (the caller selected the previous state
// for inactive elements early, so in.sig/eps need not stay live until here).
// PART: kWbAll every store; kWbState the Gauss-point state, flag and deletion log only; kWbForce the
// node forces only (the state can then be stored before the force pass, freeing its registers).
enum { kWbAll = 0, kWbState = 1, kWbForce = 2 };
template <bool DO_DELETE, bool STORE_TRIAX, bool ANY_PLASTIC, int NT, bool EXACT_NODE = false, bool OWN = false,
          bool PRESEL = false, int PART = kWbAll>
__device__ __forceinline__ void elem_writeback(const ElemArgs& a, long long e, int k, const ElemIn& in, bool active,
                                               bool kill, const double (&fk)[3], const double (&fin)[6],
                                               const double (&eps)[6], double eqp, double ys, double tri,
                                               double* sfe = nullptr) {
    const unsigned go = gp_off(e, k);
    if (PART != kWbState && OWN) {  // owner-computed assembly: the batch's forces go to LDS [element][local node][3]
        double* fo = sfe + (threadIdx.x >> 3) * kFeStride + 3 * (EXACT_NODE ? k : ref_of_sign(k));
        fo[0] = active ? fk[0] : 0.0;
        fo[1] = active ? fk[1] : 0.0;
        fo[2] = active ? fk[2] : 0.0;
    }
    if (PART != kWbState && (!OWN || STORE_TRIAX)) {  // fe; with owner assembly only on a call's last step (Q / Qe downloads, mode switches)
        double* fg = at32(a.fe, 8u * (unsigned)in.fb);
        fg[0] = active ? fk[0] : 0.0;
        fg[1] = active ? fk[1] : 0.0;
        fg[2] = active ? fk[2] : 0.0;
    }
    if (PART == kWbForce) return;
    // deletion zeroes stress/strain (:742-756); inactive elements keep their state
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        gp_st<NT>(at32(a.sc[c], go), kill ? 0.0 : (PRESEL || active ? fin[c] : in.sig[c]));
        gp_st<NT>(at32(a.ec[c], go), kill ? 0.0 : (PRESEL || active ? eps[c] : in.eps[c]));
    }
    if (ANY_PLASTIC) {
        gp_st<NT>(at32(a.eqps, go), PRESEL || active ? eqp : in.eqp);
        gp_st<NT>(at32(a.yield, go), PRESEL || active ? ys : in.ys);
    }
    if (STORE_TRIAX) *at32(a.triax, go) = active ? tri : 0.0;
    // (a wave without a deletion and without an element deleted in the previous step changes no flag
    // and logs nothing: it skips both stores; C3 fused -1.0 %, profiles/r05_flag_store_skip_ab.log)
    if (DO_DELETE && __builtin_amdgcn_ballot_w64(kill || in.fl == 2) != 0) {
        *at32(a.flag, 4u * (unsigned)e) = kill ? 2 : (in.fl == 2 ? 0 : in.fl);  // 8 lanes, same value
        // lane 0: the element's deletion step; lanes 1-7 of a killed element: slot nEp+1, "last step
        // with a deletion" (contact rebuilds its live surface lists from it); others: dump slot nEp
        const unsigned di = kill ? (k == 0 ? (unsigned)e : (unsigned)a.nEp + 1u) : (unsigned)a.nEp;
        *at32(a.del_step, 4u * di) = a.step_i;
    }
}

// Ductile table (:720-733): fracture strain at element triaxiality t_e (t_e >= 0), last row
// outside the bracketing rows.
__device__ __forceinline__ double ductile_fr(const DevMat* M, int nd, double t_e) {
#pragma clang fp contract(off)
    double fr = M->du_eps[nd - 1];
    for (int j = 0; j + 1 < nd; ++j) {
        if (t_e >= M->du_tri[j] && t_e < M->du_tri[j + 1]) {
            fr = M->du_eps[j] + (M->du_eps[j + 1] - M->du_eps[j]) / (M->du_tri[j + 1] - M->du_tri[j]) *
                                    (t_e - M->du_tri[j]);
            break;
        }
    }
    return fr;
}

// One element step for the 8 lanes of a group (every group runs it; the element flag selects what
// is stored):  flag 1 -> full update;  flag 2 (deleted in the previous step) -> Qe and triaxiality
// become 0 and the flag 0 (the reference skips deleted elements, :1116, and their stress is zero);
// flag 0 -> state written back unchanged, Qe 0.
template <bool DO_DELETE, bool STORE_TRIAX, bool ANY_PLASTIC, bool WITH_VOL, int NT = 0, bool OWN = false>
__device__ __forceinline__ void elem_step(const ElemArgs& a, const DevMat* __restrict__ mats, long long e, int k,
                                          double* nd8, const ElemIn& in, double* sfe = nullptr) {
    const DevMat* M = mats + in.mt;
    const bool active = in.fl == 1;
    const int npp = M->npp;
    const int nd = DO_DELETE ? M->nd : 0;
    double eqp = in.eqp, ys = in.ys;

    // ---- share the 8 nodes of the element through LDS (this 8-lane group only, same wave:
    // LDS operations of one wave complete in order, so a wavefront-scope fence suffices).
    nd8[6 * k + 0] = in.x[0];
    nd8[6 * k + 1] = in.x[1];
    nd8[6 * k + 2] = in.x[2];
    nd8[6 * k + 3] = in.du[0];
    nd8[6 * k + 4] = in.du[1];
    nd8[6 * k + 5] = in.du[2];
    wave_lds_fence();

    // ---- Relative node slots. Label a node by its sign bits s = (x>0)<<2 | (y>0)<<1 | (z>0); GP k
    // carries its (xi, eta, zeta) signs in the same bits (v2/HAKAI_j.jl:1913-1920). Lane k works on
    // slot j = s ^ k: the magnitudes of dN_s/dxi at GP k (cal_Pusai_hexa, :1924-1934) then depend on
    // j only -- (1+g) where node and GP signs agree, (1-g) where they differ -- and the node's own
    // sign is tau_r * sgn(j_r) with the lane constant tau_r = (k_r ? -1 : 1). So J = diag(tau) Jt,
    // det J = tau_x tau_y tau_z det Jt and J^-1 dN_s = Jt^-1 D(j): the tau never appear, and the
    // two reduce-scatters below need no per-lane selects (reduce_scatter8_rel). The node sums run in
    // slot order, a lane-dependent permutation of the reference's node order (rounding only).
    const double g = 1.0 / __builtin_sqrt(3.0);
    const double hp = 1.0 + g, hm = 1.0 - g;
    int nodej[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) nodej[j] = 6 * ref_of_sign(j ^ k);
#define HK_MG(j, b) ((((j) >> (b)) & 1) ? hm : hp)
#define HK_SG(j, b) ((((j) >> (b)) & 1) ? 1.0 : -1.0)
#define HK_D0(j) (HK_SG(j, 2) * (1.0 / 8.0 * HK_MG(j, 1) * HK_MG(j, 0)))
#define HK_D1(j) (HK_SG(j, 1) * (1.0 / 8.0 * HK_MG(j, 2) * HK_MG(j, 0)))
#define HK_D2(j) (HK_SG(j, 0) * (1.0 / 8.0 * HK_MG(j, 2) * HK_MG(j, 1)))
    // ---- Jacobian (:1424-1434), determinant and cofactor inverse (:1436-1455), on Jt
    double J[3][3] = {{0., 0., 0.}, {0., 0., 0.}, {0., 0., 0.}};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const double* X = nd8 + nodej[j];
        const double X0 = X[0], X1 = X[1], X2 = X[2];
        const double p0 = HK_D0(j), p1 = HK_D1(j), p2 = HK_D2(j);
        J[0][0] += p0 * X0; J[0][1] += p0 * X1; J[0][2] += p0 * X2;
        J[1][0] += p1 * X0; J[1][1] += p1 * X1; J[1][2] += p1 * X2;
        J[2][0] += p2 * X0; J[2][1] += p2 * X1; J[2][2] += p2 * X2;
    }
    const double c11 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
    const double c21 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
    const double c31 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
    const double dett = J[0][0] * c11 + J[0][1] * c21 + J[0][2] * c31;
    const double det = (__builtin_popcount(k) & 1) ? -dett : dett;  // signed det J (:1436-1442)
    const double rd = 1.0 / dett;
    const double i11 = c11 * rd, i21 = c21 * rd, i31 = c31 * rd;
    const double i12 = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) * rd;
    const double i22 = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) * rd;
    const double i32 = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) * rd;
    const double i13 = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) * rd;
    const double i23 = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) * rd;
    const double i33 = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) * rd;
    double P[8][3];  // dN_s/dx_c at GP k, slot j = s ^ k
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const double p0 = HK_D0(j), p1 = HK_D1(j), p2 = HK_D2(j);
        P[j][0] = i11 * p0 + i12 * p1 + i13 * p2;
        P[j][1] = i21 * p0 + i22 * p1 + i23 * p2;
        P[j][2] = i31 * p0 + i32 * p1 + i33 * p2;
    }
#undef HK_D0
#undef HK_D1
#undef HK_D2
#undef HK_SG
#undef HK_MG

    // ---- volume and B-bar (cal_BVbar_hexa, :1705-1784): V = sum |det|; lane k ends up with the
    // B-bar vector of node ref_of_sign(k), the node whose force it also stores
    const double V = allreduce8(fabs(det));
    double wbar[3];
    {
        double v[8][3];
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int c = 0; c < 3; ++c) v[j][c] = det * P[j][c];
        reduce_scatter8_rel(v, wbar);
    }
    const double r3V = 1.0 / (3.0 * V);
    const double bb0 = wbar[0] * r3V, bb1 = wbar[1] * r3V, bb2 = wbar[2] * r3V;
    // mean volumetric strain increment / 3 over the element
    const double* dn = nd8 + nodej[0] + 3;  // d_disp of that node
    const double sdot = allreduce8(bb0 * dn[0] + bb1 * dn[1] + bb2 * dn[2]);

    // ---- strain increment at GP k (= Bfinal * d_u, :1204)
    double Gm[3][3] = {{0., 0., 0.}, {0., 0., 0.}, {0., 0., 0.}};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const double* D = nd8 + nodej[j] + 3;
        const double d0 = D[0], d1 = D[1], d2 = D[2];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            Gm[0][c] += d0 * P[j][c];
            Gm[1][c] += d1 * P[j][c];
            Gm[2][c] += d2 * P[j][c];
        }
    }
    constexpr double kThird = 1.0 / 3.0;
    const double vol = sdot - (Gm[0][0] + Gm[1][1] + Gm[2][2]) * kThird;
    double de[6];
    de[0] = Gm[0][0] + vol;
    de[1] = Gm[1][1] + vol;
    de[2] = Gm[2][2] + vol;
    de[3] = Gm[0][1] + Gm[1][0];
    de[4] = Gm[1][2] + Gm[2][1];
    de[5] = Gm[0][2] + Gm[2][0];

    // ---- elastic trial (:1205, :1220) and J2 radial return (:1227-1285)
    const double Dn = M->Dn, Do = M->Do, Ds = M->Ds;
    double fin[6];
    fin[0] = in.sig[0] + (Dn * de[0] + Do * (de[1] + de[2]));
    fin[1] = in.sig[1] + (Dn * de[1] + Do * (de[0] + de[2]));
    fin[2] = in.sig[2] + (Dn * de[2] + Do * (de[0] + de[1]));
    fin[3] = in.sig[3] + Ds * de[3];
    fin[4] = in.sig[4] + Ds * de[4];
    fin[5] = in.sig[5] + Ds * de[5];
    const double mean = (fin[0] + fin[1] + fin[2]) * kThird;
    double dv0 = fin[0] - mean, dv1 = fin[1] - mean, dv2 = fin[2] - mean;
    const double q =
        sqrt(1.5 * (dv0 * dv0 + dv1 * dv1 + dv2 * dv2 + 2.0 * (fin[3] * fin[3] + fin[4] * fin[4] + fin[5] * fin[5])));
    double sc = 1.0;
    if (ANY_PLASTIC && npp > 0 && q > ys) {
        int p = npp - 2;  // segment search (:1255-1264), 0-based p = p_index-1
        for (int j = 1; j < npp; ++j) {
            if (eqp <= M->pl_eps[j]) {
                p = j - 1;
                break;
            }
        }
        const double H = M->Hd[p];
        const double dep = (q - ys) / (3.0 * M->G + H);
        sc = (ys + H * dep) / q;
        dv0 *= sc;
        dv1 *= sc;
        dv2 *= sc;
        fin[0] = dv0 + mean;
        fin[1] = dv1 + mean;
        fin[2] = dv2 + mean;
        fin[3] *= sc;
        fin[4] *= sc;
        fin[5] *= sc;
        eqp += dep;
        ys += H * dep;
    }
    double eps[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) eps[c] = in.eps[c] + de[c];

    // ---- triaxiality (cal_triax_stress, :995-1018): mean / Mises of the final stress. The Mises
    // of the returned stress is sc*q (radial return scales the deviator), so no second sqrt.
    const double oeq = q * sc;
    // (formed where stored, a call's last step, or where the deletion test can need it)
    double tri = STORE_TRIAX ? ((oeq < 1e-10) ? 0.0 : mean / oeq) : 0.0;
    bool kill = false;
    // a wave whose Gauss points all lie below du_skip has no element average that can reach the
    // ductile table (wave-uniform skip)
    if (DO_DELETE && nd > 0 && __builtin_amdgcn_ballot_w64(eqp >= M->du_skip) != 0) {
        const double v_e = allreduce8(eqp) * 0.125;
        if (!STORE_TRIAX) tri = (oeq < 1e-10) ? 0.0 : mean / oeq;
        const double t_e = allreduce8(tri) * 0.125;
        if (!(t_e < 0.0) && v_e >= M->du_floor)  // (below du_floor no table value is reached)
            kill = active && v_e >= ductile_fr(M, nd, t_e);  // ductile table (:720-733)
    }

    // ---- internal force (Qe[:,e] += detJ * Bfinal' * sigma, :1330-1340), reduce-scattered so
    // lane k writes the 3 components of node ref_of_sign(k).
    double fk[3];
    {
        const double w00 = det * dv0, w11 = det * dv1, w22 = det * dv2;
        const double w01 = det * fin[3], w12 = det * fin[4], w02 = det * fin[5];
        double v[8][3];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const double px = P[i][0], py = P[i][1], pz = P[i][2];
            v[i][0] = w00 * px + w01 * py + w02 * pz;
            v[i][1] = w01 * px + w11 * py + w12 * pz;
            v[i][2] = w02 * px + w12 * py + w22 * pz;
        }
        reduce_scatter8_rel(v, fk);
    }
    const double S = allreduce8(det * (3.0 * mean));
    fk[0] += S * bb0;
    fk[1] += S * bb1;
    fk[2] += S * bb2;
    if (WITH_VOL) a.vol[e] = V;
    elem_writeback<DO_DELETE, STORE_TRIAX, ANY_PLASTIC, NT, false, OWN>(a, e, k, in, active, kill, fk, fin, eps, eqp,
                                                                         ys, tri, sfe);
}

// ---------------------------------------------------------------------------------------------
// Reference-order element update (tuning key "elem_exact"): cal_stress_hexa's own arithmetic
// (the oracle's restatement: oracle/hakai_oracle.c cal_BVbar_hexa, cal_Bfinal, stress_one_element),
// so the Gauss-point state, the element forces and -- with the bit-exact nodal update and contact --
// whole trajectories are the reference's bits. Same mapping as elem_step (lane k = Gauss point k),
// no contraction, fma exactly where the reference's StaticArrays products use muladd:
//   * Jacobian of GP k summed in node order 1..8 (:1424-1434) from the Pusai table (cal_Pusai_hexa,
//     built on the host with the reference's expression), cofactor det/inverse (:1436-1455), and
//     P2 = dN_i/dx (:1457-1470), computed ONCE per GP: cal_BVbar_hexa (:1716-1754) forms the same
//     P2 with 1/|det| and weights it with |det|, which is (P2/3)*det with the signed det, bit for bit;
//   * BVbar[:, 3i+c] = (sum over GPs in order of (P2/3)*|det|) / V, V = sum |det| (:1729-1780): each
//     lane writes its 8 node terms to an LDS exchange area, lane i sums node i's column over the 8
//     lanes in GP order;
//   * Bfinal (:1472-1490) is never stored: its entries are Pix, Piy, Piz, t = BVbar - P2/3 (kept in
//     registers, one division by 3 per entry) and structural zeros, fed to the 6x24 * 24 chain (:1204)
//     column by column in the reference's order; the same for D*de (:1205) and Bfinal'*sigma
//     (:1330-1340). A structural zero term is fma(0, x, acc) == acc unless acc is a zero, so dropping
//     it can change only the SIGN of a zero intermediate; every stored quantity is a sum started
//     from +0 or a previous value that is never -0, so the stored bits are the same
//     (tests/test_exact_chains.py checks the chains on ±0-rich inputs);
//   * radial return with the reference's divisions (:1251-1282): x/3 and a/q are correctly rounded
//     by div3 / div_cr below (same bits as IEEE division, fewer instructions);
//   * Qe[:, e] += detJ * Bfinal' * sigma summed over the GPs in order through the exchange area;
//     deletion averages (:701-712) summed in GP order; triaxiality in invariant form (the
//     reference's eigvals agree to rounding; it only enters the deletion test and the output).
// ---------------------------------------------------------------------------------------------
constexpr int kXbStride = 74;  // doubles of LDS per element: exchange area [8 nodes][8 lanes] + one scalar row + pad
static_assert(kEPB * kLdsStride * 8 == 12800 && kEPB * kFeStride * 8 == 6400 &&
                  kEPB * kXbStride * 8 + 8 * kPusStride * 8 == 20608,
              "own_slot_cap (hakai_kernels.hpp) assumes these LDS sizes");

// x / 3.0 correctly rounded, in two FP64 operations instead of an IEEE division sequence:
// RN(x*yh + RN(x*yl)) with yh = RN(1/3) and yl = RN(1/3 - yh) = yh * 2^-54 (1/3 = yh + yl + 2^-108/3).
// The fma's exact operand differs from x/3 by at most |x| * 2^-106 (the double-double reciprocal's
// remainder plus the rounding of x*yl), while x/3 (a multiple of 1/3 of the result's last place) is
// either representable or at least 1/6 ulp from every rounding boundary: both round the same way.
// (Round 5 used q = x*yh, q + (x - 3q)*yh, three operations, which also turned -0 into +0; this
// form keeps IEEE's -0/3 = -0.) tests/test_div3.py checks the identity against IEEE division on the
// CPU, zeros and exact multiples included. Normal-range operands (stresses, shape-function
// derivatives): x*yl stays normal for |x| > 2^-960.
__device__ __forceinline__ double div3(double x) {
    constexpr double yh = 1.0 / 3.0;
    constexpr double yl = 0x1.5555555555555p-56;  // RN(1/3 - yh)
    return __builtin_fma(x, yh, x * yl);
}

// a / b correctly rounded given rb = RN(1/b) (one IEEE division per divisor): two Newton-Markstein
// corrections of q0 = RN(a*rb). q0 is within 1.5 ulp of a/b, q1 within one ulp, and then
// RN(q1 + (a - b*q1)*rb) is RN(a/b) (Markstein's theorem: the residual is exact for a faithful
// q1, rb is the correctly rounded reciprocal). Normal-range operands (the element's stresses,
// volumes); tests/test_div3.py checks it against IEEE division on the CPU.
__device__ __forceinline__ double div_cr(double a, double b, double rb) {
    const double q0 = a * rb;
    const double q1 = __builtin_fma(__builtin_fma(-q0, b, a), rb, q0);
    return __builtin_fma(__builtin_fma(-q1, b, a), rb, q1);
}

// Ordered sum over the 8 Gauss points (lanes) of an element, for every node at once: lane k
// contributes v[i] for node i; lane i returns ((v_0[i] + v_1[i]) + ...) + v_7[i] (GP order, from
// +0 like the reference's zero-initialised accumulators). w: the element's exchange area.
__device__ __forceinline__ double gp_sum8(double* w, int k, const double (&v)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) w[8 * i + k] = v[i];
    wave_lds_fence();
    double r[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) r[kk] = w[8 * k + kk];
    wave_lds_fence();
    double acc = 0.0 + r[0];
#pragma unroll
    for (int kk = 1; kk < 8; ++kk) acc += r[kk];
    return acc;
}

// Ordered sum over the 8 lanes of a scalar (one LDS round trip); every lane gets it.
__device__ __forceinline__ double gp_all8(double* w, int k, double x) {
    w[k] = x;
    wave_lds_fence();
    double r[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) r[kk] = w[kk];
    wave_lds_fence();
    double a = 0.0 + r[0];
#pragma unroll
    for (int kk = 1; kk < 8; ++kk) a += r[kk];
    return a;
}

// Diagnostic build only (-DHK_DIAG_PHASE, tools/diag_wave.py): per-wave clock totals of the phases of
// the reference-order element step (sched_barrier pins each stamp between the phases it separates).
#ifdef HK_DIAG_PHASE
struct PhaseClock {
    long long t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    long long last = 0;
};
#define HK_PH(pc, i)                                   \
    do {                                               \
        __builtin_amdgcn_sched_barrier(0);             \
        const long long now_ = clock64();              \
        (pc).t[i] += now_ - (pc).last;                 \
        (pc).last = now_;                              \
        __builtin_amdgcn_sched_barrier(0);             \
    } while (0)
#define HK_PH_ARG , PhaseClock& pc
#define HK_PH_PASS , pc
#else
#define HK_PH(pc, i) \
    do {             \
    } while (0)
#define HK_PH_ARG
#define HK_PH_PASS
#endif

template <bool DO_DELETE, bool STORE_TRIAX, bool ANY_PLASTIC, bool WITH_VOL, int NT = 0, bool OWN = false>
__device__ __forceinline__ void elem_step_exact(const ElemArgs& a, const DevMat* __restrict__ mats, long long e,
                                                int k, double* nd8, double* xb, const double* pus,
                                                const ElemIn& in, double* sfe HK_PH_ARG) {
#pragma clang fp contract(off)
    const DevMat* M = mats + in.mt;
    const bool active = in.fl == 1;
    const int npp = M->npp;
    const int nd = DO_DELETE ? M->nd : 0;
    double eqp = in.eqp, ys = in.ys;

    // position = coord + u, d_disp = u - u_pre (load_node's expressions) from the raw loads
    nd8[6 * k + 0] = in.cx[0] + in.uu[0];
    nd8[6 * k + 1] = in.cx[1] + in.uu[1];
    nd8[6 * k + 2] = in.cx[2] + in.uu[2];
    nd8[6 * k + 3] = in.uu[0] - in.up[0];
    nd8[6 * k + 4] = in.uu[1] - in.up[1];
    nd8[6 * k + 5] = in.uu[2] - in.up[2];
    wave_lds_fence();
    HK_PH(pc, 1);

    // ---- Jacobian at GP k in node order, det and inverse (cal_Bfinal :1424-1455; cal_BVbar_hexa
    // computes the same J and det at :1716-1740). The first term starts the sum (0 + x == x).
    const double* P0 = pus + kPusStride * k;  // Pusai_mat[k][r][i] = pus[26k + 8r + i] (stage_pusai pads)
    const double* P1 = P0 + 8;
    const double* P2 = P0 + 16;
    double J11, J12, J13, J21, J22, J23, J31, J32, J33;
    {
        const double X0 = nd8[0], X1 = nd8[1], X2 = nd8[2];
        J11 = P0[0] * X0; J12 = P0[0] * X1; J13 = P0[0] * X2;
        J21 = P1[0] * X0; J22 = P1[0] * X1; J23 = P1[0] * X2;
        J31 = P2[0] * X0; J32 = P2[0] * X1; J33 = P2[0] * X2;
    }
#pragma unroll
    for (int i = 1; i < 8; ++i) {
        const double X0 = nd8[6 * i + 0], X1 = nd8[6 * i + 1], X2 = nd8[6 * i + 2];
        J11 += P0[i] * X0;
        J12 += P0[i] * X1;
        J13 += P0[i] * X2;
        J21 += P1[i] * X0;
        J22 += P1[i] * X1;
        J23 += P1[i] * X2;
        J31 += P2[i] * X0;
        J32 += P2[i] * X1;
        J33 += P2[i] * X2;
    }
    const double v = J11 * J22 * J33 + J12 * J23 * J31 + J13 * J21 * J32 - J11 * J23 * J32 - J12 * J21 * J33 -
                     J13 * J22 * J31;
    const double div_v = 1.0 / v;
    double pd[8][3];  // P2 = dN_i/dx at GP k (:1457-1470)
    {
        const double iJ11 = (J22 * J33 - J23 * J32) * div_v;
        const double iJ21 = (J23 * J31 - J21 * J33) * div_v;
        const double iJ31 = (J21 * J32 - J22 * J31) * div_v;
        const double iJ12 = (J13 * J32 - J12 * J33) * div_v;
        const double iJ22 = (J11 * J33 - J13 * J31) * div_v;
        const double iJ32 = (J12 * J31 - J11 * J32) * div_v;
        const double iJ13 = (J12 * J23 - J13 * J22) * div_v;
        const double iJ23 = (J13 * J21 - J11 * J23) * div_v;
        const double iJ33 = (J11 * J22 - J12 * J21) * div_v;
        // pd[i][r] = iJr1 * P0[i] + iJr2 * P1[i] + iJr3 * P2[i]. The Pusai table is odd in the node's
        // r-th sign, ((1/8 * delta_r) * f) * g with delta_r = +-1 (hkc::pusai_table), so
        // Pusai[k][r][i] == -Pusai[k][r][partner_r(i)] bit for bit with partner_r flipping that sign
        // (i^1, i^3, i^4 in C3D8 order); RN(-x) = -RN(x), so each product is formed once per
        // partner pair and the sums take it with a sign modifier: the same bits, 36 fewer multiplies.
        auto row = [&](int r, double a, double b, double c) {
            double q0[8], q1[8], q2[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (!(((i + 1) >> 1) & 1)) q0[i] = a * P0[i];
                if (!((i >> 1) & 1)) q1[i] = b * P1[i];
                if (!((i >> 2) & 1)) q2[i] = c * P2[i];
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const double s0 = (((i + 1) >> 1) & 1) ? -q0[i ^ 1] : q0[i];
                const double s1 = ((i >> 1) & 1) ? -q1[i ^ 3] : q1[i];
                const double s2 = ((i >> 2) & 1) ? -q2[i ^ 4] : q2[i];
                pd[i][r] = s0 + s1 + s2;
            }
        };
        row(0, iJ11, iJ12, iJ13);
        row(1, iJ21, iJ22, iJ23);
        row(2, iJ31, iJ32, iJ33);
    }

    HK_PH(pc, 2);
    // P2/3 (cal_BVbar_hexa's P2 / 3 at :1745-1750 and Bfinal's -P2/3 at :1482-1490: the same
    // correctly rounded quotient), formed once; it becomes t(i,c) below, in place
    double tk[8][3];
    // ---- V and BVbar (:1729-1780)
    double V;  // sum of |det| in GP order, in the first component's round trip
    {
        // software-pipelined: a component's exchange reads are in flight while the next
        // component's P2/3 and terms are formed (C3 exact element 1.083 -> 1.077 ms, one box)
        auto comp = [&](int c, double (&w)[8]) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                tk[i][c] = div3(pd[i][c]);
                w[i] = tk[i][c] * v;
            }
        };
        auto sum = [&](const double (&r)[8]) {
            double acc = 0.0 + r[0];
#pragma unroll
            for (int kk = 1; kk < 8; ++kk) acc += r[kk];
            return acc;
        };
        double w[8], r[8], bs[3];
        comp(0, w);
#pragma unroll
        for (int i = 0; i < 8; ++i) xb[8 * i + k] = w[i];
        xb[64 + k] = fabs(v);
        wave_lds_fence();
        double q[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) r[kk] = xb[8 * k + kk];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) q[kk] = xb[64 + kk];
        wave_lds_fence();
        comp(1, w);
        bs[0] = sum(r);
        V = sum(q);
#pragma unroll
        for (int i = 0; i < 8; ++i) xb[8 * i + k] = w[i];
        wave_lds_fence();
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) r[kk] = xb[8 * k + kk];
        wave_lds_fence();
        comp(2, w);
        bs[1] = sum(r);
#pragma unroll
        for (int i = 0; i < 8; ++i) xb[8 * i + k] = w[i];
        wave_lds_fence();
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) r[kk] = xb[8 * k + kk];
        wave_lds_fence();
        bs[2] = sum(r);
        const double rV = 1.0 / V;
#pragma unroll
        for (int c = 0; c < 3; ++c) nd8[6 * k + c] = div_cr(bs[c], V, rV);
    }
    wave_lds_fence();
    // Bfinal rows 1-3 carry t(i,c) = -P2/3 + BVbar (:1482-1490), formed once per node and component
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) tk[i][c] = nd8[6 * i + c] - tk[i][c];
    auto tq = [&](int i, int c) { return tk[i][c]; };
    HK_PH(pc, 3);

    // ---- de = Bfinal * d_u (:1204): per row, the fma chain over columns j = 3i+c in order.
    // Bfinal column (i,c) by rows: c=0: (Pix+t0, t0, t0, Piy, 0, Piz); c=1: (t1, Piy+t1, t1, Pix,
    // Piz, 0); c=2: (t2, t2, Piz+t2, 0, Piy, Pix).
    double de[6];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double* D = nd8 + 6 * i + 3;
        const double u0 = D[0], u1 = D[1], u2 = D[2];
        const double t0 = tq(i, 0), t1 = tq(i, 1), t2 = tq(i, 2);
        const double px = pd[i][0], py = pd[i][1], pz = pd[i][2];
        if (i == 0) {
            de[0] = (px + t0) * u0;
            de[1] = t0 * u0;
            de[2] = t0 * u0;
            de[3] = py * u0;
            de[4] = pz * u1;  // column 0 of row 5 is a structural zero
            de[5] = pz * u0;
        } else {
            de[0] = __builtin_fma(px + t0, u0, de[0]);
            de[1] = __builtin_fma(t0, u0, de[1]);
            de[2] = __builtin_fma(t0, u0, de[2]);
            de[3] = __builtin_fma(py, u0, de[3]);
            de[5] = __builtin_fma(pz, u0, de[5]);
            de[4] = __builtin_fma(pz, u1, de[4]);
        }
        de[0] = __builtin_fma(t1, u1, de[0]);
        de[1] = __builtin_fma(py + t1, u1, de[1]);
        de[2] = __builtin_fma(t1, u1, de[2]);
        de[3] = __builtin_fma(px, u1, de[3]);
        de[0] = __builtin_fma(t2, u2, de[0]);
        de[1] = __builtin_fma(t2, u2, de[1]);
        de[2] = __builtin_fma(pz + t2, u2, de[2]);
        de[4] = __builtin_fma(py, u2, de[4]);
        de[5] = __builtin_fma(px, u2, de[5]);
        asm volatile("" ::: "memory");  // one node's LDS operands in flight at a time (VGPRs)
    }

    HK_PH(pc, 4);
    // ---- d_o = Dmat * de (:1205): the 6x6 chain without its structural zeros
    const double Dn = M->Dn, Do = M->Do, Ds = M->Ds;
    double fin[6];
    fin[0] = in.sig[0] + __builtin_fma(Do, de[2], __builtin_fma(Do, de[1], Dn * de[0]));
    fin[1] = in.sig[1] + __builtin_fma(Do, de[2], __builtin_fma(Dn, de[1], Do * de[0]));
    fin[2] = in.sig[2] + __builtin_fma(Dn, de[2], __builtin_fma(Do, de[1], Do * de[0]));
    fin[3] = in.sig[3] + Ds * de[3];
    fin[4] = in.sig[4] + Ds * de[4];
    fin[5] = in.sig[5] + Ds * de[5];
    // ---- J2 radial return (:1227-1289)
    if (ANY_PLASTIC && npp > 0) {
        const double mean = div3(fin[0] + fin[1] + fin[2]);
        const double dev[6] = {fin[0] - mean, fin[1] - mean, fin[2] - mean, fin[3], fin[4], fin[5]};
        const double q = sqrt(1.5 * (dev[0] * dev[0] + dev[1] * dev[1] + dev[2] * dev[2] + 2.0 * (dev[3] * dev[3]) +
                                     2.0 * (dev[4] * dev[4]) + 2.0 * (dev[5] * dev[5])));
        if (q > ys) {
            int p = npp - 2;  // segment search (:1255-1264), 0-based p = p_index-1
            for (int j = 1; j < npp; ++j) {
                if (eqp <= M->pl_eps[j]) {
                    p = j - 1;
                    break;
                }
            }
            const double H = M->Hd[p];
            const double dep = (q - ys) / (3.0 * M->G + H);
            const double s = ys + H * dep;
            const double rq = 1.0 / q;
#pragma unroll
            for (int r = 0; r < 3; ++r) fin[r] = div_cr(dev[r] * s, q, rq) + mean;
#pragma unroll
            for (int r = 3; r < 6; ++r) fin[r] = div_cr(dev[r] * s, q, rq) + 0.0;
            eqp = eqp + dep;
            ys = ys + H * dep;
        }
    }
    // ---- triaxiality of the final stress (invariant form of :995-1018; the reference's eigenvalue
    // differences give the same value to rounding -- it enters only the deletion test and the output).
    // Formed where it is stored (a call's last step) or the deletion test needs it (below); an
    // inactive element's value is never used, so forming it after the inactive select changes nothing.
    auto triax = [&]() {
        const double mean = div3(fin[0] + fin[1] + fin[2]);
        const double a01 = fin[0] - fin[1], a12 = fin[1] - fin[2], a20 = fin[2] - fin[0];
        const double oeq = sqrt(0.5 * (a01 * a01 + a12 * a12 + a20 * a20) +
                                3.0 * (fin[3] * fin[3] + fin[4] * fin[4] + fin[5] * fin[5]));
        return (oeq < 1e-10) ? 0.0 : mean / oeq;
    };
    double eps[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) eps[c] = active ? in.eps[c] + de[c] : in.eps[c];
    // inactive elements keep their state (:1116-1118); selected here so the previous state does not
    // stay live through the force pass (their forces are masked at the write-back)
#pragma unroll
    for (int c = 0; c < 6; ++c) fin[c] = active ? fin[c] : in.sig[c];
    if (!active) {
        eqp = in.eqp;
        ys = in.ys;
    }

    HK_PH(pc, 5);
    double tri = STORE_TRIAX ? triax() : 0.0;
    bool kill = false;
    // element averages in GP order (:701-712); a wave whose Gauss points all lie below du_skip has
    // none that can reach the ductile table (wave-uniform skip, the same decisions)
    if (DO_DELETE && nd > 0 && __builtin_amdgcn_ballot_w64(eqp >= M->du_skip) != 0) {
        const double v_e = gp_all8(xb, k, eqp) * 0.125;  // /8, exact
        // below du_floor no fracture strain of the table is reached whatever the triaxiality: the
        // average triaxiality (a second round trip) only where it can matter; the 8 lanes of an
        // element share v_e, so the branch is uniform over them
        if (v_e >= M->du_floor) {
            if (!STORE_TRIAX) tri = triax();
            const double t_e = gp_all8(xb, k, tri) * 0.125;
            if (!(t_e < 0.0)) kill = active && v_e >= ductile_fr(M, nd, t_e);
        }
    }

    // the Gauss-point state, flag and deletion log are final here: stored before the force pass, so
    // their registers are free for it and the stores stream out under its arithmetic
    if (WITH_VOL) a.vol[e] = V;
    {
        const double nofk[3] = {0.0, 0.0, 0.0};
        elem_writeback<DO_DELETE, STORE_TRIAX, ANY_PLASTIC, NT, true, OWN, true, kWbState>(a, e, k, in, active, kill,
                                                                                          nofk, fin, eps, eqp, ys, tri);
    }
    // ---- Qe[:, e] += detJ * Bfinal' * sigma (:1330-1340), GP contributions summed in GP order
    double fk[3];
    {
        double w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // column (i, 0): (Pix+t0, t0, t0, Piy, 0, Piz)
            const double t0 = tq(i, 0);
            double acc = (pd[i][0] + t0) * fin[0];
            acc = __builtin_fma(t0, fin[1], acc);
            acc = __builtin_fma(t0, fin[2], acc);
            acc = __builtin_fma(pd[i][1], fin[3], acc);
            acc = __builtin_fma(pd[i][2], fin[5], acc);
            w[i] = v * acc;  // W*W*W*detJ*acc with W = 1
        }
        fk[0] = gp_sum8(xb, k, w);
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // column (i, 1): (t1, Piy+t1, t1, Pix, Piz, 0)
            const double t1 = tq(i, 1);
            double acc = t1 * fin[0];
            acc = __builtin_fma(pd[i][1] + t1, fin[1], acc);
            acc = __builtin_fma(t1, fin[2], acc);
            acc = __builtin_fma(pd[i][0], fin[3], acc);
            acc = __builtin_fma(pd[i][2], fin[4], acc);
            w[i] = v * acc;
        }
        fk[1] = gp_sum8(xb, k, w);
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // column (i, 2): (t2, t2, Piz+t2, 0, Piy, Pix)
            const double t2 = tq(i, 2);
            double acc = t2 * fin[0];
            acc = __builtin_fma(t2, fin[1], acc);
            acc = __builtin_fma(pd[i][2] + t2, fin[2], acc);
            acc = __builtin_fma(pd[i][1], fin[4], acc);
            acc = __builtin_fma(pd[i][0], fin[5], acc);
            w[i] = v * acc;
        }
        fk[2] = gp_sum8(xb, k, w);
    }
    HK_PH(pc, 6);
    elem_writeback<DO_DELETE, STORE_TRIAX, ANY_PLASTIC, NT, true, OWN, true, kWbForce>(a, e, k, in, active, kill, fk,
                                                                                      fin, eps, eqp, ys, tri, sfe);
    HK_PH(pc, 7);
}

// Pusai table (cal_Pusai_hexa, 192 doubles, built on the host) into LDS.
__device__ __forceinline__ void stage_pusai(const ElemArgs& a, double* s_pus) {
    for (int w = threadIdx.x; w < 192; w += blockDim.x) s_pus[w / 24 * kPusStride + w % 24] = a.pusai[w];
}

// Graph mode (hipGraph of two steps, hakai_step): the step number is not a kernel argument but a
// device counter. Every kernel of a step reads slot 1-p (the previous step's number) and adds 1;
// the element kernel, the last of the step, stores that number into slot p, which the next step
// reads. A divergent lane stores it, so it is an ordinary vector store.
// A contact buffer overflowed earlier in this hakai_step call (hakai_contact.hip, k_ct_count):
// every state-writing kernel returns at once, so the state stays the last good step's.
__device__ __forceinline__ bool poisoned(const int* p) { return p && *p; }

__device__ __forceinline__ void graph_step(ElemArgs& a) {
    if (a.t_rd) {
        const double tp = *a.t_rd;
        a.step_i = (int)tp + 1;
        if (a.t_wr && blockIdx.x == 0 && threadIdx.x == 0) *a.t_wr = tp + 1.0;
    }
}

// One batch of 32 elements per block (simple form; small meshes, the literal drop-in).
template <bool DO_DELETE, bool STORE_TRIAX, bool WITH_VOL, bool EXACT>
__global__ __launch_bounds__(kBlock, 2) void k_element(ElemArgs a) {
    __shared__ __attribute__((aligned(16))) double s_nd[kEPB * kLdsStride];
    __shared__ __attribute__((aligned(16))) double s_xb[EXACT ? kEPB * kXbStride : 1];
    __shared__ __attribute__((aligned(16))) double s_pus[EXACT ? 8 * kPusStride : 1];
    const long long vb = xcd_remap(blockIdx.x, gridDim.x);
    if (poisoned(a.poison)) return;  // block-uniform
    graph_step(a);
    const int k = threadIdx.x & 7;
    const int grp = threadIdx.x >> 3;
    if (EXACT) {
        stage_pusai(a, s_pus);
        __syncthreads();
    }
    const long long e = vb * kEPB + grp;
    ElemIn in;
    load_stage_a<EXACT>(a, e, k, in);
    if (EXACT) {
        load_node_raw(a, in);
        load_gp<true>(a, e, k, in);
    } else {
        load_stage_b<true>(a, e, k, in);
    }
#ifdef HK_DIAG_PHASE
    PhaseClock pc;
#endif
    if (EXACT)
        elem_step_exact<DO_DELETE, STORE_TRIAX, true, WITH_VOL>(a, a.mats, e, k, s_nd + grp * kLdsStride,
                                                                s_xb + grp * kXbStride, s_pus, in, nullptr HK_PH_PASS);
    else
        elem_step<DO_DELETE, STORE_TRIAX, true, WITH_VOL>(a, a.mats, e, k, s_nd + grp * kLdsStride, in);
}

// ---------------------------------------------------------------------------------------------
// Owner-computed assembly (ElemArgs::own). The block sums node forces per SUPER-BATCH of OS
// consecutive batches of its range (the last one may be shorter), one 16-B entry per thread:
//   x = target (node for ACC entries, row for EXP), y = slot bits 0-9 | flags << 10 | n << 14 |
//   lane7 << 18 | kOwnRound2 (bit 27, set in the kernel) | slot bit 10 << 28,
//   z | w << 32 = lanes 0-6, 9 bits each; a lane is ((schedule position of the element's batch -
//   the super-batch's first position) * 32 + element % 32) * 8 + local node, in ascending element
//   order.
// An ACC entry continues node `target`'s running sum in LDS slot `slot` (INIT: from 0.0, the nodal
// gather's own start) with the super-batch's contributions in element order; FIN stores the sum to
// own_q (the node's Q, or its prefix partial when later blocks hold more incidences); EXP copies one
// up to kOwnExpRows contributions (of any nodes) unchanged to consecutive own_rows. Stores are issued
// unconditionally (unused ones to a per-block dump line, which a wave's lanes share) so the loads of
// the pipeline stay in flight across the pass. The force staging is double-buffered by super-batch, so one barrier per super-batch suffices.
// ---------------------------------------------------------------------------------------------
// LDS running sums per block: what two blocks per CU leave (own_slot_cap, up to 2048), sized per
// launch to what the lists use (ElemArgs::own_slots, dynamic LDS next to the staged materials)
// batches per super-batch: 2, or 1 for meshes whose 64-element super-batches need more than 512
// entries; the host picks (own_choose), the kernel is instantiated for both
constexpr int kOwnExpRows = 4;            // contributions of one node per EXP entry
enum { kOwnInit = 1, kOwnFin = 2, kOwnExp = 4, kOwnNop = 8 };

// LDS-only barrier: the pipeline's global prefetches stay in flight.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// The thread's entry of super-batch b, prefetched a batch ahead; bit 27 of .y (free in the list's
// encoding) marks a super-batch with a second round of entries, so the pass itself loads nothing
// unless that round exists (a load inside the pass waits for every prefetch issued before it).
constexpr int kOwnRound2 = 1 << 27;
__device__ __forceinline__ int4 own_load(const ElemArgs& a, long long b) {
    const int o0 = a.own_off[b], o1 = a.own_off[b + 1];
    const int idx = o0 + (int)threadIdx.x;
    int4 en = a.own_list[idx < o1 ? idx : a.own_nop];
    en.y |= (o1 - o0 > kBlock) ? kOwnRound2 : 0;
    return en;
}

__device__ __forceinline__ int own_lane(int4 en, int j) {
    const unsigned long long lo = (unsigned long long)(unsigned)en.z | ((unsigned long long)(unsigned)en.w << 32);
    return j < 7 ? (int)((lo >> (9 * j)) & 511) : (int)(((unsigned)en.y >> 18) & 511);  // bits 18-26
}

__device__ __forceinline__ void own_entry(const ElemArgs& a, int4 en, const double* s_fe, double* s_part) {
#pragma clang fp contract(off)
    // slot: bits 0-9 and bit 28 (11 bits); bit 27: kOwnRound2
    const int slot = (en.y & 1023) | ((en.y >> 18) & 1024), flags = (en.y >> 10) & 15, n = (en.y >> 14) & 15;
    double* dump = a.own_dump + 8 * (long long)blockIdx.x;
    double v[3];
    if (flags & (kOwnExp | kOwnNop)) {  // EXP: up to kOwnExpRows contributions -> rows target + j * stride
        // (stride: the entry's group of EXP entries in this wave, in the slot field; consecutive
        // lanes write consecutive rows, own_plan)
#pragma unroll
        for (int j = 0; j < kOwnExpRows; ++j) {
            const int l = own_lane(en, j);
            double* dst = ((flags & kOwnExp) && j < n) ? a.own_rows + 3 * ((long long)en.x + (long long)j * slot) : dump;
#pragma unroll
            for (int c = 0; c < 3; ++c) dst[c] = s_fe[fe_at(l, c)];
        }
        return;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = (flags & kOwnInit) ? 0.0 : s_part[3 * slot + c];
    for (int j = 0; j < n; ++j) {
        const int l = own_lane(en, j);
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] += s_fe[fe_at(l, c)];
    }
    if (!(flags & kOwnFin)) {
#pragma unroll
        for (int c = 0; c < 3; ++c) s_part[3 * slot + c] = v[c];
    }
    double* dst = (flags & kOwnFin) ? a.own_q + 3 * (long long)en.x : dump;
#pragma unroll
    for (int c = 0; c < 3; ++c) dst[c] = v[c];
}

// Diagnostic build only (tools/variants.sh with -DHK_DIAG_WAVE, tools/diag_wave.py): per-wave clock
// totals of the persistent kernel -- loop, block-barrier wait, summing pass -- accumulated over launches
// into a device table the tool reads back. Product builds compile none of it.
#ifdef HK_DIAG_WAVE
constexpr int kDiagWaves = 8192, kDiagWords = 8;
__device__ unsigned long long g_diag[kDiagWaves * kDiagWords];
struct PassClock {
    long long bar = 0, pass = 0, n = 0;
};
#define HK_DIAG_ARG , PassClock& dg
#define HK_DIAG_PASS , dg
#else
#define HK_DIAG_ARG
#define HK_DIAG_PASS
#endif

// One summing pass: the prefetched entry of this thread, then -- only for a super-batch with more
// than kBlock entries (wide cross-sections) -- a second one, loaded here (that pass waits for it).
// Entries of one pass touch distinct LDS slots, so the two rounds need no barrier between them.
__device__ __forceinline__ void own_pass(const ElemArgs& a, int4 en, long long sb, const double* s_fe,
                                         double* s_part HK_DIAG_ARG) {
#ifdef HK_DIAG_WAVE
    const long long t0 = clock64();
#endif
    lds_barrier();  // the super-batch's forces are in s_fe, the previous pass is done with s_part
#ifdef HK_DIAG_WAVE
    const long long t1 = clock64();
#endif
    // a wave whose threads hold no entry of this round skips it (wave-uniform: no-op entries only
    // store to the dump line; C3 -0.8 to -1.0 %, C4 -1.0 %, profiles/r05_pass_skip_empty_waves_ab.log)
    const int o0 = a.own_off[sb], o1 = a.own_off[sb + 1];
    if (o0 + (int)(threadIdx.x & ~63u) < o1) own_entry(a, en, s_fe, s_part);
    if (en.y & kOwnRound2) {  // block-uniform
        const int idx = o0 + kBlock + (int)threadIdx.x;
        if (o0 + kBlock + (int)(threadIdx.x & ~63u) < o1)
            own_entry(a, a.own_list[idx < o1 ? idx : a.own_nop], s_fe, s_part);
    }
#ifdef HK_DIAG_WAVE
    const long long t2 = clock64();
    dg.bar += t1 - t0;
    dg.pass += t2 - t1;
    dg.n += 1;
#endif
}

// Persistent, software-pipelined form: each block walks a contiguous range of batches (XCD-aware),
// issuing the loads of batch b+2 (connectivity, flags) and b+1 (node gathers, Gauss-point state)
// before computing batch b, so HBM latency hides under the FP64 work even at 2 waves per SIMD.
// Material tables are staged in LDS (segment searches hit LDS, not L2).
template <bool DO_DELETE, bool STORE_TRIAX, bool ANY_PLASTIC, bool LDS_MATS, int NT, bool EXACT, int OS = 0>
__global__ __launch_bounds__(kBlock, 2) void k_element_pipe(ElemArgs a) {
    constexpr bool OWN = OS > 0;                 // owner-computed assembly, OS batches per super-batch
    constexpr int kOwnFe = OS * kEPB * kFeStride;  // staged forces per pass (doubles)
    __shared__ __attribute__((aligned(16))) double s_nd[kEPB * kLdsStride];
    __shared__ __attribute__((aligned(16))) double s_fe[OWN ? 2 * kOwnFe : 1];
    // dynamic LDS (sized by the launch, launch_pipe): [own_slots][3] running sums, then the
    // nmat staged materials
    extern __shared__ __attribute__((aligned(16))) double s_dyn[];
    double* s_part = s_dyn;
    DevMat* s_mats = reinterpret_cast<DevMat*>(s_dyn + (OWN ? 3 * a.own_slots : 0));
    __shared__ __attribute__((aligned(16))) double s_xb[EXACT ? kEPB * kXbStride : 1];
    __shared__ __attribute__((aligned(16))) double s_pus[EXACT ? 8 * kPusStride : 1];
    if (poisoned(a.poison)) return;  // block-uniform
    graph_step(a);
    const int k = threadIdx.x & 7;
    const int grp = threadIdx.x >> 3;
    if (LDS_MATS) {
        const int words = a.nmat * (int)(sizeof(DevMat) / sizeof(double));
        const double* src = reinterpret_cast<const double*>(a.mats);
        double* dst = reinterpret_cast<double*>(s_mats);
        for (int w = threadIdx.x; w < words; w += kBlock) dst[w] = src[w];
    }
    if (EXACT) stage_pusai(a, s_pus);
    if (LDS_MATS || EXACT) __syncthreads();
    const DevMat* mats = LDS_MATS ? s_mats : a.mats;
    double* nd8 = s_nd + grp * kLdsStride;
    double* xb = s_xb + (EXACT ? grp * kXbStride : 0);
    const long long nb = a.nEp / kEPB;
    // Batch schedule, as (first, stride, count):
    //  * owner assembly: each block walks a contiguous run of batches, in order (own_build's partition);
    //  * otherwise each XCD owns a contiguous run and its blocks stride through it together, so the
    //    batches that share a node layer (one element layer apart) are processed close in time on
    //    the same L2 (blocks are dealt round-robin over the 8 XCDs; C3 element reads 2.39 -> 2.20 GB).
    long long first, stride, count;
    if (OWN) {  // the block's run of schedule positions (own_build: contiguous batches, or row bands)
        first = a.own_bstart[blockIdx.x];
        stride = 1;
        count = a.own_bstart[blockIdx.x + 1] - first;
    } else if (gridDim.x % 8 != 0) {
        first = (long long)blockIdx.x * nb / gridDim.x;
        stride = 1;
        count = ((long long)blockIdx.x + 1) * nb / gridDim.x - first;
    } else {
        const long long x = blockIdx.x & 7, j = blockIdx.x >> 3, per = gridDim.x >> 3;
        const long long r0 = x * nb / 8, r1 = (x + 1) * nb / 8;
        first = r0 + j;
        stride = per;
        count = first < r1 ? (r1 - first + per - 1) / per : 0;
    }
    if (count <= 0) return;  // block-uniform
    // iterations past the end are clamped to the last batch (loaded, never computed)
    auto pos_of = [&](long long i) { return first + (i < count ? i : count - 1) * stride; };
    auto vb_of = [&](long long i) { return OWN ? (long long)a.own_seq[pos_of(i)] : pos_of(i); };
    auto elem_of = [&](long long i) { return vb_of(i) * kEPB + grp; };

#ifdef HK_DIAG_WAVE
    PassClock dg;
    const long long dg_t0 = clock64();
#endif
#ifdef HK_DIAG_PHASE
    PhaseClock pc;
#endif
    ElemIn cur, nxt;
    int4 ent_cur = {0, 0, 0, 0}, ent_nxt = {0, 0, 0, 0};
    load_stage_a<EXACT>(a, elem_of(0), k, cur);
    load_stage_a<EXACT>(a, elem_of(1), k, nxt);
    if (!EXACT) load_stage_b<ANY_PLASTIC, NT>(a, elem_of(0), k, cur);
    // (OWN: super-batch of iteration i starts at iteration i - i % OS; its entries are listed under
    // the schedule position of its first batch)
    constexpr int S = OS > 0 ? OS : 1;
    auto sb_of = [&](long long i) { return pos_of((i < count ? i : count - 1) / S * S); };
    if (OWN) ent_cur = own_load(a, sb_of(0));
    for (long long i = 0; i < count; ++i) {
        ElemIn nn;
        load_stage_a<EXACT>(a, elem_of(i + 2), k, nn);
        // (reference-order mode: its longer arithmetic holds more registers, so nothing of the
        // current batch's nodes or Gauss points is loaded a batch ahead -- only connectivity and
        // flags, two batches ahead. The node gathers are issued at the start of the batch and
        // first used by the Jacobian, the Gauss-point state first after the B-bar and strain passes.
        // Measured on C3, one box: 1.090 against 1.120 ms per step with the node gathers a batch ahead;
        // issuing this batch's node and/or Gauss-point loads at the end of the previous batch (before
        // its summing pass) spills and measured 1.18-1.28 against 1.10 ms, profiles/r03_exact_early_loads_ab.log.)
        if (!EXACT) load_stage_b<ANY_PLASTIC, NT>(a, elem_of(i + 1), k, nxt);
        if (OWN) ent_nxt = own_load(a, sb_of(i + 1));
        double* sfe = s_fe + ((i / S) & 1) * kOwnFe + (i % S) * (kEPB * kFeStride);
        if (EXACT) {
#ifdef HK_DIAG_PHASE
            pc.last = clock64();
#endif
            load_node_raw(a, cur);
            load_gp<ANY_PLASTIC, NT>(a, elem_of(i), k, cur);
            HK_PH(pc, 0);
            elem_step_exact<DO_DELETE, STORE_TRIAX, ANY_PLASTIC, false, NT, OWN>(a, mats, elem_of(i), k, nd8, xb, s_pus,
                                                                                 cur, sfe HK_PH_PASS);
        }
        else
            elem_step<DO_DELETE, STORE_TRIAX, ANY_PLASTIC, false, NT, OWN>(a, mats, elem_of(i), k, nd8, cur, sfe);
        if (OWN) {
            // block-uniform branch; the compiler's load accounting is the same on both sides
            // (checked in the ISA: identical vmcnt waits with or without balancing stores)
            if ((i + 1) % S == 0 || i + 1 == count)
                own_pass(a, ent_cur, sb_of(i), s_fe + ((i / S) & 1) * kOwnFe, s_part HK_DIAG_PASS);
            ent_cur = ent_nxt;
        }
        cur = nxt;
        nxt = nn;
    }
#ifdef HK_DIAG_WAVE
    const long long dg_t1 = clock64();
    const unsigned gw = blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0 && gw < (unsigned)kDiagWaves) {
        unsigned long long* d = g_diag + (size_t)kDiagWords * gw;
        atomicAdd(d + 0, (unsigned long long)(dg_t1 - dg_t0));
        atomicAdd(d + 1, (unsigned long long)dg.bar);
        atomicAdd(d + 2, (unsigned long long)dg.pass);
        atomicAdd(d + 3, (unsigned long long)dg.n);
        atomicAdd(d + 4, (unsigned long long)count);
        atomicAdd(d + 5, 1ull);
        atomicExch(d + 6, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4));  // HW_ID
#ifdef HK_DIAG_PHASE
        unsigned long long* q = g_diag + (size_t)kDiagWords * (kDiagWaves / 2 + gw);
        for (int j = 0; j < 8; ++j) atomicAdd(q + j, (unsigned long long)pc.t[j]);
#endif
    }
#endif
}

#ifdef HK_DIAG_WAVE
extern "C" int hk_diag_reset() {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_diag)) != hipSuccess) return -1;
    return hipMemset(p, 0, sizeof(g_diag)) == hipSuccess ? 0 : -1;
}
extern "C" int hk_diag_read(unsigned long long* out, int n) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag), sizeof(unsigned long long) * (size_t)std::min(n, kDiagWaves * kDiagWords)) == hipSuccess ? 0 : -1;
}
#endif

// Runtime flags -> template instantiations.
template <bool EXACT>
static void launch_element_w(const ElemArgs& a, bool do_delete, bool store_triax, bool with_vol, unsigned grid,
                             hipStream_t s) {
    if (with_vol) {
        hipLaunchKernelGGL((k_element<false, false, true, EXACT>), dim3(grid), dim3(kBlock), 0, s, a);
    } else if (do_delete) {
        if (store_triax)
            hipLaunchKernelGGL((k_element<true, true, false, EXACT>), dim3(grid), dim3(kBlock), 0, s, a);
        else
            hipLaunchKernelGGL((k_element<true, false, false, EXACT>), dim3(grid), dim3(kBlock), 0, s, a);
    } else {
        if (store_triax)
            hipLaunchKernelGGL((k_element<false, true, false, EXACT>), dim3(grid), dim3(kBlock), 0, s, a);
        else
            hipLaunchKernelGGL((k_element<false, false, false, EXACT>), dim3(grid), dim3(kBlock), 0, s, a);
    }
}

template <bool ANY_PLASTIC, bool LDS_MATS, int NT, bool EXACT, int OS>
static void launch_pipe(const ElemArgs& a, bool do_delete, bool store_triax, unsigned grid, hipStream_t s) {
    const size_t dyn = (OS > 0 ? 24 * (size_t)a.own_slots : 0) + (LDS_MATS ? sizeof(DevMat) * (size_t)a.nmat : 0);
    if (do_delete) {
        if (store_triax)
            hipLaunchKernelGGL((k_element_pipe<true, true, ANY_PLASTIC, LDS_MATS, NT, EXACT, OS>), dim3(grid),
                               dim3(kBlock), dyn, s, a);
        else
            hipLaunchKernelGGL((k_element_pipe<true, false, ANY_PLASTIC, LDS_MATS, NT, EXACT, OS>), dim3(grid),
                               dim3(kBlock), dyn, s, a);
    } else {
        if (store_triax)
            hipLaunchKernelGGL((k_element_pipe<false, true, ANY_PLASTIC, LDS_MATS, NT, EXACT, OS>), dim3(grid),
                               dim3(kBlock), dyn, s, a);
        else
            hipLaunchKernelGGL((k_element_pipe<false, false, ANY_PLASTIC, LDS_MATS, NT, EXACT, OS>), dim3(grid),
                               dim3(kBlock), dyn, s, a);
    }
}

template <bool ANY_PLASTIC, bool LDS_MATS, bool EXACT, int OS>
static void launch_pipe_nt(const ElemArgs& a, bool do_delete, bool store_triax, unsigned grid, hipStream_t s) {
    if (a.gp_nt)
        launch_pipe<ANY_PLASTIC, LDS_MATS, 3, EXACT, OS>(a, do_delete, store_triax, grid, s);
    else
        launch_pipe<ANY_PLASTIC, LDS_MATS, 0, EXACT, OS>(a, do_delete, store_triax, grid, s);
}

template <bool ANY_PLASTIC, bool LDS_MATS, bool EXACT>
static void launch_pipe_os(const ElemArgs& a, bool do_delete, bool store_triax, unsigned grid, hipStream_t s) {
    if (a.own == 1)
        launch_pipe_nt<ANY_PLASTIC, true, EXACT, 1>(a, do_delete, store_triax, grid, s);
    else if (a.own == 2)
        launch_pipe_nt<ANY_PLASTIC, true, EXACT, 2>(a, do_delete, store_triax, grid, s);
    else
        launch_pipe_nt<ANY_PLASTIC, LDS_MATS, EXACT, 0>(a, do_delete, store_triax, grid, s);
}

template <bool EXACT>
static void launch_pipe_p(const ElemArgs& a, bool do_delete, bool store_triax, unsigned grid, hipStream_t s) {
    const bool lds = a.nmat <= kMaxLdsMats;
    if (a.any_plastic) {
        if (lds) launch_pipe_os<true, true, EXACT>(a, do_delete, store_triax, grid, s);
        else launch_pipe_os<true, false, EXACT>(a, do_delete, store_triax, grid, s);
    } else {
        if (lds) launch_pipe_os<false, true, EXACT>(a, do_delete, store_triax, grid, s);
        else launch_pipe_os<false, false, EXACT>(a, do_delete, store_triax, grid, s);
    }
}

hipError_t launch_element(const ElemArgs& a, bool do_delete, bool store_triax, hipStream_t s) {
    if (a.nE <= 0) return hipSuccess;
    if (a.exact && !a.pusai) return hipErrorInvalidValue;
    const long long nb = a.nEp / kEPB;
    if (nb <= 0) return hipSuccess;
    if (a.own) {  // owner-computed assembly: persistent kernel only (own_build sized its lists for it)
        if (a.own > 2 || a.vol || a.pipe_blocks <= 0 || a.nmat > kMaxLdsMats || !a.own_off || !a.own_list ||
            !a.own_seq || !a.own_bstart || !a.own_q || !a.own_dump || a.own_slots < 1 ||
            a.own_slots > own_slot_cap(a.exact != 0, a.own, a.nmat))
            return hipErrorInvalidValue;
        if (a.own_grid <= 0 || a.own_grid > nb) return hipErrorInvalidValue;  // (own_bstart has grid+1 entries)
        if (a.exact)
            launch_pipe_p<true>(a, do_delete, store_triax, (unsigned)a.own_grid, s);
        else
            launch_pipe_p<false>(a, do_delete, store_triax, (unsigned)a.own_grid, s);
        return hipGetLastError();
    }
    if (a.pipe_blocks > 0 && !a.vol) {
        const unsigned grid = (unsigned)std::min<long long>(nb, a.pipe_blocks);
        if (a.exact)
            launch_pipe_p<true>(a, do_delete, store_triax, grid, s);
        else
            launch_pipe_p<false>(a, do_delete, store_triax, grid, s);
        return hipGetLastError();
    }
    if (a.exact)
        launch_element_w<true>(a, do_delete, store_triax, a.vol != nullptr, (unsigned)nb, s);
    else
        launch_element_w<false>(a, do_delete, store_triax, a.vol != nullptr, (unsigned)nb, s);
    return hipGetLastError();
}

// Negative-Jacobian diagnostic (the reference prints a warning, v2/HAKAI_j.jl:1736-1739): counts
// Gauss points of active elements with det J < 0 at the current configuration. Off the hot path.
__global__ void k_negjac(ElemArgs a, unsigned long long* count) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 8 * a.nE) return;
    const long long e = t >> 3;
    const int k = t & 7;
    if (a.flag[e] != 1) return;
    const double g = 1.0 / __builtin_sqrt(3.0);
    const double gz = (k & 4) ? g : -g, et = (k & 2) ? g : -g, tu = (k & 1) ? g : -g;
    double J[3][3] = {{0., 0., 0.}, {0., 0., 0.}, {0., 0., 0.}};
    for (int i = 0; i < 8; ++i) {
        const long long n = a.conn[8 * e + i];
        const double p0 = 0.125 * kSx[i] * (1.0 + et * kSy[i]) * (1.0 + tu * kSz[i]);
        const double p1 = 0.125 * kSy[i] * (1.0 + gz * kSx[i]) * (1.0 + tu * kSz[i]);
        const double p2 = 0.125 * kSz[i] * (1.0 + gz * kSx[i]) * (1.0 + et * kSy[i]);
        for (int c = 0; c < 3; ++c) {
            const double X = a.coord[3 * n + c] + a.u[3 * n + c];
            J[0][c] += p0 * X;
            J[1][c] += p1 * X;
            J[2][c] += p2 * X;
        }
    }
    const double det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) +
                       J[0][1] * (J[1][2] * J[2][0] - J[1][0] * J[2][2]) +
                       J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
    if (det < 0.0) atomicAdd(count, 1ull);
}

hipError_t launch_negjac(const ElemArgs& a, unsigned long long* count, hipStream_t s) {
    if (a.nE <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_negjac, dim3((unsigned)((8 * a.nE + 255) / 256)), dim3(256), 0, s, a, count);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Nodal kernel: one thread per node. Q is assembled by GATHER over the node's incidences in
// ascending element order, which is exactly the order of the reference's serial scatter
// (v2/HAKAI_j.jl:669-675) -- deterministic, no atomics, bit-identical Q.
// The update expression is the reference's (:564) with diag_C = 0 (:217-218), evaluated without
// contraction so it matches the reference bit for bit.
// Fast path: a padded [nN][8] incidence table (16-B vector loads, all 8 gathers in flight; padding
// points at a zero row of fe, and x + 0.0 == x leaves the sum unchanged). Nodes with more than 8
// incidences (unstructured meshes) use the CSR path.
// ---------------------------------------------------------------------------------------------
// The node's own operands are loaded FIRST, so they are in flight together with the incidence
// indices; loaded after the gather they add a third dependent memory round trip (measured with
// tools/nodal_probe.hip: 0.174 -> 0.141 ms on the C3 node count).
// Prescribed value of resolved BC entry i at the step's time (v2/HAKAI_j.jl:585-617): the entry's
// value times its group's piecewise-linear amplitude, first segment extrapolated.
__device__ __forceinline__ double bc_value(const BCArgs& a, int i) {
#pragma clang fp contract(off)
    const int g = a.grp[i];
    const double ct = a.t_rd ? (*a.t_rd + 1.0) * a.dt : a.ct;  // t * d_time, as on the host
    double amp = 1.0;
    const int na = a.amp_n[g];
    if (na > 0) {
        const double* at = a.amp_t + a.amp_off[g];
        const double* av = a.amp_v + a.amp_off[g];
        int ti = 0;
        for (int j = 0; j < na - 1; ++j)
            if (ct >= at[j] && ct <= at[j + 1]) {
                ti = j;
                break;
            }
        amp = av[ti] + (av[ti + 1] - av[ti]) * (ct - at[ti]) / (at[ti + 1] - at[ti]);
    }
    return a.val[i] * amp;
}

struct NodeIn {
    double m, uc[3], up[3], f[3];
};

template <bool FEXT>
__device__ __forceinline__ void nodal_load(const NodalArgs& a, long long n, NodeIn& in) {
    in.m = a.mass[n];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        in.uc[c] = a.u[3 * n + c];
        in.up[c] = a.u_pre_out[3 * n + c];
        in.f[c] = FEXT ? a.fext[3 * n + c] : 0.0;
    }
}

template <bool BCF>
__device__ __forceinline__ void nodal_update(const NodalArgs& a, long long n, const NodeIn& in, double Q0, double Q1,
                                             double Q2) {
#pragma clang fp contract(off)
    const double m = in.m;
    const double dt = a.dt;
    const double dC = 0.0 * m;  // diag_C .= diag_M * C, C = 0
    const double mdt2 = m / (dt * dt);
    const double inv = 1.0 / (mdt2 + dC / 2.0 / dt);
    const double Q[3] = {Q0, Q1, Q2};
    const int b0 = BCF ? a.bc_of_node[n] : -1;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double up = in.up[c];
        double v = inv * (in.f[c] - Q[c] + mdt2 * (2.0 * in.uc[c] - up) + dC / 2.0 / dt * up);
        if (BCF) {  // what k_bc would overwrite afterwards: the node's entries are consecutive
            const long long dc = 3 * n + c;
            for (int j = b0; j >= 0 && j < a.bc.n && a.bc.dof[j] <= dc; ++j)
                if (a.bc.dof[j] == dc) v = bc_value(a.bc, j);
        }
        a.u_pre_out[3 * n + c] = v;
    }
}

// MODE 0: padded [nN][8] table; 1: CSR; 2: Q from an uploaded buffer; 3: owner-computed Q + rows.
// Compile-time modes keep the kernel branch-free: a runtime branch makes the compiler drain all loads
// (vmcnt(0)) at the join, which serialises the node loads with the gather again. Blocks are dealt
// to XCDs round-robin and each XCD walks its contiguous node chunk from the END (xcd_remap_rev):
// the element kernel wrote each XCD's element range in ascending order, so the forces written last
// (still in the Infinity Cache) are gathered first (C3: 0.180 -> 0.164 ms, DESIGN.md §2 k_nodal).
template <int MODE, bool FEXT, bool BCF>
__global__ __launch_bounds__(kBlock) void k_nodal(NodalArgs a) {
#pragma clang fp contract(off)
    if (poisoned(a.poison)) return;
    const unsigned lb = xcd_remap_rev(blockIdx.x, gridDim.x);
    const long long n = (long long)lb * kBlock + threadIdx.x;
    if (n >= a.nN) return;
    NodeIn in;
    nodal_load<FEXT>(a, n, in);  // in flight with the incidence indices
    double Q0 = 0.0, Q1 = 0.0, Q2 = 0.0;
    if (MODE == 2) {
        Q0 = a.qbuf[3 * n + 0];
        Q1 = a.qbuf[3 * n + 1];
        Q2 = a.qbuf[3 * n + 2];
    } else if (MODE == 3) {  // owner-computed assembly: Q (or prefix partial) + later rows, in order
        Q0 = a.own_q[3 * n + 0];
        Q1 = a.own_q[3 * n + 1];
        Q2 = a.own_q[3 * n + 2];
        const int j0 = a.own_rp[n], j1 = a.own_rp[n + 1];
        for (int j = j0; j < j1; ++j) {
            const long long r = a.own_ridx[j];
            Q0 += a.own_rows[3 * r + 0];
            Q1 += a.own_rows[3 * r + 1];
            Q2 += a.own_rows[3 * r + 2];
        }
    } else if (MODE == 0) {
        const int4 lo = reinterpret_cast<const int4*>(a.inc8)[2 * n];
        const int4 hi = reinterpret_cast<const int4*>(a.inc8)[2 * n + 1];
        const int idx[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        double f[8][3];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const double* p = a.fe + idx[j];
            f[j][0] = p[0];
            f[j][1] = p[1];
            f[j][2] = p[2];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            Q0 += f[j][0];
            Q1 += f[j][1];
            Q2 += f[j][2];
        }
    } else {
        const int j0 = a.inc_ptr[n], j1 = a.inc_ptr[n + 1];
        for (int j = j0; j < j1; ++j) {
            const double* f = a.fe + a.inc[j];
            Q0 += f[0];
            Q1 += f[1];
            Q2 += f[2];
        }
    }
    nodal_update<BCF>(a, n, in, Q0, Q1, Q2);
}

template <bool FEXT, bool BCF>
static void launch_nodal_m(const NodalArgs& a, unsigned grid, hipStream_t s) {
    if (a.qbuf)
        hipLaunchKernelGGL((k_nodal<2, FEXT, BCF>), dim3(grid), dim3(kBlock), 0, s, a);
    else if (a.own_q)
        hipLaunchKernelGGL((k_nodal<3, FEXT, BCF>), dim3(grid), dim3(kBlock), 0, s, a);
    else if (a.inc8)
        hipLaunchKernelGGL((k_nodal<0, FEXT, BCF>), dim3(grid), dim3(kBlock), 0, s, a);
    else
        hipLaunchKernelGGL((k_nodal<1, FEXT, BCF>), dim3(grid), dim3(kBlock), 0, s, a);
}

hipError_t launch_nodal(const NodalArgs& a, hipStream_t s) {
    if (a.nN <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((a.nN + kBlock - 1) / kBlock);
    if (a.bc_of_node) {
        if (a.fext)
            launch_nodal_m<true, true>(a, grid, s);
        else
            launch_nodal_m<false, true>(a, grid, s);
    } else {
        if (a.fext)
            launch_nodal_m<true, false>(a, grid, s);
        else
            launch_nodal_m<false, false>(a, grid, s);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Prescribed displacements (v2/HAKAI_j.jl:585-617). Entries are pre-resolved on the host so that
// each dof appears once with its LAST writer's (group, value), which is what the reference's
// in-order overwrite leaves behind.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_bc(BCArgs a) {
    if (poisoned(a.poison)) return;
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.n) return;
    a.out[a.dof[i]] = bc_value(a, i);
}

hipError_t launch_bc(const BCArgs& a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_bc, dim3((a.n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

__global__ void k_set_step(double* slot, double t_prev) {
    if (threadIdx.x == 0) *slot = t_prev;
}

// Timing aid (hakai_step_group with group_serial 2): one wave sleeps a fixed number of s_sleep
// rounds (no memory access, always exits), so the host can enqueue a whole phase behind it and the
// phase then runs back to back instead of at the host's enqueue pace.
__global__ void k_hold(int rounds) {
    for (int i = 0; i < rounds; ++i) __builtin_amdgcn_s_sleep(127);
}

hipError_t launch_hold(int rounds, hipStream_t s) {
    hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, s, rounds);
    return hipGetLastError();
}

hipError_t launch_set_step(double* slot, double t_prev, hipStream_t s) {
    hipLaunchKernelGGL(k_set_step, dim3(1), dim3(64), 0, s, slot, t_prev);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Helpers: Q gather for downloads, layout transposes, state reset, stand-alone triaxiality,
// node averages for output.
// ---------------------------------------------------------------------------------------------
__global__ void k_gather_q(const int* __restrict__ ptr, const int* __restrict__ inc, const double* __restrict__ fe,
                           double* Q, long long nN) {
#pragma clang fp contract(off)
    const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= nN) return;
    double q0 = 0.0, q1 = 0.0, q2 = 0.0;
    for (int j = ptr[n]; j < ptr[n + 1]; ++j) {
        const double* f = fe + inc[j];
        q0 += f[0];
        q1 += f[1];
        q2 += f[2];
    }
    Q[3 * n + 0] = q0;
    Q[3 * n + 1] = q1;
    Q[3 * n + 2] = q2;
}

hipError_t launch_gather_q(const int* inc_ptr, const int* inc, const double* fe, double* Q, long long nN,
                           hipStream_t s) {
    if (nN <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_q, dim3((unsigned)((nN + 255) / 256)), dim3(256), 0, s, inc_ptr, inc, fe, Q, nN);
    return hipGetLastError();
}

// Q of every node from the owner-computed sums (for downloads, and for handing the nodal update
// a Q when owner assembly stops being used): own_q[n] + its exported rows, in element order --
// the same additions as k_nodal MODE 3, so the same bits.
__global__ void k_own_q(const double* __restrict__ own_q, const int* __restrict__ rp, const int* __restrict__ ridx,
                        const double* __restrict__ rows, double* Q, long long nN) {
#pragma clang fp contract(off)
    const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= nN) return;
    double q0 = own_q[3 * n + 0], q1 = own_q[3 * n + 1], q2 = own_q[3 * n + 2];
    for (int j = rp[n]; j < rp[n + 1]; ++j) {
        const long long r = ridx[j];
        q0 += rows[3 * r + 0];
        q1 += rows[3 * r + 1];
        q2 += rows[3 * r + 2];
    }
    Q[3 * n + 0] = q0;
    Q[3 * n + 1] = q1;
    Q[3 * n + 2] = q2;
}

hipError_t launch_own_q(const double* own_q, const int* rp, const int* ridx, const double* rows, double* Q,
                        long long nN, hipStream_t s) {
    if (nN <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_own_q, dim3((unsigned)((nN + 255) / 256)), dim3(256), 0, s, own_q, rp, ridx, rows, Q, nN);
    return hipGetLastError();
}

__global__ void k_aos_to_soa6(const double* __restrict__ aos, double* __restrict__ soa, long long n, long long ld) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 6 * n) return;
    const long long g = i / 6, c = i % 6;
    soa[c * ld + g] = aos[i];
}
__global__ void k_soa_to_aos6(const double* __restrict__ soa, double* __restrict__ aos, long long n, long long ld) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 6 * n) return;
    const long long g = i / 6, c = i % 6;
    aos[i] = soa[c * ld + g];
}

hipError_t launch_aos_to_soa6(const double* aos, double* soa, long long nGP, long long ld, hipStream_t s) {
    if (nGP <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_aos_to_soa6, dim3((unsigned)((6 * nGP + 255) / 256)), dim3(256), 0, s, aos, soa, nGP, ld);
    return hipGetLastError();
}
hipError_t launch_soa_to_aos6(const double* soa, double* aos, long long nGP, long long ld, hipStream_t s) {
    if (nGP <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_soa_to_aos6, dim3((unsigned)((6 * nGP + 255) / 256)), dim3(256), 0, s, soa, aos, nGP, ld);
    return hipGetLastError();
}

__global__ void k_reset_gp(double* stress, double* strain, double* eqps, double* yield, double* triax, int* flag,
                           const int* mat, const DevMat* mats, long long nE, long long nEp, long long ld) {
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= 8 * nEp) return;
    const long long e = g >> 3;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        stress[c * ld + g] = 0.0;
        strain[c * ld + g] = 0.0;
    }
    eqps[g] = 0.0;
    triax[g] = 0.0;
    const DevMat* M = mats + mat[e];
    yield[g] = (e < nE && M->npp > 0) ? M->yield0 : 0.0;
    if ((g & 7) == 0) flag[e] = e < nE ? 1 : 0;  // padding elements behave as deleted
}

hipError_t launch_reset_gp(double* stress, double* strain, double* eqps, double* yield, double* triax, int* flag,
                           const int* mat, const DevMat* mats, long long nE, long long nEp, long long ld, hipStream_t s) {
    if (nEp <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_reset_gp, dim3((unsigned)((8 * nEp + 255) / 256)), dim3(256), 0, s, stress, strain, eqps,
                       yield, triax, flag, mat, mats, nE, nEp, ld);
    return hipGetLastError();
}

__global__ void k_triax_aos(const double* __restrict__ st, double* __restrict__ tx, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* s = st + 6 * i;
    const double mean = (s[0] + s[1] + s[2]) / 3.0;
    const double a01 = s[0] - s[1], a12 = s[1] - s[2], a20 = s[2] - s[0];
    const double oeq = sqrt(0.5 * (a01 * a01 + a12 * a12 + a20 * a20) + 3.0 * (s[3] * s[3] + s[4] * s[4] + s[5] * s[5]));
    tx[i] = (oeq < 1e-10) ? 0.0 : mean / oeq;
}

hipError_t launch_triax_aos(const double* stress_aos, double* triax, long long nGP, hipStream_t s) {
    if (nGP <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_triax_aos, dim3((unsigned)((nGP + 255) / 256)), dim3(256), 0, s, stress_aos, triax, nGP);
    return hipGetLastError();
}

// cal_node_stress_strain (v2/HAKAI_j.jl:3408-3486): element averages (sequential over the 8 GPs),
// summed per node in element order, divided by the incidence count; Mises from the node average.
__global__ void k_node_average(const int* __restrict__ ptr, const int* __restrict__ inc, const double* __restrict__ st,
                               const double* __restrict__ sn, const double* __restrict__ eq,
                               const double* __restrict__ tx, long long ld, long long nN, double* ns, double* nn,
                               double* neq, double* nmis, double* ntx) {
#pragma clang fp contract(off)
    const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= nN) return;
    double as[6] = {0, 0, 0, 0, 0, 0}, an[6] = {0, 0, 0, 0, 0, 0}, ae = 0.0, at = 0.0;
    const int j0 = ptr[n], j1 = ptr[n + 1];
    for (int j = j0; j < j1; ++j) {
        const long long e = inc[j] >> 3;
        for (int c = 0; c < 6; ++c) {
            double s1 = 0.0, s2 = 0.0;
            for (int k = 0; k < 8; ++k) {
                s1 += st[c * ld + 8 * e + k];
                s2 += sn[c * ld + 8 * e + k];
            }
            as[c] += s1 / 8;
            an[c] += s2 / 8;
        }
        double s1 = 0.0, s2 = 0.0;
        for (int k = 0; k < 8; ++k) {
            s1 += eq[8 * e + k];
            s2 += tx[8 * e + k];
        }
        ae += s1 / 8;
        at += s2 / 8;
    }
    const double cnt = (double)(j1 - j0);
    for (int c = 0; c < 6; ++c) {
        as[c] /= cnt;
        an[c] /= cnt;
    }
    ae /= cnt;
    at /= cnt;
    if (ns)
        for (int c = 0; c < 6; ++c) ns[6 * n + c] = as[c];
    if (nn)
        for (int c = 0; c < 6; ++c) nn[6 * n + c] = an[c];
    if (neq) neq[n] = ae;
    if (ntx) ntx[n] = at;
    if (nmis) {
        const double ox = as[0], oy = as[1], oz = as[2], txy = as[3], tyz = as[4], txz = as[5];
        nmis[n] = sqrt(0.5 * ((ox - oy) * (ox - oy) + (oy - oz) * (oy - oz) + (ox - oz) * (ox - oz) +
                              6 * (txy * txy + tyz * tyz + txz * txz)));
    }
}

hipError_t launch_node_average(const int* inc_ptr, const int* inc, const double* stress, const double* strain,
                               const double* eqps, const double* triax, long long ld, long long nN,
                               double* node_stress, double* node_strain, double* node_eqps, double* node_mises,
                               double* node_triax, hipStream_t s) {
    if (nN <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_node_average, dim3((unsigned)((nN + 255) / 256)), dim3(256), 0, s, inc_ptr, inc, stress,
                       strain, eqps, triax, ld, nN, node_stress, node_strain, node_eqps, node_mises, node_triax);
    return hipGetLastError();
}

}  // namespace hk
