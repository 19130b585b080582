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

#include "hakai_kernels.hpp"

namespace hk {

constexpr int kBlock = 256;
constexpr int kEPB = kBlock / 8;     // elements per block
constexpr int kLdsStride = 50;       // doubles per element slot: 8 nodes x (X,du) + pad (bank spread)

// Node sign table delta_mat (v2/HAKAI_j.jl:1900-1907).
__device__ constexpr double kSx[8] = {-1., 1., 1., -1., -1., 1., 1., -1.};
__device__ constexpr double kSy[8] = {-1., -1., 1., 1., -1., -1., 1., 1.};
__device__ constexpr double kSz[8] = {-1., -1., -1., -1., 1., 1., 1., 1.};

// ---------------------------------------------------------------------------------------------
// Element kernel: one 8-lane group per hex8 element, lane k = Gauss point k (gc order of
// v2/HAKAI_j.jl:1913-1920: k bits = (xi, eta, zeta) signs).
//
// Math (identical to the reference's Bfinal algebra, reorganised so no 6x24 matrix is formed):
//   P_k   = J_k^{-1} Pusai_k                    (dN_i/dx at GP k, signed det_k)
//   bbar_i = sum_k det_k P_k[:,i] / (3V),  V = sum_k |det_k|      (= BVbar rows 1-3, :1766-1780)
//   de    = sym(grad du) + (sum_i bbar_i.du_i - div_k(du)/3) (1,1,1,0,0,0)     (= Bfinal*d_u)
//   f_i  += det_k ( sigma P_k[:,i] - P_k[:,i] tr(sigma)/3 ) ;  f_i += (sum_k det_k tr sigma_k) bbar_i
//                                                                            (= sum_k det_k Bfinal' sigma)
// ---------------------------------------------------------------------------------------------
template <bool DO_DELETE, bool STORE_TRIAX>
__global__ __launch_bounds__(kBlock) void k_element(ElemArgs a) {
    __shared__ __attribute__((aligned(16))) double s_nd[kEPB * kLdsStride];
    const int tid = threadIdx.x;
    const int k = tid & 7;
    const int grp = tid >> 3;
    const long long e = (long long)xcd_remap(blockIdx.x, gridDim.x) * kEPB + grp;
    if (e >= a.nE) return;  // whole 8-lane groups leave together
    const int fl = a.flag[e];
    if (fl != 1) {
        if (fl == 2) {  // deleted last step: its Qe becomes 0 from now on (reference skips it, :1116)
            double* f = a.fe + 24 * e + 3 * k;
            f[0] = 0.0;
            f[1] = 0.0;
            f[2] = 0.0;
            a.triax[8 * e + k] = 0.0;  // triaxiality of zero stress (:1012-1014)
            if (k == 0) a.flag[e] = 0;
        }
        return;
    }
    const long long gp = 8 * e + k;
    const long long ld = a.ld;
    const DevMat* M = a.mats + a.mat[e];
    const int npp = M->npp;
    const int nd = DO_DELETE ? M->nd : 0;

    // ---- gather this lane's node: position = coord + u (:650-652), d_disp = u - u_pre (:625)
    const long long n = a.conn[8 * e + k];
    double xo[3], duo[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double uc = a.u[3 * n + c];
        xo[c] = a.coord[3 * n + c] + uc;
        duo[c] = uc - a.u_pre[3 * n + c];
    }
    // ---- Gauss-point state, issued early (coalesced SoA, 512 B per wave per component)
    double sig[6], eps[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) sig[c] = a.stress[c * ld + gp];
#pragma unroll
    for (int c = 0; c < 6; ++c) eps[c] = a.strain[c * ld + gp];
    double eqp = 0.0, ys = 0.0;
    if (npp > 0 || nd > 0) eqp = a.eqps[gp];
    if (npp > 0) ys = a.yield[gp];

    // ---- share the 8 nodes of the element through LDS (this 8-lane group only, same wave:
    // LDS operations of one wave complete in order, so a wavefront-scope fence suffices).
    double* nd8 = s_nd + grp * kLdsStride;
    nd8[6 * k + 0] = xo[0];
    nd8[6 * k + 1] = xo[1];
    nd8[6 * k + 2] = xo[2];
    nd8[6 * k + 3] = duo[0];
    nd8[6 * k + 4] = duo[1];
    nd8[6 * k + 5] = duo[2];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- shape-function derivatives at GP k (cal_Pusai_hexa, v2/HAKAI_j.jl:1924-1934)
    const double g = 1.0 / __builtin_sqrt(3.0);
    const double gz = (k & 4) ? g : -g, et = (k & 2) ? g : -g, tu = (k & 1) ? g : -g;
    const double Ap = 1.0 + gz, Am = 1.0 - gz, Bp = 1.0 + et, Bm = 1.0 - et, Cp = 1.0 + tu, Cm = 1.0 - tu;
    double pxi[8], pet[8], pze[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double A = kSx[i] > 0 ? Ap : Am, B = kSy[i] > 0 ? Bp : Bm, C = kSz[i] > 0 ? Cp : Cm;
        pxi[i] = 1.0 / 8.0 * kSx[i] * B * C;
        pet[i] = 1.0 / 8.0 * kSy[i] * A * C;
        pze[i] = 1.0 / 8.0 * kSz[i] * A * B;
    }
    // ---- Jacobian (:1424-1434), determinant and cofactor inverse (:1436-1455)
    double J[3][3] = {{0., 0., 0.}, {0., 0., 0.}, {0., 0., 0.}};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double X0 = nd8[6 * i + 0], X1 = nd8[6 * i + 1], X2 = nd8[6 * i + 2];
        J[0][0] += pxi[i] * X0; J[0][1] += pxi[i] * X1; J[0][2] += pxi[i] * X2;
        J[1][0] += pet[i] * X0; J[1][1] += pet[i] * X1; J[1][2] += pet[i] * X2;
        J[2][0] += pze[i] * X0; J[2][1] += pze[i] * X1; J[2][2] += pze[i] * X2;
    }
    const double det = J[0][0] * J[1][1] * J[2][2] + J[0][1] * J[1][2] * J[2][0] + J[0][2] * J[1][0] * J[2][1] -
                       J[0][0] * J[1][2] * J[2][1] - J[0][1] * J[1][0] * J[2][2] - J[0][2] * J[1][1] * J[2][0];
    if (det < 0.0 && a.negjac) atomicAdd(a.negjac, 1ull);
    const double rd = 1.0 / det;
    const double i11 = (J[1][1] * J[2][2] - J[1][2] * J[2][1]) * rd;
    const double i21 = (J[1][2] * J[2][0] - J[1][0] * J[2][2]) * rd;
    const double i31 = (J[1][0] * J[2][1] - J[1][1] * J[2][0]) * rd;
    const double i12 = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) * rd;
    const double i22 = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) * rd;
    const double i32 = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) * rd;
    const double i13 = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) * rd;
    const double i23 = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) * rd;
    const double i33 = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) * rd;
    double P[8][3];  // dN_i/dx_c at GP k
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        P[i][0] = i11 * pxi[i] + i12 * pet[i] + i13 * pze[i];
        P[i][1] = i21 * pxi[i] + i22 * pet[i] + i23 * pze[i];
        P[i][2] = i31 * pxi[i] + i32 * pet[i] + i33 * pze[i];
    }

    // ---- volume and B-bar (cal_BVbar_hexa, :1705-1784): V = sum |det|, bbar_k owned by lane k
    const double V = allreduce8(fabs(det));
    double wbar[3];
    {
        double v[8][3];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int c = 0; c < 3; ++c) v[i][c] = det * P[i][c];
        reduce_scatter8(v, wbar, k);
    }
    const double r3V = 1.0 / (3.0 * V);
    const double bb0 = wbar[0] * r3V, bb1 = wbar[1] * r3V, bb2 = wbar[2] * r3V;
    // mean volumetric strain increment / 3 over the element
    const double sdot = allreduce8(bb0 * duo[0] + bb1 * duo[1] + bb2 * duo[2]);

    // ---- strain increment at GP k (= Bfinal * d_u, :1204)
    double Gm[3][3] = {{0., 0., 0.}, {0., 0., 0.}, {0., 0., 0.}};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double d0 = nd8[6 * i + 3], d1 = nd8[6 * i + 4], d2 = nd8[6 * i + 5];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            Gm[0][c] += d0 * P[i][c];
            Gm[1][c] += d1 * P[i][c];
            Gm[2][c] += d2 * P[i][c];
        }
    }
    const double th3 = (Gm[0][0] + Gm[1][1] + Gm[2][2]) / 3.0;
    double de[6];
    de[0] = Gm[0][0] - th3 + sdot;
    de[1] = Gm[1][1] - th3 + sdot;
    de[2] = Gm[2][2] - th3 + sdot;
    de[3] = Gm[0][1] + Gm[1][0];
    de[4] = Gm[1][2] + Gm[2][1];
    de[5] = Gm[0][2] + Gm[2][0];

    // ---- elastic trial (:1205, :1220) and J2 radial return (:1227-1285)
    const double Dn = M->Dn, Do = M->Do, Ds = M->Ds;
    double fin[6];
    fin[0] = sig[0] + (Dn * de[0] + Do * (de[1] + de[2]));
    fin[1] = sig[1] + (Dn * de[1] + Do * (de[0] + de[2]));
    fin[2] = sig[2] + (Dn * de[2] + Do * (de[0] + de[1]));
    fin[3] = sig[3] + Ds * de[3];
    fin[4] = sig[4] + Ds * de[4];
    fin[5] = sig[5] + Ds * de[5];
    if (npp > 0) {
        const double mean = (fin[0] + fin[1] + fin[2]) / 3.0;
        const double d0 = fin[0] - mean, d1 = fin[1] - mean, d2 = fin[2] - mean;
        const double q = sqrt(1.5 * (d0 * d0 + d1 * d1 + d2 * d2 +
                                     2.0 * (fin[3] * fin[3] + fin[4] * fin[4] + fin[5] * fin[5])));
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
            const double sc = (ys + H * dep) / q;
            fin[0] = d0 * sc + mean;
            fin[1] = d1 * sc + mean;
            fin[2] = d2 * sc + mean;
            fin[3] *= sc;
            fin[4] *= sc;
            fin[5] *= sc;
            eqp += dep;
            ys += H * dep;
        }
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) eps[c] += de[c];

    // ---- triaxiality (cal_triax_stress, :995-1018) in invariant form and ductile deletion (:701-758)
    bool kill = false;
    if (DO_DELETE || STORE_TRIAX) {
        const double mean = (fin[0] + fin[1] + fin[2]) / 3.0;
        const double a01 = fin[0] - fin[1], a12 = fin[1] - fin[2], a20 = fin[2] - fin[0];
        const double oeq = sqrt(0.5 * (a01 * a01 + a12 * a12 + a20 * a20) +
                                3.0 * (fin[3] * fin[3] + fin[4] * fin[4] + fin[5] * fin[5]));
        const double tri = (oeq < 1e-10) ? 0.0 : mean / oeq;
        if (STORE_TRIAX) a.triax[gp] = tri;
        if (nd > 0) {
            const double v_e = allreduce8(eqp) / 8.0;
            const double t_e = allreduce8(tri) / 8.0;
            if (!(t_e < 0.0)) {
                double fr = M->du_eps[nd - 1];
                for (int j = 0; j + 1 < nd; ++j) {
                    if (t_e >= M->du_tri[j] && t_e < M->du_tri[j + 1]) {
                        fr = M->du_eps[j] + (M->du_eps[j + 1] - M->du_eps[j]) / (M->du_tri[j + 1] - M->du_tri[j]) *
                                                (t_e - M->du_tri[j]);
                        break;
                    }
                }
                kill = v_e >= fr;
            }
        }
    }

    // ---- internal force (Qe[:,e] += detJ * Bfinal' * sigma, :1330-1340), reduce-scattered so lane k
    // writes the 3 components of local node k.
    const double tr3 = (fin[0] + fin[1] + fin[2]) / 3.0;
    double fk[3];
    {
        double v[8][3];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const double px = P[i][0], py = P[i][1], pz = P[i][2];
            v[i][0] = det * (fin[0] * px + fin[3] * py + fin[5] * pz - px * tr3);
            v[i][1] = det * (fin[3] * px + fin[1] * py + fin[4] * pz - py * tr3);
            v[i][2] = det * (fin[5] * px + fin[4] * py + fin[2] * pz - pz * tr3);
        }
        reduce_scatter8(v, fk, k);
    }
    const double S = allreduce8(det * (3.0 * tr3));
    double* fo = a.fe + 24 * e + 3 * k;
    fo[0] = fk[0] + S * bb0;
    fo[1] = fk[1] + S * bb1;
    fo[2] = fk[2] + S * bb2;
    if (a.vol && k == 0) a.vol[e] = V;

    // ---- state write-back (:1281-1282, :1304-1323); deletion zeroes stress/strain (:742-756)
    if (kill) {
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            fin[c] = 0.0;
            eps[c] = 0.0;
        }
        if (k == 0) {
            a.flag[e] = 2;
            const int slot = atomicAdd(a.del_count, 1);
            if (slot < a.del_cap) {
                a.del_log[2 * slot + 0] = (long long)a.t_step;
                a.del_log[2 * slot + 1] = e + 1;
            }
        }
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) a.stress[c * ld + gp] = fin[c];
#pragma unroll
    for (int c = 0; c < 6; ++c) a.strain[c * ld + gp] = eps[c];
    if (npp > 0) {
        a.eqps[gp] = eqp;
        a.yield[gp] = ys;
    }
}

hipError_t launch_element(const ElemArgs& a, bool do_delete, bool store_triax, hipStream_t s) {
    if (a.nE <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((a.nE + kEPB - 1) / kEPB);
    if (do_delete) {
        if (store_triax)
            hipLaunchKernelGGL((k_element<true, true>), dim3(grid), dim3(kBlock), 0, s, a);
        else
            hipLaunchKernelGGL((k_element<true, false>), dim3(grid), dim3(kBlock), 0, s, a);
    } else {
        if (store_triax)
            hipLaunchKernelGGL((k_element<false, true>), dim3(grid), dim3(kBlock), 0, s, a);
        else
            hipLaunchKernelGGL((k_element<false, false>), dim3(grid), dim3(kBlock), 0, s, a);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Nodal kernel: one thread per node. Q is assembled by GATHER over the node's incidences in
// ascending element order, which is exactly the order of the reference's serial scatter
// (v2/HAKAI_j.jl:669-675) -- deterministic, no atomics, bit-identical Q.
// The update expression is the reference's (:564) with diag_C = 0 (:217-218), evaluated without
// contraction so it matches the reference bit for bit.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_nodal(NodalArgs a) {
#pragma clang fp contract(off)
    const long long n = (long long)xcd_remap(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
    if (n >= a.nN) return;
    double Q0 = 0.0, Q1 = 0.0, Q2 = 0.0;
    if (a.qbuf) {
        Q0 = a.qbuf[3 * n + 0];
        Q1 = a.qbuf[3 * n + 1];
        Q2 = a.qbuf[3 * n + 2];
    } else {
        const int j0 = a.inc_ptr[n], j1 = a.inc_ptr[n + 1];
        for (int j = j0; j < j1; ++j) {
            const double* f = a.fe + 3 * (long long)a.inc[j];
            Q0 += f[0];
            Q1 += f[1];
            Q2 += f[2];
        }
    }
    const double m = a.mass[n];
    const double dt = a.dt;
    const double dC = 0.0 * m;  // diag_C .= diag_M * C, C = 0
    const double mdt2 = m / (dt * dt);
    const double inv = 1.0 / (mdt2 + dC / 2.0 / dt);
    const double Q[3] = {Q0, Q1, Q2};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double f = a.fext ? a.fext[3 * n + c] : 0.0;
        const double uc = a.u[3 * n + c];
        const double up = a.u_pre_out[3 * n + c];
        a.u_pre_out[3 * n + c] = inv * (f - Q[c] + mdt2 * (2.0 * uc - up) + dC / 2.0 / dt * up);
    }
}

hipError_t launch_nodal(const NodalArgs& a, hipStream_t s) {
    if (a.nN <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((a.nN + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_nodal, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Prescribed displacements (v2/HAKAI_j.jl:585-617). Entries are pre-resolved on the host so that
// each dof appears once with its LAST writer's (group, value), which is what the reference's
// in-order overwrite leaves behind.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_bc(BCArgs a) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.n) return;
    const int g = a.grp[i];
    double amp = 1.0;
    const int na = a.amp_n[g];
    if (na > 0) {
        const double* at = a.amp_t + a.amp_off[g];
        const double* av = a.amp_v + a.amp_off[g];
        int ti = 0;
        for (int j = 0; j < na - 1; ++j)
            if (a.ct >= at[j] && a.ct <= at[j + 1]) {
                ti = j;
                break;
            }
        amp = av[ti] + (av[ti + 1] - av[ti]) * (a.ct - at[ti]) / (at[ti + 1] - at[ti]);
    }
    a.out[a.dof[i]] = a.val[i] * amp;
}

hipError_t launch_bc(const BCArgs& a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_bc, dim3((a.n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, a);
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
        const double* f = fe + 3 * (long long)inc[j];
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
                           const int* mat, const DevMat* mats, long long nE, long long ld) {
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= 8 * nE) return;
    const long long e = g >> 3;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        stress[c * ld + g] = 0.0;
        strain[c * ld + g] = 0.0;
    }
    eqps[g] = 0.0;
    triax[g] = 0.0;
    const DevMat* M = mats + mat[e];
    yield[g] = (M->npp > 0) ? M->yield0 : 0.0;
    if ((g & 7) == 0) flag[e] = 1;
}

hipError_t launch_reset_gp(double* stress, double* strain, double* eqps, double* yield, double* triax, int* flag,
                           const int* mat, const DevMat* mats, long long nE, long long ld, hipStream_t s) {
    if (nE <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_reset_gp, dim3((unsigned)((8 * nE + 255) / 256)), dim3(256), 0, s, stress, strain, eqps,
                       yield, triax, flag, mat, mats, nE, ld);
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
