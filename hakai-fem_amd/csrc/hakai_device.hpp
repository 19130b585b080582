// hakai_device.hpp -- device-side types and wave-level primitives for the gfx950 (CDNA4) kernels.
//
// Layout decisions (DESIGN.md "Data layout in HBM"):
//   * Gauss-point state is SoA: component c of GP g lives at base[c * ld + g], g = 8e + k, so the
//     8 lanes of an element and the 8 elements of a wave read 64 consecutive doubles (512 B)
//     per load instruction.
//   * One element = 8 consecutive lanes; lane k owns Gauss point k AND, after the reduce-scatter,
//     local node k. Cross-lane traffic never leaves the 8-lane group, so it is done with DPP
//     (quad_perm / row_half_mirror) and needs no LDS round trip and no barrier.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hk {

constexpr int kMaxPlastic = 64;
constexpr int kMaxDuctile = 32;
constexpr int kMaxLdsMats = 8;   // materials staged in LDS by the pipelined element kernel

// Per-material constants, derived on the host exactly like hakai() does (v2/HAKAI_j.jl:143-172)
// and readInpFile builds Hd (v2/readInpFile_j.jl:763-768).
struct DevMat {
    double Dn, Do, Ds;   // Dmat[1,1], Dmat[1,2], Dmat[4,4] of the isotropic 6x6
    double G;
    double density;
    double yield0;       // plastic[1,1] -> initial yield (v2/HAKAI_j.jl:456-465)
    int npp;             // plastic rows (0 = elastic)
    int nd;              // ductile rows (0 = no deletion)
    double pl_eps[kMaxPlastic];   // plastic[:,2]
    double Hd[kMaxPlastic];       // hardening slope of segment j
    double du_eps[kMaxDuctile];   // ductile[:,1] fracture strain
    double du_tri[kMaxDuctile];   // ductile[:,2] triaxiality
    double du_floor;              // below every fracture strain ductile_fr can return (skips the table)
    double du_skip;               // a wave whose Gauss points all lie below this skips the deletion test
};

// DPP control words (gfx9 encoding).
constexpr int kDppXor1 = 0xB1;     // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;     // quad_perm [2,3,0,1]
constexpr int kDppHalfMir = 0x141; // row_half_mirror: lane i <- lane 7-i inside each 8-lane half-row

template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
    const unsigned long long v = (unsigned long long)__double_as_longlong(x);
    int lo = (int)(unsigned)v;
    int hi = (int)(unsigned)(v >> 32);
    lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xF, 0xF, false);
    hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// Sum over the 8 lanes of an element; every lane gets the bit-identical total (each step adds a
// pair in both orders, and fp addition is commutative).
__device__ __forceinline__ double allreduce8(double x) {
    x += dpp<kDppXor1>(x);
    x += dpp<kDppXor2>(x);
    x += dpp<kDppHalfMir>(x);
    return x;
}

// Reduce-scatter in RELATIVE slots: lane k holds v[j] for node s = j ^ k (s a node label in
// 0..7), and partners are k^7 (half mirror), k^2, k^1. The partner's slot for the same node is
// j ^ (partner mask), so every lane keeps slots with the mask bit clear and reads the partner's
// slot j ^ mask: no per-lane selects. Lane k returns the sum over lanes for node s = k.
// 21 double exchanges + 21 adds.
__device__ __forceinline__ void reduce_scatter8_rel(const double (&v)[8][3], double (&out)[3]) {
    double w[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int c = 0; c < 3; ++c) w[j][c] = v[j][c] + dpp<kDppHalfMir>(v[j ^ 7][c]);
    double u[2][3];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int c = 0; c < 3; ++c) u[j][c] = w[j][c] + dpp<kDppXor2>(w[j ^ 2][c]);
#pragma unroll
    for (int c = 0; c < 3; ++c) out[c] = u[0][c] + dpp<kDppXor1>(u[1][c]);
}

// Reduce-scatter of a per-lane [8 nodes][3] array over the 8 lanes: lane k returns the sum over
// lanes of v[k][0..2]. 21 double exchanges instead of 72 for an all-reduce.
__device__ __forceinline__ void reduce_scatter8(const double (&v)[8][3], double (&out)[3], int k) {
    const bool b2 = (k & 4) != 0, b1 = (k & 2) != 0, b0 = (k & 1) != 0;
    double w[4][3];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double lo = v[s][c], hi = v[4 + s][c];
            const double keep = b2 ? hi : lo, send = b2 ? lo : hi;
            w[s][c] = keep + dpp<kDppHalfMir>(send);
        }
    double u[2][3];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double lo = w[s][c], hi = w[2 + s][c];
            const double keep = b1 ? hi : lo, send = b1 ? lo : hi;
            u[s][c] = keep + dpp<kDppXor2>(send);
        }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double lo = u[0][c], hi = u[1][c];
        const double keep = b0 ? hi : lo, send = b0 ? lo : hi;
        out[c] = keep + dpp<kDppXor1>(send);
    }
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks dealt round-robin over the 8 XCDs get contiguous logical ranges per XCD, so the nodes
// shared by neighbouring elements are re-read from the same L2.
__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned nwg) {
    if (nwg < 16) return b;
    const unsigned xcd = b & 7u, q = nwg >> 3, r = nwg & 7u;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// The same chunks, each walked from its END: a kernel that reads what the previous kernel wrote
// chunk-wise in ascending order meets the most recently written lines (still in the Infinity
// Cache) first, instead of evicting them before it gets there.
__device__ __forceinline__ unsigned xcd_remap_rev(unsigned b, unsigned nwg) {
    if (nwg < 16) return nwg - 1 - b;
    const unsigned xcd = b & 7u, q = nwg >> 3, r = nwg & 7u;
    const unsigned len = xcd < r ? q + 1 : q;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (len - 1 - (b >> 3));
}

}  // namespace hk
