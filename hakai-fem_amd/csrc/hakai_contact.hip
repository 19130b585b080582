// hakai_contact.hip -- all-exterior instance-vs-instance contact on gfx950.
//
// Reference: v2/HAKAI_j.jl (v2 = HAKAI-v0.0.2/Julia)
//   setup            :244-421   pairs (instance_pair, cp_index), CT lists, element sizes
//   get_element_face :1944-1992, get_surface_triangle :1996-2164, add_surface_triangle :2167-2245
//   surface update   :766-804   (after element deletion)
//   cal_contact_force:2248-2706 (CPU path; the CUDA.jl path :2899-3157 deliberately differs, §9 Q14)
//   accumulation     :435, :511-538  (Float128 per thread, rounded once into external_force)
//
// Design (MI355X-first, same results):
//   * The contact lists the reference grows at run time (appending newly exposed faces when an
//     element is deleted) are enumerated ONCE on the host: every triangle / contact node that can
//     ever appear carries the elements whose deletion adds it. On the device an entry is live at
//     step t iff it was in the initial list or one of its adders was deleted before t (del_step).
//     Same sets as the reference at every step, no host round trip, no reallocation.
//   * The reference's candidate filter |cell(j0) - cell(i)| <= 1 per axis (cells of size
//     1.1*elementMaxSize, 0.6 for self-contact) becomes a hash grid over the i-nodes: a triangle
//     visits the distinct buckets of the 27 neighbouring cells and applies the exact same integer
//     test, so the candidate set is identical and the work is O(contact nodes), not O(T x N).
//   * Every contact event computes the reference's FP64 expressions verbatim (no contraction).
//     Forces are gathered per node and summed in double-double, then rounded once: the reference
//     sums in Float128 and rounds once, so both are the correctly rounded sum up to a 2^-106
//     relative window (order-independent, no atomics on doubles).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "hakai_internal.hpp"

using hkc::fail;
using hkc::hip_fail;

#define HIPCHK(x)                                      \
    do {                                               \
        hipError_t _e = (x);                           \
        if (_e != hipSuccess) return hip_fail(_e, #x); \
    } while (0)

namespace hkc {

struct PairParam {
    double young, kc, Cr, ddiv;
    int self;
    int hash_off, hash_size;
    int pad;
};

struct Contact {
    int npairs = 0;
    std::vector<PairParam> h_par;
    PairParam* d_par = nullptr;
    // i-side (contact points) and j-side (triangle nodes) node entries, all pairs concatenated
    int n_ni = 0, n_nj = 0;
    int *d_ni_pair = nullptr, *d_ni_node = nullptr, *d_ni_orig = nullptr, *d_ni_aptr = nullptr, *d_ni_add = nullptr;
    int *d_nj_pair = nullptr, *d_nj_node = nullptr, *d_nj_orig = nullptr, *d_nj_aptr = nullptr, *d_nj_add = nullptr;
    int nseg = 0;
    int* d_seg = nullptr;  // [nseg][4] (start, end, pair, side) node-entry segments
    // triangles
    int n_tri = 0;
    int *d_tri_pair = nullptr, *d_tri_nodes = nullptr, *d_tri_ele = nullptr, *d_tri_adder = nullptr;
    // hash grid over i-nodes
    int htot = 0;
    int *d_bcnt = nullptr, *d_boff = nullptr, *d_blist = nullptr, *d_ni_bucket = nullptr;
    long long* d_ni_map = nullptr;
    unsigned long long* d_bbox = nullptr;  // [npairs][12] ordered-integer encoded doubles
    // events and per-node gather
    long long cap = 0;
    unsigned int* d_evn = nullptr;  // [0] events this step, [1] max seen (overflow check)
    int* d_ev_nodes = nullptr;      // [cap][4]
    double* d_ev_f = nullptr;       // [cap][3]
    int *d_cnt = nullptr, *d_off = nullptr;
    double* d_terms = nullptr;      // [4 cap][3]
    void* d_tmp = nullptr;
    size_t tmp_bytes = 0;
    // velocity before the first step (initial condition / uploaded), v2/HAKAI_j.jl:233-239
    double* d_velo0 = nullptr;
    bool use_velo0 = true;
    double min_size = 0, max_size = 0, d_lim = 0;
    double myu = 0.25, kc_o = 1.0, kc_s = 1.0, Cr_o = 0.0, Cr_s = 0.0;  // :2255-2259
    std::vector<int> pair_inst;  // [npairs][2] (1-based instances), for hakai_contact_info
    std::vector<long long> pair_counts;  // [npairs][3] initial #nodes_i, #triangles, #nodes_j
};

}  // namespace hkc

namespace {

using hkc::Contact;
using hkc::PairParam;

constexpr int kB = 256;

__device__ __forceinline__ unsigned long long enc(double d) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
__device__ __forceinline__ double dec(unsigned long long e) {
    const unsigned long long u = (e >> 63) ? (e & 0x7FFFFFFFFFFFFFFFULL) : ~e;
    return __longlong_as_double((long long)u);
}

__device__ __forceinline__ bool live(int orig, const int* aptr, const int* add, int k, const int* del_step, int t) {
    if (orig) return true;
    for (int a = aptr[k]; a < aptr[k + 1]; ++a) {
        const int s = del_step[add[a]];  // -1: deleted before an upload_state
        if (s != 0 && s < t) return true;
    }
    return false;
}

__device__ __forceinline__ double my3norm(double a, double b, double c) {
#pragma clang fp contract(off)
    return sqrt(a * a + b * b + c * c);
}

__device__ __forceinline__ unsigned hash3(long long x, long long y, long long z) {
    const unsigned long long h = (unsigned long long)x * 0x9E3779B97F4A7C15ULL ^
                                 (unsigned long long)y * 0xC2B2AE3D27D4EB4FULL ^
                                 (unsigned long long)z * 0x165667B19E3779F9ULL;
    return (unsigned)(h ^ (h >> 29));
}

struct Range {
    double mn[3], mx[3], amn[3];
    bool empty;
};

__device__ __forceinline__ Range pair_range(const unsigned long long* bb) {
    Range r;
    r.empty = false;
    for (int d = 0; d < 3; ++d) {
        if (bb[d] == ~0ULL || bb[6 + d] == ~0ULL) {  // a side without live nodes
            r.empty = true;
            r.mn[d] = r.mx[d] = r.amn[d] = 0.0;
            continue;
        }
        const double mni = dec(bb[d]), mxi = dec(bb[3 + d]), mnj = dec(bb[6 + d]), mxj = dec(bb[9 + d]);
        r.mn[d] = fmax(mni, mnj);
        r.mx[d] = fmin(mxi, mxj);
        r.amn[d] = fmin(mni, mnj);
    }
    if (!r.empty && (r.mn[0] > r.mx[0] || r.mn[1] > r.mx[1] || r.mn[2] > r.mx[2])) r.empty = true;  // :2304-2306
    return r;
}

__global__ void k_ct_reset(unsigned long long* bbox, int npairs, unsigned int* evn) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 12 * npairs) bbox[i] = ((i % 12) / 3) % 2 == 0 ? ~0ULL : 0ULL;  // min slots +inf, max slots -inf
    if (i == 0) evn[0] = 0;
}

struct StepIn {
    const double* coord;
    const double* u;       // disp at the start of the step
    const double* u_pre;   // disp_pre
    const double* velo0;   // non-null before the first step
    double d_time;
    const int* del_step;
    const int* flag;
    const int* conn;
    const double* mass;
    int t;
};

__device__ __forceinline__ void pos(const StepIn& s, int n, double p[3]) {
#pragma clang fp contract(off)
    for (int c = 0; c < 3; ++c) p[c] = s.coord[3 * n + c] + s.u[3 * n + c];  // position, :653-655
}

// live flags + bounding boxes of the live node lists per pair (:2281-2299)
// Segment = the node entries of one pair side (entries are stored pair by pair). kSegBlocks blocks
// per segment reduce in registers, then across the block (DPP-free shuffles + LDS), then issue ONE
// atomic per bound: per-entry atomics on 12 shared addresses serialised the whole step.
constexpr int kSegBlocks = 64;

struct Seg {
    int start, end, pair, side;  // side 0: i-nodes, 1: j-nodes
};

__device__ __forceinline__ unsigned long long umin64(unsigned long long a, unsigned long long b) { return a < b ? a : b; }
__device__ __forceinline__ unsigned long long umax64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }

__global__ __launch_bounds__(kB) void k_ct_bbox(StepIn s, const Seg* segs, const int* ni_node, const int* ni_orig,
                                                const int* ni_aptr, const int* ni_add, const int* nj_node,
                                                const int* nj_orig, const int* nj_aptr, const int* nj_add,
                                                unsigned long long* bbox, int* ni_bucket) {
    const Seg sg = segs[blockIdx.x / kSegBlocks];
    const int sub = blockIdx.x % kSegBlocks;
    const bool side_i = sg.side == 0;
    const int* node = side_i ? ni_node : nj_node;
    const int* orig = side_i ? ni_orig : nj_orig;
    const int* aptr = side_i ? ni_aptr : nj_aptr;
    const int* add = side_i ? ni_add : nj_add;
    unsigned long long mn[3] = {~0ULL, ~0ULL, ~0ULL}, mx[3] = {0ULL, 0ULL, 0ULL};
    for (int k = sg.start + sub * kB + (int)threadIdx.x; k < sg.end; k += kSegBlocks * kB) {
        const bool on = live(orig[k], aptr, add, k, s.del_step, s.t);
        if (side_i) ni_bucket[k] = on ? 0 : -1;
        if (!on) continue;
        double p[3];
        pos(s, node[k], p);
        for (int d = 0; d < 3; ++d) {
            const unsigned long long e = enc(p[d]);
            mn[d] = umin64(mn[d], e);
            mx[d] = umax64(mx[d], e);
        }
    }
    for (int off = 32; off > 0; off >>= 1)
        for (int d = 0; d < 3; ++d) {
            mn[d] = umin64(mn[d], __shfl_xor(mn[d], off));
            mx[d] = umax64(mx[d], __shfl_xor(mx[d], off));
        }
    __shared__ unsigned long long red[kB / 64][6];
    const int w = threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0)
        for (int d = 0; d < 3; ++d) {
            red[w][d] = mn[d];
            red[w][3 + d] = mx[d];
        }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int q = threadIdx.x;
        unsigned long long v = red[0][q];
        for (int ww = 1; ww < kB / 64; ++ww) v = q < 3 ? umin64(v, red[ww][q]) : umax64(v, red[ww][q]);
        unsigned long long* bb = bbox + 12 * sg.pair + (side_i ? 0 : 6);
        if (q < 3) {
            if (v != ~0ULL) atomicMin(&bb[q], v);
        } else if (v != 0ULL) {
            atomicMax(&bb[q], v);
        }
    }
}

// cells of the live i-nodes inside the pair's range box (:2333-2346) -> hash bucket counts
__global__ void k_ct_bin(StepIn s, int n_ni, const int* ni_pair, const int* ni_node, const PairParam* par,
                         const unsigned long long* bbox, int* ni_bucket, long long* ni_map, int* bcnt) {
#pragma clang fp contract(off)
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_ni || ni_bucket[k] < 0) return;
    const int pr = ni_pair[k];
    const Range r = pair_range(bbox + 12 * pr);
    double p[3];
    pos(s, ni_node[k], p);
    if (r.empty || p[0] < r.mn[0] || p[1] < r.mn[1] || p[2] < r.mn[2] || p[0] > r.mx[0] || p[1] > r.mx[1] ||
        p[2] > r.mx[2]) {  // the candidate test of :2514-2519, applied before binning
        ni_bucket[k] = -1;
        return;
    }
    const PairParam pp = par[pr];
    long long m[3];
    for (int d = 0; d < 3; ++d) {
        m[d] = (long long)ceil((p[d] - r.amn[d]) / pp.ddiv);
        ni_map[3 * (long long)k + d] = m[d];
    }
    const int b = pp.hash_off + (int)(hash3(m[0], m[1], m[2]) & (unsigned)(pp.hash_size - 1));
    ni_bucket[k] = b;
    atomicAdd(&bcnt[b], 1);
}

__global__ void k_ct_fill(int n_ni, const int* ni_bucket, const int* boff, int* bcnt, int* blist) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_ni) return;
    const int b = ni_bucket[k];
    if (b < 0) return;
    const int slot = boff[b] + atomicSub(&bcnt[b], 1) - 1;  // leaves bcnt zeroed for the next step
    blist[slot] = k;
}

// one thread per triangle: the body of the @floop at :2371-2698
__global__ void k_ct_tri(StepIn s, int n_tri, const int* tri_pair, const int* tri_nodes, const int* tri_ele,
                         const int* tri_adder, const PairParam* par, const unsigned long long* bbox, const int* boff,
                         const int* blist, const int* ni_node, const long long* ni_map, double d_lim, double myu,
                         unsigned int* evn, long long cap, int* ev_nodes, double* ev_f) {
#pragma clang fp contract(off)
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_tri) return;
    const int eleid = tri_ele[j];
    if (s.flag[eleid] != 1) return;  // :2374-2377
    const int ad = tri_adder[j];
    if (ad >= 0) {
        const int st = s.del_step[ad];
        if (!(st != 0 && st < s.t)) return;  // face not exposed yet
    }
    const int pr = tri_pair[j];
    const Range r = pair_range(bbox + 12 * pr);
    if (r.empty) return;
    const PairParam pp = par[pr];
    const int j0 = tri_nodes[3 * j], j1 = tri_nodes[3 * j + 1], j2 = tri_nodes[3 * j + 2];
    double q0[3], q1[3], q2[3];
    pos(s, j0, q0);
    pos(s, j1, q1);
    pos(s, j2, q2);
    for (int d = 0; d < 3; ++d) {  // :2394-2411
        if (q0[d] < r.mn[d] && q1[d] < r.mn[d] && q2[d] < r.mn[d]) return;
        if (q0[d] > r.mx[d] && q1[d] > r.mx[d] && q2[d] > r.mx[d]) return;
    }
    const double cx = (q0[0] + q1[0] + q2[0]) / 3.0, cy = (q0[1] + q1[1] + q2[1]) / 3.0,
                 cz = (q0[2] + q1[2] + q2[2]) / 3.0;
    const double R0 = my3norm(q0[0] - cx, q0[1] - cy, q0[2] - cz);
    const double R1 = my3norm(q1[0] - cx, q1[1] - cy, q1[2] - cz);
    const double R2 = my3norm(q2[0] - cx, q2[1] - cy, q2[2] - cz);
    const double Rmax = fmax(fmax(R0, R1), R2);
    const double v1x = q1[0] - q0[0], v1y = q1[1] - q0[1], v1z = q1[2] - q0[2];
    const double v2x = q2[0] - q0[0], v2y = q2[1] - q0[1], v2z = q2[2] - q0[2];
    const double L1 = my3norm(v1x, v1y, v1z), L2 = my3norm(v2x, v2y, v2z);
    const double Lmax = fmax(L1, L2);
    double nx = v1y * v2z - v1z * v2y, ny = v1z * v2x - v1x * v2z, nz = v1x * v2y - v1y * v2x;  // my3crossNNz
    const double mag_n = sqrt(nx * nx + ny * ny + nz * nz);
    nx = nx / mag_n;
    ny = ny / mag_n;
    nz = nz / mag_n;
    const double d12 = v1x * v2x + v1y * v2y + v1z * v2z;
    const double S = 0.5 * sqrt(L1 * L1 * L2 * L2 - d12 * d12);
    const double A11 = v1x, A21 = v1y, A31 = v1z, A12 = v2x, A22 = v2y, A32 = v2z, A13 = -nx, A23 = -ny, A33 = -nz;
    // my3SolveAb (:3342-3373): determinant and adjugate do not depend on the point
    const double vdet = (A11 * A22 * A33 + A12 * A23 * A31 + A13 * A21 * A32 - A11 * A23 * A32 - A12 * A21 * A33 -
                         A13 * A22 * A31);
    const double im11 = A22 * A33 - A23 * A32, im21 = A23 * A31 - A21 * A33, im31 = A21 * A32 - A22 * A31;
    const double im12 = A13 * A32 - A12 * A33, im22 = A11 * A33 - A13 * A31, im32 = A12 * A31 - A11 * A32;
    const double im13 = A12 * A23 - A13 * A22, im23 = A13 * A21 - A11 * A23, im33 = A11 * A22 - A12 * A21;
    const double kk = pp.young * S / Lmax * pp.kc;  // :2575
    long long mj[3];
    for (int d = 0; d < 3; ++d) mj[d] = (long long)ceil((q0[d] - r.amn[d]) / pp.ddiv);
    int el[8];
    if (pp.self)
        for (int a = 0; a < 8; ++a) el[a] = s.conn[8 * (long long)eleid + a];
    int seen[27];
    int ns = 0;
    for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                const int b =
                    pp.hash_off + (int)(hash3(mj[0] + dx, mj[1] + dy, mj[2] + dz) & (unsigned)(pp.hash_size - 1));
                bool dup = false;
                for (int q = 0; q < ns; ++q) dup |= (seen[q] == b);
                if (dup) continue;
                seen[ns++] = b;
                for (int sl = boff[b]; sl < boff[b + 1]; ++sl) {
                    const int k = blist[sl];
                    const long long* mk = ni_map + 3 * (long long)k;
                    if (llabs(mj[0] - mk[0]) > 1 || llabs(mj[1] - mk[1]) > 1 || llabs(mj[2] - mk[2]) > 1) continue;
                    const int i = ni_node[k];
                    if (pp.self) {
                        bool own = false;
                        for (int a = 0; a < 8; ++a) own |= (i == el[a]);
                        if (own) continue;
                    }
                    double p[3];
                    pos(s, i, p);
                    const double dpc = my3norm(p[0] - cx, p[1] - cy, p[2] - cz);
                    if (dpc >= Rmax) continue;
                    const double bx = p[0] - q0[0], by = p[1] - q0[1], bz = p[2] - q0[2];
                    const double x1 = (im11 * bx + im12 * by + im13 * bz) / vdet;
                    const double x2 = (im21 * bx + im22 * by + im23 * bz) / vdet;
                    const double d = (im31 * bx + im32 * by + im33 * bz) / vdet;
                    if (!(0.0 <= x1 && 0.0 <= x2 && x1 + x2 <= 1.0 && d > 0.0 && d <= d_lim)) continue;
                    // velo = d_disp / d_time of the previous step (:628); the IC before step 1
                    double vi[3], vj[3];
                    for (int c = 0; c < 3; ++c) {
                        if (s.velo0) {
                            vi[c] = s.velo0[3 * i + c];
                            vj[c] = s.velo0[3 * j0 + c];
                        } else {
                            vi[c] = (s.u[3 * i + c] - s.u_pre[3 * i + c]) / s.d_time;
                            vj[c] = (s.u[3 * j0 + c] - s.u_pre[3 * j0 + c]) / s.d_time;
                        }
                    }
                    const double vx = vi[0] - vj[0], vy = vi[1] - vj[1], vz = vi[2] - vj[2];
                    const double mag_v = my3norm(vx, vy, vz);
                    double vex = 0.0, vey = 0.0, vez = 0.0;
                    if (mag_v > 0.0) {
                        vex = vx / mag_v;
                        vey = vy / mag_v;
                        vez = vz / mag_v;
                    }
                    const double F = kk * d;
                    double fx = F * nx, fy = F * ny, fz = F * nz;
                    // damping: diag_M[i] indexes the dof vector with a node id (:2592)
                    const double Cd = 2 * sqrt(s.mass[(i) / 3] * kk) * pp.Cr;
                    const double fc_x = -Cd * vx, fc_y = -Cd * vy, fc_z = -Cd * vz;
                    const double dot_ve_n = vex * nx + vey * ny + vez * nz;
                    const double vsx = vex - dot_ve_n * nx, vsy = vey - dot_ve_n * ny, vsz = vez - dot_ve_n * nz;
                    const double fric_x = -myu * F * vsx, fric_y = -myu * F * vsy, fric_z = -myu * F * vsz;
                    fx += fric_x + fc_x;
                    fy += fric_y + fc_y;
                    fz += fric_z + fc_z;
                    const unsigned e = atomicAdd(&evn[0], 1u);
                    if ((long long)e < cap) {
                        int* en = ev_nodes + 4 * (long long)e;
                        en[0] = i;
                        en[1] = j0;
                        en[2] = j1;
                        en[3] = j2;
                        double* ef = ev_f + 3 * (long long)e;
                        ef[0] = fx;
                        ef[1] = fy;
                        ef[2] = fz;
                    }
                }
            }
}

__global__ void k_ct_count(const unsigned int* evn, long long cap, const int* ev_nodes, int* cnt, unsigned int* evmax) {
    const long long n = std::min<long long>((long long)evn[0], cap);
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicMax(evmax, evn[0]);
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < 4 * n;
         e += (long long)gridDim.x * blockDim.x)
        atomicAdd(&cnt[ev_nodes[e]], 1);
}

__global__ void k_ct_scatter(const unsigned int* evn, long long cap, const int* ev_nodes, const double* ev_f,
                             const int* off, int* cnt, double* terms) {
#pragma clang fp contract(off)
    const long long n = std::min<long long>((long long)evn[0], cap);
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < 4 * n;
         e += (long long)gridDim.x * blockDim.x) {
        const int node = ev_nodes[e];
        const long long ev = e >> 2;
        const int role = (int)(e & 3);
        const int slot = off[node] + atomicSub(&cnt[node], 1) - 1;  // leaves cnt zeroed
        const double* f = ev_f + 3 * ev;
        double* o = terms + 3 * (long long)slot;
        if (role == 0) {  // c_force3[i] += f
            o[0] = f[0];
            o[1] = f[1];
            o[2] = f[2];
        } else {  // triangle nodes: += -f / 3.0
            o[0] = -f[0] / 3.0;
            o[1] = -f[1] / 3.0;
            o[2] = -f[2] / 3.0;
        }
    }
}

// external_force = 0.0 + (sum of the node's terms), summed in double-double and rounded once
__global__ void k_ct_sum(long long nN, const int* off, const double* terms, double* fext) {
#pragma clang fp contract(off)
    const long long n = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (n >= nN) return;
    const int a = off[n], b = off[n + 1];
    for (int c = 0; c < 3; ++c) {
        double s = 0.0, e = 0.0;
        for (int q = a; q < b; ++q) {
            const double x = terms[3 * (long long)q + c];
            const double t = s + x;  // TwoSum
            const double bp = t - s;
            const double err = (s - (t - bp)) + (x - bp);
            s = t;
            e += err;
        }
        fext[3 * n + c] = s + e;
    }
}

template <class T>
hipError_t dalloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    return hipMalloc((void**)p, n * sizeof(T));
}
template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}
template <class T>
hipError_t upload(T** p, const std::vector<T>& v, hipStream_t s) {
    hipError_t e = dalloc(p, v.size());
    if (e != hipSuccess || v.empty()) return e;
    return hipMemcpyAsync(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
}

// ---- host: surface extraction with the reference's semantics ------------------------------
struct Face {
    int n[4];    // oriented (global 0-based nodes)
    int key[4];  // sorted
    int ele;     // global 0-based element
};

struct Inst {
    int e0 = -1, nE = 0;
    std::vector<Face> faces;       // 6 per element, in the reference's order
    std::vector<int> order;        // face indices sorted by (key, index)
    std::vector<int> exterior;     // exterior face indices, ascending
    std::vector<std::vector<int>> added;  // per local element: faces exposed by its deletion
    double young = 0;
};

bool key_less(const Face& a, const Face& b) {
    for (int q = 0; q < 4; ++q)
        if (a.key[q] != b.key[q]) return a.key[q] < b.key[q];
    return false;
}
bool key_eq(const Face& a, const Face& b) {
    return a.key[0] == b.key[0] && a.key[1] == b.key[1] && a.key[2] == b.key[2] && a.key[3] == b.key[3];
}

void build_instance(Inst& I, const std::vector<double>& X, const std::vector<int>& conn) {
#pragma clang fp contract(off)
    static const int fidx[6][4] = {{0, 1, 2, 3}, {4, 5, 6, 7}, {0, 1, 5, 4}, {1, 2, 6, 5}, {2, 3, 7, 6}, {3, 0, 4, 7}};
    const int F = 6 * I.nE;
    I.faces.resize(F);
    for (int j = 0; j < I.nE; ++j) {  // get_element_face, :1944-1992
        const int e = I.e0 + j;
        const int* el = &conn[8 * (size_t)e];
        double ctr[3] = {0, 0, 0};
        for (int a = 0; a < 8; ++a)
            for (int c = 0; c < 3; ++c) ctr[c] += X[3 * (size_t)el[a] + c];
        for (int c = 0; c < 3; ++c) ctr[c] /= 8;
        for (int k = 0; k < 6; ++k) {
            Face& f = I.faces[6 * j + k];
            for (int q = 0; q < 4; ++q) f.n[q] = el[fidx[k][q]];
            const double* x1 = &X[3 * (size_t)f.n[0]];
            const double* x2 = &X[3 * (size_t)f.n[1]];
            const double* x4 = &X[3 * (size_t)f.n[3]];
            const double v1[3] = {x2[0] - x1[0], x2[1] - x1[1], x2[2] - x1[2]};
            const double v2[3] = {x4[0] - x1[0], x4[1] - x1[1], x4[2] - x1[2]};
            const double nv[3] = {v1[1] * v2[2] - v1[2] * v2[1], v1[2] * v2[0] - v1[0] * v2[2],
                                  v1[0] * v2[1] - v1[1] * v2[0]};
            const double vc[3] = {ctr[0] - x1[0], ctr[1] - x1[1], ctr[2] - x1[2]};
            if (nv[0] * vc[0] + nv[1] * vc[1] + nv[2] * vc[2] > 0.) std::swap(f.n[1], f.n[3]);
            for (int q = 0; q < 4; ++q) f.key[q] = f.n[q];
            std::sort(f.key, f.key + 4);
            f.ele = e;
        }
    }
    // faces ordered by (key, index): counting sort on the smallest node, then a stable insertion
    // sort inside each (tiny) bucket -- linear time at millions of faces
    I.order.resize(F);
    {
        int kmin = INT32_MAX, kmax = -1;
        for (const Face& f : I.faces) {
            kmin = std::min(kmin, f.key[0]);
            kmax = std::max(kmax, f.key[0]);
        }
        const int nb = F ? kmax - kmin + 1 : 0;
        std::vector<int> start((size_t)nb + 1, 0);
        for (const Face& f : I.faces) start[f.key[0] - kmin + 1]++;
        for (int b = 0; b < nb; ++b) start[b + 1] += start[b];
        std::vector<int> fill(start.begin(), start.end() - 1);
        for (int i = 0; i < F; ++i) I.order[fill[I.faces[i].key[0] - kmin]++] = i;  // ascending index per bucket
        for (int b = 0; b < nb; ++b)
            for (int q = start[b] + 1; q < start[b + 1]; ++q) {
                const int v = I.order[q];
                int r = q - 1;
                while (r >= start[b] && key_less(I.faces[v], I.faces[I.order[r]])) {
                    I.order[r + 1] = I.order[r];
                    --r;
                }
                I.order[r + 1] = v;
            }
    }
    // get_surface_triangle's scan (:2040-2084): in each run of equal keys o1<o2<..<om the scan
    // pairs (o1,o2), (o3,o4), ...; an odd run keeps its LAST face, unless that is the very last
    // face of the instance (the loop stops at nE*6-1) -- SURVEY §9 Q13.
    I.exterior.clear();
    for (int a = 0; a < F;) {
        int b = a;
        while (b < F && key_eq(I.faces[I.order[a]], I.faces[I.order[b]])) ++b;
        const int m = b - a;
        const int last = I.order[b - 1];
        if ((m & 1) && last != F - 1) I.exterior.push_back(last);
        a = b;
    }
    std::sort(I.exterior.begin(), I.exterior.end());
    // add_surface_triangle (:2167-2245): for each face of the deleted element, the FIRST face (in
    // face order) with the same key that belongs to another element
    I.added.assign(I.nE, {});
    std::vector<int> run_start(F), pos_in_order(F);
    for (int i = 0; i < F; ++i) pos_in_order[I.order[i]] = i;
    for (int a = 0; a < F;) {
        int b = a;
        while (b < F && key_eq(I.faces[I.order[a]], I.faces[I.order[b]])) ++b;
        for (int q = a; q < b; ++q) run_start[I.order[q]] = a;
        a = b;
    }
    for (int j = 0; j < I.nE; ++j)
        for (int k = 0; k < 6; ++k) {
            const int fi = 6 * j + k;
            for (int q = run_start[fi]; q < F && key_eq(I.faces[I.order[q]], I.faces[fi]); ++q) {
                const int cand = I.order[q];
                if (I.faces[cand].ele == I.e0 + j) continue;
                I.added[j].push_back(cand);
                break;
            }
        }
}

}  // namespace

namespace hkc {

void contact_destroy(hakai_ctx* c) {
    Contact* C = c->contact;
    if (!C) return;
    (void)hipStreamSynchronize(c->stream);
    dfree(C->d_par);
    dfree(C->d_seg);
    dfree(C->d_ni_pair); dfree(C->d_ni_node); dfree(C->d_ni_orig); dfree(C->d_ni_aptr); dfree(C->d_ni_add);
    dfree(C->d_nj_pair); dfree(C->d_nj_node); dfree(C->d_nj_orig); dfree(C->d_nj_aptr); dfree(C->d_nj_add);
    dfree(C->d_tri_pair); dfree(C->d_tri_nodes); dfree(C->d_tri_ele); dfree(C->d_tri_adder);
    dfree(C->d_bcnt); dfree(C->d_boff); dfree(C->d_blist); dfree(C->d_ni_bucket); dfree(C->d_ni_map);
    dfree(C->d_bbox); dfree(C->d_evn); dfree(C->d_ev_nodes); dfree(C->d_ev_f); dfree(C->d_cnt); dfree(C->d_off);
    dfree(C->d_terms); dfree(C->d_velo0);
    if (C->d_tmp) (void)hipFree(C->d_tmp);
    delete C;
    c->contact = nullptr;
    dfree(c->d_fext);
}

void contact_state_reset(hakai_ctx* c, const double* velo0_host) {
    Contact* C = c->contact;
    if (!C) return;
    C->use_velo0 = true;
    if (velo0_host)
        (void)hipMemcpyAsync(C->d_velo0, velo0_host, 3 * (size_t)c->nN * sizeof(double), hipMemcpyHostToDevice,
                             c->stream);
}

// contact force of step t into c->d_fext (before the nodal update, :500-560)
int contact_step(hakai_ctx* c, double t, double d_time) {
    Contact* C = c->contact;
    hipStream_t s = c->stream;
    StepIn in;
    in.coord = c->d_coord;
    in.u = c->d_u[c->cur];
    in.u_pre = c->d_u[1 - c->cur];
    in.velo0 = C->use_velo0 ? C->d_velo0 : nullptr;
    in.d_time = d_time;
    in.del_step = c->d_del_step;
    in.flag = c->d_flag;
    in.conn = c->d_conn;
    in.mass = c->d_mass;
    in.t = (int)t;
    const int g12 = (12 * C->npairs + kB - 1) / kB;
    hipLaunchKernelGGL(k_ct_reset, dim3(std::max(g12, 1)), dim3(kB), 0, s, C->d_bbox, C->npairs, C->d_evn);
    if (C->nseg > 0)
        hipLaunchKernelGGL(k_ct_bbox, dim3(C->nseg * kSegBlocks), dim3(kB), 0, s, in, (const Seg*)C->d_seg, C->d_ni_node,
                           C->d_ni_orig, C->d_ni_aptr, C->d_ni_add, C->d_nj_node, C->d_nj_orig, C->d_nj_aptr,
                           C->d_nj_add, C->d_bbox, C->d_ni_bucket);
    if (C->n_ni > 0) {
        hipLaunchKernelGGL(k_ct_bin, dim3((C->n_ni + kB - 1) / kB), dim3(kB), 0, s, in, C->n_ni, C->d_ni_pair,
                           C->d_ni_node, C->d_par, C->d_bbox, C->d_ni_bucket, C->d_ni_map, C->d_bcnt);
    }
    size_t tb = C->tmp_bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(C->d_tmp, tb, C->d_bcnt, C->d_boff, C->htot + 1, s));
    if (C->n_ni > 0)
        hipLaunchKernelGGL(k_ct_fill, dim3((C->n_ni + kB - 1) / kB), dim3(kB), 0, s, C->n_ni, C->d_ni_bucket,
                           C->d_boff, C->d_bcnt, C->d_blist);
    if (C->n_tri > 0)
        hipLaunchKernelGGL(k_ct_tri, dim3((C->n_tri + 127) / 128), dim3(128), 0, s, in, C->n_tri, C->d_tri_pair,
                           C->d_tri_nodes, C->d_tri_ele, C->d_tri_adder, C->d_par, C->d_bbox, C->d_boff, C->d_blist,
                           C->d_ni_node, C->d_ni_map, C->d_lim, C->myu, C->d_evn, C->cap, C->d_ev_nodes, C->d_ev_f);
    const unsigned ge = (unsigned)std::min<long long>((4 * C->cap + kB - 1) / kB, 2048);
    hipLaunchKernelGGL(k_ct_count, dim3(ge), dim3(kB), 0, s, C->d_evn, C->cap, C->d_ev_nodes, C->d_cnt, C->d_evn + 1);
    tb = C->tmp_bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(C->d_tmp, tb, C->d_cnt, C->d_off, (int)c->nN + 1, s));
    hipLaunchKernelGGL(k_ct_scatter, dim3(ge), dim3(kB), 0, s, C->d_evn, C->cap, C->d_ev_nodes, C->d_ev_f, C->d_off,
                       C->d_cnt, C->d_terms);
    hipLaunchKernelGGL(k_ct_sum, dim3((unsigned)((c->nN + kB - 1) / kB)), dim3(kB), 0, s, (long long)c->nN, C->d_off,
                       C->d_terms, c->d_fext);
    HIPCHK(hipGetLastError());
    C->use_velo0 = false;
    return 0;
}

int contact_check(hakai_ctx* c) {
    Contact* C = c->contact;
    if (!C) return 0;
    unsigned int mx = 0;
    HIPCHK(hipMemcpyAsync(&mx, C->d_evn + 1, sizeof(unsigned int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if ((long long)mx > C->cap)
        return fail(HAKAI_ERR_STATE, "contact: %u events in one step exceed the buffer (%lld); raise "
                    "hakai_set_tuning(\"contact_event_cap\")", mx, C->cap);
    return 0;
}

}  // namespace hkc

extern "C" {

int hakai_set_contact(hakai_ctx* c, int32_t contact_flag, const int64_t* element_instance) {
    return hakai_set_contact_cp(c, contact_flag, element_instance, 0, nullptr, nullptr, nullptr);
}

int hakai_set_contact_cp(hakai_ctx* c, int32_t contact_flag, const int64_t* element_instance, int32_t n_cp,
                         const int32_t* cp_instance, const int64_t* cp_elem_off, const int64_t* cp_elems) {
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    if (n_cp < 0 || (n_cp > 0 && (!cp_instance || !cp_elem_off || !cp_elems)))
        return fail(HAKAI_ERR_ARG, "set_contact_cp: bad contact-pair arrays");
    if (!c->model_ok) return fail(HAKAI_ERR_STATE, "set_contact before upload_model");
    HIPCHK(hipSetDevice(c->device));
    hkc::contact_destroy(c);
    if (contact_flag < 1) return 0;
    if (contact_flag > 2) return fail(HAKAI_ERR_ARG, "contact_flag %d (0, 1 or 2)", contact_flag);
    if (c->comm) return fail(HAKAI_ERR_STATE, "contact with a multi-GPU communicator is not supported");
    const int nE = (int)c->nE;
    // instances: contiguous element blocks 1, 2, ... (readInpFile numbers them this way)
    std::vector<Inst> inst;
    for (int e = 0; e < nE; ++e) {
        const long long id = element_instance ? element_instance[e] : 1;
        if (id < 1) return fail(HAKAI_ERR_ARG, "element_instance[%d] = %lld", e + 1, id);
        if ((size_t)id > inst.size()) {
            if ((size_t)id != inst.size() + 1)
                return fail(HAKAI_ERR_ARG, "element_instance must number contiguous element blocks 1, 2, ...");
            inst.emplace_back();
            inst.back().e0 = e;
            inst.back().young = c->h_young[c->h_mat[e]];
        } else if ((size_t)id != inst.size()) {
            return fail(HAKAI_ERR_ARG, "element_instance must number contiguous element blocks 1, 2, ...");
        }
        inst.back().nE++;
    }
    const int ni = (int)inst.size();
    if (ni == 0) return 0;
    for (auto& I : inst) build_instance(I, c->h_coord, c->h_conn);
    // pairs (:273-311) and CT entries (:332-396). With *Contact Pair surfaces the exterior faces of
    // each side are restricted to the surface's elements (get_surface_triangle's "pick up only
    // contact element", :2087-2112 -- applied only when the list is not the whole instance).
    struct CtDef {
        int a, b;                                  // a: points (i side), b: triangles (j side)
        const std::vector<char>* fa = nullptr;     // element filters (instance-local), null = all
        const std::vector<char>* fb = nullptr;
    };
    std::vector<std::vector<char>> filters;
    filters.reserve(2 * (size_t)n_cp);
    std::vector<std::pair<int, int>> cp;
    std::vector<std::pair<const std::vector<char>*, const std::vector<char>*>> cpf;
    if (n_cp > 0) {
        for (int k = 0; k < n_cp; ++k) {
            const std::vector<char>* f[2] = {nullptr, nullptr};
            int id[2];
            for (int s = 0; s < 2; ++s) {
                id[s] = cp_instance[2 * k + s] - 1;
                if (id[s] < 0 || id[s] >= ni) return fail(HAKAI_ERR_ARG, "contact pair %d: instance %d", k + 1, id[s] + 1);
                const long long b0 = cp_elem_off[2 * k + s], b1 = cp_elem_off[2 * k + s + 1];
                std::vector<char> bm((size_t)inst[id[s]].nE, 0);
                for (long long q = b0; q < b1; ++q) {
                    const long long el = cp_elems[q];
                    if (el < 1 || el > inst[id[s]].nE)
                        return fail(HAKAI_ERR_ARG, "contact pair %d: element %lld not in instance %d", k + 1, el, id[s] + 1);
                    bm[el - 1] = 1;
                }
                if (b1 - b0 != inst[id[s]].nE) {  // the reference compares the list length only (:2087)
                    filters.push_back(std::move(bm));
                    f[s] = &filters.back();
                }
            }
            cp.push_back({id[0], id[1]});
            cpf.push_back({f[0], f[1]});
        }
    } else if (ni > 1) {
        for (int i = 0; i < ni; ++i)
            for (int j = (contact_flag == 2 ? i : i + 1); j < ni; ++j) {
                cp.push_back({i, j});
                cpf.push_back({nullptr, nullptr});
            }
    } else {
        cp.push_back({0, 0});
        cpf.push_back({nullptr, nullptr});
    }
    std::vector<CtDef> ct;
    for (size_t k = 0; k < cp.size(); ++k) {
        ct.push_back({cp[k].first, cp[k].second, cpf[k].first, cpf[k].second});
        if (cp[k].first != cp[k].second) ct.push_back({cp[k].second, cp[k].first, cpf[k].second, cpf[k].first});
    }
    auto* C = new hkc::Contact();
    C->npairs = (int)ct.size();
    // element sizes (:404-421)
    {
#pragma clang fp contract(off)
        double mn = INFINITY, mx = -INFINITY;
        for (int e = 0; e < nE; ++e) {
            const int* el = &c->h_conn[8 * (size_t)e];
            const double* p1 = &c->h_coord[3 * (size_t)el[0]];
            const int oth[3] = {1, 3, 4};
            for (int q = 0; q < 3; ++q) {
                const double* p = &c->h_coord[3 * (size_t)el[oth[q]]];
                const double a = p1[0] - p[0], b = p1[1] - p[1], d = p1[2] - p[2];
                const double L = std::sqrt(a * a + b * b + d * d);
                mn = std::min(mn, L);
                mx = std::max(mx, L);
            }
        }
        C->min_size = mn;
        C->max_size = mx;
        C->d_lim = mn * 0.3;  // :2253
    }
    std::vector<int> ni_pair, ni_node, ni_orig, ni_aptr{0}, ni_add;
    std::vector<int> nj_pair, nj_node, nj_orig, nj_aptr{0}, nj_add;
    std::vector<int> tri_pair, tri_nodes, tri_ele, tri_adder, seg;
    // node list of a pair side: initial exterior nodes + nodes exposed by each element's deletion
    auto keep = [](const Inst& I, const std::vector<char>* filt, int f) {
        return !filt || (*filt)[I.faces[f].ele - I.e0];
    };
    auto node_list = [&](int pr, const Inst& I, const std::vector<char>* filt, bool with_adds, std::vector<int>& vp,
                         std::vector<int>& vn, std::vector<int>& vo, std::vector<int>& va, std::vector<int>& vadd) {
        // per node: initial (exterior) or the ascending list of elements whose deletion exposes it;
        // bucketed by node id in linear time (adders arrive in ascending element order)
        const int nN = (int)c->nN;
        std::vector<char> orig((size_t)nN, 0), seen((size_t)nN, 0);
        for (int f : I.exterior)
            if (keep(I, filt, f))
                for (int q = 0; q < 4; ++q) orig[I.faces[f].n[q]] = seen[I.faces[f].n[q]] = 1;
        std::vector<int> cnt((size_t)nN + 1, 0), adders;
        if (with_adds) {
            for (int j = 0; j < I.nE; ++j)
                for (int f : I.added[j])
                    for (int q = 0; q < 4; ++q) {
                        const int n = I.faces[f].n[q];
                        seen[n] = 1;
                        if (!orig[n]) cnt[n + 1]++;
                    }
            for (int n = 0; n < nN; ++n) cnt[n + 1] += cnt[n];
            adders.resize((size_t)cnt[nN]);
            std::vector<int> fill(cnt.begin(), cnt.end() - 1);
            for (int j = 0; j < I.nE; ++j)
                for (int f : I.added[j])
                    for (int q = 0; q < 4; ++q) {
                        const int n = I.faces[f].n[q];
                        if (!orig[n]) adders[fill[n]++] = I.e0 + j;
                    }
        }
        long long count = 0;
        for (int n = 0; n < nN; ++n) {
            if (!seen[n]) continue;
            vp.push_back(pr);
            vn.push_back(n);
            vo.push_back(orig[n]);
            if (!orig[n] && with_adds) {
                int last = -1;
                for (int a = cnt[n]; a < cnt[n + 1]; ++a)
                    if (adders[a] != last) vadd.push_back(last = adders[a]);  // duplicates are adjacent
            }
            va.push_back((int)vadd.size());
            count += orig[n];
        }
        return count;
    };
    int hoff = 0;
    for (int pr = 0; pr < C->npairs; ++pr) {
        const int a = ct[pr].a, b = ct[pr].b;  // a: points (i), b: triangles (j)
        const bool self = a == b;
        PairParam pp;
        pp.young = inst[b].young;  // :367
        pp.self = self;
        pp.kc = self ? C->kc_s : C->kc_o;
        pp.Cr = self ? C->Cr_s : C->Cr_o;
        pp.ddiv = self ? C->max_size * 0.6 : C->max_size * 1.1;  // :2322-2325
        const size_t ni0 = ni_node.size(), nj0 = nj_node.size();
        // surface update (:766-804): c_nodes_i grows for every pair whose point instance lost an
        // element; triangles and c_nodes_j grow only when the triangle instance differs
        const long long c_i = node_list(pr, inst[a], ct[pr].fa, true, ni_pair, ni_node, ni_orig, ni_aptr, ni_add);
        const long long c_j = node_list(pr, inst[b], ct[pr].fb, !self, nj_pair, nj_node, nj_orig, nj_aptr, nj_add);
        long long c_t = 0;
        for (int f : inst[b].exterior) {
            if (!keep(inst[b], ct[pr].fb, f)) continue;
            const int* n = inst[b].faces[f].n;
            const int tv[6] = {n[0], n[1], n[2], n[2], n[3], n[0]};  // :2140-2145
            for (int h = 0; h < 2; ++h) {
                tri_pair.push_back(pr);
                tri_nodes.insert(tri_nodes.end(), tv + 3 * h, tv + 3 * h + 3);
                tri_ele.push_back(inst[b].faces[f].ele);
                tri_adder.push_back(-1);
                ++c_t;
            }
        }
        if (!self)
            for (int j = 0; j < inst[b].nE; ++j)
                for (int f : inst[b].added[j]) {
                    const int* n = inst[b].faces[f].n;
                    const int tv[6] = {n[0], n[1], n[2], n[2], n[3], n[0]};
                    for (int h = 0; h < 2; ++h) {
                        tri_pair.push_back(pr);
                        tri_nodes.insert(tri_nodes.end(), tv + 3 * h, tv + 3 * h + 3);
                        tri_ele.push_back(inst[b].faces[f].ele);
                        tri_adder.push_back(inst[b].e0 + j);
                    }
                }
        if (ni_node.size() > ni0) seg.insert(seg.end(), {(int)ni0, (int)ni_node.size(), pr, 0});
        if (nj_node.size() > nj0) seg.insert(seg.end(), {(int)nj0, (int)nj_node.size(), pr, 1});
        int hs = 64;
        while (hs < 2 * (int)(ni_node.size() - ni0)) hs <<= 1;
        pp.hash_off = hoff;
        pp.hash_size = hs;
        hoff += hs;
        C->h_par.push_back(pp);
        C->pair_inst.push_back(a + 1);
        C->pair_inst.push_back(b + 1);
        C->pair_counts.push_back(c_i);
        C->pair_counts.push_back(c_t);
        C->pair_counts.push_back(c_j);
    }
    C->htot = hoff;
    C->n_ni = (int)ni_node.size();
    C->n_nj = (int)nj_node.size();
    C->n_tri = (int)tri_ele.size();
    C->nseg = (int)seg.size() / 4;
    C->cap = std::max<long long>(1 << 16, 8LL * C->n_ni);
    hipStream_t s = c->stream;
    int rc = 0;
#define UP(dst, v)                                          \
    do {                                                    \
        hipError_t _e = upload(&C->dst, v, s);              \
        if (_e != hipSuccess) rc = hip_fail(_e, #dst);      \
    } while (0)
    UP(d_par, C->h_par);
    UP(d_seg, seg);
    UP(d_ni_pair, ni_pair); UP(d_ni_node, ni_node); UP(d_ni_orig, ni_orig); UP(d_ni_aptr, ni_aptr); UP(d_ni_add, ni_add);
    UP(d_nj_pair, nj_pair); UP(d_nj_node, nj_node); UP(d_nj_orig, nj_orig); UP(d_nj_aptr, nj_aptr); UP(d_nj_add, nj_add);
    UP(d_tri_pair, tri_pair); UP(d_tri_nodes, tri_nodes); UP(d_tri_ele, tri_ele); UP(d_tri_adder, tri_adder);
#undef UP
    c->contact = C;
    if (rc) {
        hkc::contact_destroy(c);
        return rc;
    }
    HIPCHK(dalloc(&C->d_bcnt, (size_t)C->htot + 1));
    HIPCHK(dalloc(&C->d_boff, (size_t)C->htot + 1));
    HIPCHK(dalloc(&C->d_blist, (size_t)C->n_ni));
    HIPCHK(dalloc(&C->d_ni_bucket, (size_t)C->n_ni));
    HIPCHK(dalloc(&C->d_ni_map, 3 * (size_t)C->n_ni));
    HIPCHK(dalloc(&C->d_bbox, 12 * (size_t)C->npairs));
    HIPCHK(dalloc(&C->d_evn, 2));
    HIPCHK(dalloc(&C->d_ev_nodes, 4 * (size_t)C->cap));
    HIPCHK(dalloc(&C->d_ev_f, 3 * (size_t)C->cap));
    HIPCHK(dalloc(&C->d_cnt, (size_t)c->nN + 1));
    HIPCHK(dalloc(&C->d_off, (size_t)c->nN + 1));
    HIPCHK(dalloc(&C->d_terms, 12 * (size_t)C->cap));
    HIPCHK(dalloc(&C->d_velo0, 3 * (size_t)c->nN));
    HIPCHK(dalloc(&c->d_fext, 3 * (size_t)c->nN));
    HIPCHK(hipMemsetAsync(C->d_bcnt, 0, ((size_t)C->htot + 1) * sizeof(int), s));
    HIPCHK(hipMemsetAsync(C->d_cnt, 0, ((size_t)c->nN + 1) * sizeof(int), s));
    HIPCHK(hipMemsetAsync(C->d_evn, 0, 2 * sizeof(unsigned int), s));
    HIPCHK(hipMemsetAsync(c->d_fext, 0, 3 * (size_t)c->nN * sizeof(double), s));
    // velocity before the first step: the state's (IC / uploaded) velocity
    if (!c->h_velo0.empty())
        HIPCHK(hipMemcpyAsync(C->d_velo0, c->h_velo0.data(), 3 * (size_t)c->nN * sizeof(double), hipMemcpyHostToDevice, s));
    else
        HIPCHK(hipMemsetAsync(C->d_velo0, 0, 3 * (size_t)c->nN * sizeof(double), s));
    C->use_velo0 = c->steps_done == 0 || !c->h_velo0.empty();
    size_t t1 = 0, t2 = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, C->d_bcnt, C->d_boff, C->htot + 1, s));
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, C->d_cnt, C->d_off, (int)c->nN + 1, s));
    C->tmp_bytes = std::max(t1, t2);
    HIPCHK(hipMalloc(&C->d_tmp, std::max<size_t>(C->tmp_bytes, 1)));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

int hakai_set_contact_params(hakai_ctx* c, double myu, double kc_o, double kc_s, double Cr_o, double Cr_s) {
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    hkc::Contact* C = c->contact;
    if (!C) return fail(HAKAI_ERR_STATE, "set_contact_params before set_contact");
    C->myu = myu;
    C->kc_o = kc_o;
    C->kc_s = kc_s;
    C->Cr_o = Cr_o;
    C->Cr_s = Cr_s;
    for (auto& p : C->h_par) {
        p.kc = p.self ? kc_s : kc_o;
        p.Cr = p.self ? Cr_s : Cr_o;
    }
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(C->d_par, C->h_par.data(), C->h_par.size() * sizeof(PairParam), hipMemcpyHostToDevice,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int hakai_contact_info(hakai_ctx* c, int32_t* n_pairs, int64_t* info, int32_t cap, double* sizes) {
    if (!c || !n_pairs) return fail(HAKAI_ERR_ARG, "null");
    hkc::Contact* C = c->contact;
    *n_pairs = C ? C->npairs : 0;
    if (!C) return 0;
    for (int p = 0; p < C->npairs && p < cap; ++p) {
        info[5 * p + 0] = C->pair_inst[2 * p];
        info[5 * p + 1] = C->pair_inst[2 * p + 1];
        info[5 * p + 2] = C->pair_counts[3 * p];
        info[5 * p + 3] = C->pair_counts[3 * p + 1];
        info[5 * p + 4] = C->pair_counts[3 * p + 2];
    }
    if (sizes) {
        sizes[0] = C->min_size;
        sizes[1] = C->max_size;
    }
    return 0;
}

int hakai_contact_force(hakai_ctx* c, double t, double d_time, double* external_force) {
    if (!c || !external_force) return fail(HAKAI_ERR_ARG, "null");
    if (!c->contact) return fail(HAKAI_ERR_STATE, "contact_force before set_contact");
    if (!c->state_ok) return fail(HAKAI_ERR_STATE, "contact_force before reset/upload_state");
    HIPCHK(hipSetDevice(c->device));
    const bool keep = c->contact->use_velo0;
    int rc = hkc::contact_step(c, t, d_time);
    c->contact->use_velo0 = keep;  // a probe, not a step
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(external_force, c->d_fext, 3 * (size_t)c->nN * sizeof(double), hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return hkc::contact_check(c);
}

}  // extern "C"
