// nodal_probe.hip -- what bounds the nodal kernel? Times variants of the C3 nodal gather on a
// 20x20x5000 structured bar (2.2 M nodes, 2 M elements) with the library's data layout:
//   full      the product kernel's work: inc8 table, 8 gathers of 24 B, central difference;
//   gather    inc8 + gathers, writes Q only;
//   stream    no gather: u, u_pre, mass -> u_new;
//   noidx     gathers with the incidence computed from the structured index (no inc8 loads);
//   wide      full, but 2 nodes per thread (more loads in flight per wave).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/nodal_probe tools/nodal_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

constexpr int NX = 20, NY = 20, NZ = 5000;
constexpr long long NN = (long long)(NX + 1) * (NY + 1) * (NZ + 1);
constexpr long long NE = (long long)NX * NY * NZ;

struct Args {
    const double* u;
    double* out;
    const double* mass;
    const int* inc8;
    const double* fe;
    double dt;
};

__device__ __forceinline__ void update(const Args& a, long long n, double Q0, double Q1, double Q2) {
#pragma clang fp contract(off)
    const double m = a.mass[n], dt = a.dt;
    const double mdt2 = m / (dt * dt), inv = 1.0 / mdt2;
    const double Q[3] = {Q0, Q1, Q2};
    for (int c = 0; c < 3; ++c) {
        const double uc = a.u[3 * n + c], up = a.out[3 * n + c];
        a.out[3 * n + c] = inv * (0.0 - Q[c] + mdt2 * (2.0 * uc - up));
    }
}

__device__ __forceinline__ void gather(const Args& a, const int* idx, double& Q0, double& Q1, double& Q2) {
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
}

__device__ __forceinline__ void load_idx(const Args& a, long long n, int* idx) {
    const int4 lo = reinterpret_cast<const int4*>(a.inc8)[2 * n];
    const int4 hi = reinterpret_cast<const int4*>(a.inc8)[2 * n + 1];
    idx[0] = lo.x; idx[1] = lo.y; idx[2] = lo.z; idx[3] = lo.w;
    idx[4] = hi.x; idx[5] = hi.y; idx[6] = hi.z; idx[7] = hi.w;
}

__global__ __launch_bounds__(256) void k_full(Args a) {
#pragma clang fp contract(off)
    const long long n = blockIdx.x * 256LL + threadIdx.x;
    if (n >= NN) return;
    int idx[8];
    load_idx(a, n, idx);
    double Q0 = 0, Q1 = 0, Q2 = 0;
    gather(a, idx, Q0, Q1, Q2);
    update(a, n, Q0, Q1, Q2);
}

__global__ __launch_bounds__(256) void k_gather(Args a) {
#pragma clang fp contract(off)
    const long long n = blockIdx.x * 256LL + threadIdx.x;
    if (n >= NN) return;
    int idx[8];
    load_idx(a, n, idx);
    double Q0 = 0, Q1 = 0, Q2 = 0;
    gather(a, idx, Q0, Q1, Q2);
    a.out[3 * n] = Q0;
    a.out[3 * n + 1] = Q1;
    a.out[3 * n + 2] = Q2;
}

__global__ __launch_bounds__(256) void k_stream(Args a) {
    const long long n = blockIdx.x * 256LL + threadIdx.x;
    if (n >= NN) return;
    update(a, n, 0.0, 0.0, 0.0);
}

__device__ __forceinline__ void structured_idx(long long n, int* idx) {
    const int ix = (int)(n % (NX + 1)), iy = (int)((n / (NX + 1)) % (NY + 1)), iz = (int)(n / ((NX + 1) * (NY + 1)));
    int c = 0;
    const int pad = (int)(24 * ((NE + 31) / 32 * 32));
    for (int dz = -1; dz <= 0; ++dz)
        for (int dy = -1; dy <= 0; ++dy)
            for (int dx = -1; dx <= 0; ++dx) {
                const int ex = ix + dx, ey = iy + dy, ez = iz + dz;
                if (ex < 0 || ey < 0 || ez < 0 || ex >= NX || ey >= NY || ez >= NZ) continue;
                const int e = ex + NX * (ey + NY * ez);
                const int k = (dx == 0 ? 0 : 1) + (dy == 0 ? 0 : 2) + (dz == 0 ? 0 : 4);  // local node (bit order)
                const int kk[8] = {0, 1, 3, 2, 4, 5, 7, 6};
                idx[c++] = 24 * e + 3 * kk[k];
            }
    while (c < 8) idx[c++] = pad;
}

__global__ __launch_bounds__(256) void k_noidx(Args a) {
#pragma clang fp contract(off)
    const long long n = blockIdx.x * 256LL + threadIdx.x;
    if (n >= NN) return;
    int idx[8];
    structured_idx(n, idx);
    double Q0 = 0, Q1 = 0, Q2 = 0;
    gather(a, idx, Q0, Q1, Q2);
    update(a, n, Q0, Q1, Q2);
}

__global__ __launch_bounds__(256) void k_wide(Args a) {
#pragma clang fp contract(off)
    const long long n0 = (blockIdx.x * 256LL + threadIdx.x);
    const long long half = (NN + 1) / 2;
    if (n0 >= half) return;
    const long long n1 = n0 + half;
    int i0[8], i1[8];
    load_idx(a, n0, i0);
    if (n1 < NN) load_idx(a, n1, i1);
    double Q0 = 0, Q1 = 0, Q2 = 0, R0 = 0, R1 = 0, R2 = 0;
    gather(a, i0, Q0, Q1, Q2);
    if (n1 < NN) gather(a, i1, R0, R1, R2);
    update(a, n0, Q0, Q1, Q2);
    if (n1 < NN) update(a, n1, R0, R1, R2);
}

__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned nwg) {
    if (nwg < 16) return b;
    const unsigned xcd = b & 7u, q = nwg >> 3, r = nwg & 7u;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// product form (XCD remap), loads in program order
__global__ __launch_bounds__(256) void k_remap(Args a) {
#pragma clang fp contract(off)
    const long long n = xcd_remap(blockIdx.x, gridDim.x) * 256LL + threadIdx.x;
    if (n >= NN) return;
    int idx[8];
    load_idx(a, n, idx);
    double Q0 = 0, Q1 = 0, Q2 = 0;
    gather(a, idx, Q0, Q1, Q2);
    update(a, n, Q0, Q1, Q2);
}

// XCD remap + the update's loads issued first, so they fly with the index loads
__global__ __launch_bounds__(256) void k_early(Args a) {
#pragma clang fp contract(off)
    const long long n = xcd_remap(blockIdx.x, gridDim.x) * 256LL + threadIdx.x;
    if (n >= NN) return;
    const double m = a.mass[n];
    double uc[3], up[3];
    for (int c = 0; c < 3; ++c) {
        uc[c] = a.u[3 * n + c];
        up[c] = a.out[3 * n + c];
    }
    int idx[8];
    load_idx(a, n, idx);
    double Q[3] = {0, 0, 0};
    gather(a, idx, Q[0], Q[1], Q[2]);
    const double dt = a.dt, mdt2 = m / (dt * dt), inv = 1.0 / mdt2;
    for (int c = 0; c < 3; ++c) a.out[3 * n + c] = inv * (0.0 - Q[c] + mdt2 * (2.0 * uc[c] - up[c]));
}

// XCD remap, early loads, 2 nodes per thread (n and n + 256 within a 512-node block)
__global__ __launch_bounds__(256) void k_early2(Args a) {
#pragma clang fp contract(off)
    const long long base = xcd_remap(blockIdx.x, gridDim.x) * 512LL + threadIdx.x;
    double m[2], uc[2][3], up[2][3], Q[2][3] = {{0, 0, 0}, {0, 0, 0}};
    int idx[2][8];
    bool ok[2];
    for (int h = 0; h < 2; ++h) {
        const long long n = base + 256 * h;
        ok[h] = n < NN;
        const long long nn = ok[h] ? n : NN - 1;
        m[h] = a.mass[nn];
        for (int c = 0; c < 3; ++c) {
            uc[h][c] = a.u[3 * nn + c];
            up[h][c] = a.out[3 * nn + c];
        }
        load_idx(a, nn, idx[h]);
    }
    for (int h = 0; h < 2; ++h) gather(a, idx[h], Q[h][0], Q[h][1], Q[h][2]);
    const double dt = a.dt;
    for (int h = 0; h < 2; ++h) {
        if (!ok[h]) continue;
        const long long n = base + 256 * h;
        const double mdt2 = m[h] / (dt * dt), inv = 1.0 / mdt2;
        for (int c = 0; c < 3; ++c) a.out[3 * n + c] = inv * (0.0 - Q[h][c] + mdt2 * (2.0 * uc[h][c] - up[h][c]));
    }
}

int main() {
    // incidence like the library: ascending element order, rows 24e+3k, pad -> zero row
    const long long nEp = (NE + 31) / 32 * 32;
    std::vector<int> cnt(NN, 0), inc8(8 * NN, (int)(24 * nEp));
    const int kmap[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};
    for (long long e = 0; e < NE; ++e) {
        const int ex = (int)(e % NX), ey = (int)((e / NX) % NY), ez = (int)(e / (NX * NY));
        for (int k = 0; k < 8; ++k) {
            const long long n = (ex + kmap[k][0]) + (NX + 1) * ((ey + kmap[k][1]) + (NY + 1) * (long long)(ez + kmap[k][2]));
            inc8[8 * n + cnt[n]++] = (int)(24 * e + 3 * k);
        }
    }
    double *u, *out, *mass, *fe;
    int* d_inc8;
    CK(hipMalloc(&u, 3 * NN * 8));
    CK(hipMalloc(&out, 3 * NN * 8));
    CK(hipMalloc(&mass, NN * 8));
    CK(hipMalloc(&fe, (24 * nEp + 8) * 8));
    CK(hipMalloc(&d_inc8, 8 * NN * 4));
    CK(hipMemcpy(d_inc8, inc8.data(), 8 * NN * 4, hipMemcpyHostToDevice));
    CK(hipMemset(u, 0, 3 * NN * 8));
    CK(hipMemset(out, 0, 3 * NN * 8));
    CK(hipMemset(fe, 0, (24 * nEp + 8) * 8));
    std::vector<double> ms(NN, 1e-8);
    CK(hipMemcpy(mass, ms.data(), NN * 8, hipMemcpyHostToDevice));
    Args a{u, out, mass, d_inc8, fe, 1e-7};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned g = (unsigned)((NN + 255) / 256), g2 = (unsigned)(((NN + 1) / 2 + 255) / 256);
    struct V { const char* name; void (*k)(Args); unsigned grid; double mb; };
    const double nb = (double)NN;
    V vs[] = {{"full", k_full, g, nb * (32 + 192 + 48 + 8 + 24) / 1e6},
              {"gather", k_gather, g, nb * (32 + 192 + 24) / 1e6},
              {"stream", k_stream, g, nb * (48 + 8 + 24) / 1e6},
              {"noidx", k_noidx, g, nb * (192 + 48 + 8 + 24) / 1e6},
              {"wide", k_wide, g2, nb * (32 + 192 + 48 + 8 + 24) / 1e6},
              {"remap", k_remap, g, nb * (32 + 192 + 48 + 8 + 24) / 1e6},
              {"early", k_early, g, nb * (32 + 192 + 48 + 8 + 24) / 1e6},
              {"early2", k_early2, (unsigned)((NN + 511) / 512), nb * (32 + 192 + 48 + 8 + 24) / 1e6}};
    for (int rep = 0; rep < 2; ++rep)
        for (auto& v : vs) {
            hipLaunchKernelGGL(v.k, dim3(v.grid), dim3(256), 0, 0, a);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(v.k, dim3(v.grid), dim3(256), 0, 0, a);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (rep) std::printf("%-8s %.4f ms  %.0f MB  %.2f TB/s\n", v.name, t / 20, v.mb, v.mb / (t / 20) / 1e3);
        }
    return 0;
}
