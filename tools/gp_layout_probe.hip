// gp_layout_probe.hip -- profiling helper (not part of the product): does the Gauss-point state's
// HBM layout limit the element kernel's streaming rate?
//
// The element kernel reads and writes 14 FP64 components per Gauss point (stress 6, strain 6, eqps,
// yield) in SoA arrays [14][ld]: per 32-element batch a block touches 14 separate 2 KB runs for
// reading and 14 for writing, so 512 blocks keep ~14 000 streams open. This probe streams the same
// bytes with the same grid and per-block batch ranges in three layouts and prints GB/s:
//   soa   : component c of GP g at c*ld + g (the product's layout);
//   aosoa : per batch, all 14 components contiguous: [batch][c][256] (one 28 KB run per batch);
//   copy  : float4 read + write of the same byte count (the copy rate).
// Loads are plain, stores nontemporal (as gp_nt in the element kernel), read-modify-write in place.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHK(x)                                                                        \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

constexpr int kC = 14;

__global__ __launch_bounds__(256, 2) void k_soa(double* base, long long ld, long long nb, double s) {
    const long long b0 = (long long)blockIdx.x * nb / gridDim.x, b1 = ((long long)blockIdx.x + 1) * nb / gridDim.x;
    for (long long b = b0; b < b1; ++b) {
        const long long g = b * 256 + threadIdx.x;
        double v[kC];
#pragma unroll
        for (int c = 0; c < kC; ++c) v[c] = base[c * ld + g];
#pragma unroll
        for (int c = 0; c < kC; ++c) __builtin_nontemporal_store(v[c] * s, base + c * ld + g);
    }
}

__global__ __launch_bounds__(256, 2) void k_aosoa(double* base, long long nb, double s) {
    const long long b0 = (long long)blockIdx.x * nb / gridDim.x, b1 = ((long long)blockIdx.x + 1) * nb / gridDim.x;
    for (long long b = b0; b < b1; ++b) {
        double* p = base + b * (kC * 256) + threadIdx.x;
        double v[kC];
#pragma unroll
        for (int c = 0; c < kC; ++c) v[c] = p[c * 256];
#pragma unroll
        for (int c = 0; c < kC; ++c) __builtin_nontemporal_store(v[c] * s, p + c * 256);
    }
}

__global__ __launch_bounds__(256, 2) void k_copy(const float4* a, float4* b, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        b[i] = a[i];
}

int main() {
    const long long nE = 2000000, nb = nE / 32, ld = nb * 256;
    const size_t bytes = (size_t)kC * ld * sizeof(double);
    double* d = nullptr;
    float4 *x = nullptr, *y = nullptr;
    CHK(hipMalloc(&d, bytes));
    CHK(hipMemset(d, 0, bytes));
    CHK(hipMalloc(&x, bytes));
    CHK(hipMalloc(&y, bytes));
    CHK(hipMemset(x, 0, bytes));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const int grid = 512, reps = 20;
    for (int round = 0; round < 3; ++round) {
        for (int mode = 0; mode < 3; ++mode) {
            auto launch = [&]() {
                if (mode == 0) hipLaunchKernelGGL(k_soa, dim3(grid), dim3(256), 0, 0, d, ld, nb, 1.0);
                else if (mode == 1) hipLaunchKernelGGL(k_aosoa, dim3(grid), dim3(256), 0, 0, d, nb, 1.0);
                else hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, x, y, (long long)(bytes / 16));
            };
            launch();
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(e0));
            for (int r = 0; r < reps; ++r) launch();
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms = 0.f;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            const double per = ms / reps;
            const double gbs = 2.0 * (double)bytes / (per * 1e-3) / 1e9;
            std::printf("{\"round\": %d, \"layout\": \"%s\", \"ms\": %.4f, \"GBs_read_plus_write\": %.1f}\n", round,
                        mode == 0 ? "soa" : mode == 1 ? "aosoa" : "copy", per, gbs);
        }
    }
    return 0;
}
