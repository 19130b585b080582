// pmc_calib.hip -- known-byte kernels for calibrating rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950
// in the access widths the element and nodal kernels use (MI355X_MICROARCH.md "HBM": only 16-B/lane
// reads (FETCH_SIZE = 1/2 bytes) and 16-B/lane writes (exact) are calibrated there).
// Each kernel moves exactly kBytes of HBM traffic (arrays 1 GiB, well past the 256 MiB L3).
// Run under rocprofv3 --pmc FETCH_SIZE (one pass) and --pmc WRITE_SIZE (another pass);
// tools/pmc_report.py divides the counters by kBytes to get the per-pattern factor.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr size_t kBytes = size_t(1) << 30;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

template <class T>
__global__ void calib_read(const T* __restrict__ in, size_t n, double* __restrict__ sink) {
    double acc = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = in[i];
        acc += (double)((const unsigned char*)&v)[0];
    }
    if (acc == -1.0) sink[0] = acc;  // never true; keeps the loads alive without extra traffic
}

__global__ void calib_read_d2(const double2* __restrict__ in, size_t n, double* __restrict__ sink) {
    double acc = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = in[i];
        acc += v.x + v.y;
    }
    if (acc == -1.0) sink[0] = acc;
}

template <class T>
__global__ void calib_write(T* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = (T)i;
}

__global__ void calib_write_d2(double2* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = make_double2((double)i, 1.0);
}

// Nontemporal forms (the element kernel streams its Gauss-point state with these)
__global__ void calib_read_nt(const double* __restrict__ in, size_t n, double* __restrict__ sink) {
    double acc = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += __builtin_nontemporal_load(in + i);
    if (acc == -1.0) sink[0] = acc;
}

__global__ void calib_write_nt(double* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store((double)i, out + i);
}

// The element kernel's force store: lane writes 3 doubles at a 24-B stride ([8 nE][3] AoS).
__global__ void calib_write_aos3(double* __restrict__ out, size_t n3) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n3; i += (size_t)gridDim.x * blockDim.x) {
        out[3 * i + 0] = (double)i;
        out[3 * i + 1] = 1.0;
        out[3 * i + 2] = 2.0;
    }
}

// The node gathers: lane reads 3 doubles at a 24-B stride.
__global__ void calib_read_aos3(const double* __restrict__ in, size_t n3, double* __restrict__ sink) {
    double acc = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n3; i += (size_t)gridDim.x * blockDim.x)
        acc += in[3 * i] + in[3 * i + 1] + in[3 * i + 2];
    if (acc == -1.0) sink[0] = acc;
}

int main() {
    void* a = nullptr;
    double* sink = nullptr;
    CK(hipMalloc(&a, kBytes));
    CK(hipMalloc((void**)&sink, 64));
    CK(hipMemset(a, 1, kBytes));
    const dim3 g(4096), b(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(calib_read<double>, g, b, 0, 0, (const double*)a, kBytes / 8, sink);
        hipLaunchKernelGGL(calib_read<int>, g, b, 0, 0, (const int*)a, kBytes / 4, sink);
        hipLaunchKernelGGL(calib_read_d2, g, b, 0, 0, (const double2*)a, kBytes / 16, sink);
        hipLaunchKernelGGL(calib_read_aos3, g, b, 0, 0, (const double*)a, kBytes / 24, sink);
        hipLaunchKernelGGL(calib_write<double>, g, b, 0, 0, (double*)a, kBytes / 8);
        hipLaunchKernelGGL(calib_write<int>, g, b, 0, 0, (int*)a, kBytes / 4);
        hipLaunchKernelGGL(calib_write_d2, g, b, 0, 0, (double2*)a, kBytes / 16);
        hipLaunchKernelGGL(calib_write_aos3, g, b, 0, 0, (double*)a, kBytes / 24);
        hipLaunchKernelGGL(calib_read_nt, g, b, 0, 0, (const double*)a, kBytes / 8, sink);
        hipLaunchKernelGGL(calib_write_nt, g, b, 0, 0, (double*)a, kBytes / 8);
        CK(hipGetLastError());
    }
    CK(hipDeviceSynchronize());
    std::printf("pmc_calib: %zu bytes per kernel\n", kBytes);
    CK(hipFree(a));
    CK(hipFree(sink));
    return 0;
}
