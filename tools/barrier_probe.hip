// Grid-barrier probe: what does a software barrier between the phases of ONE persistent kernel
// cost on gfx950, against a kernel boundary in a hipGraph? (Candidate for fusing the ~13 small
// contact kernels of the reference's decks into one launch.) Variants: the working workgroups
// spread over all XCDs, or all on XCD 0 (blockIdx % 8 == 0; the others exit at once), where one
// L2 holds every line the phases exchange. Every spin is bounded: on timeout the kernel records an
// error and carries on, so a missing workgroup cannot hang the GPU.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

__device__ __forceinline__ void grid_barrier(unsigned* bar, unsigned target, int* err) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        int it = 0;
        while (__hip_atomic_load(&bar[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (++it > (1 << 20)) {
                atomicExch(err, 1);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

// P phases; phase p: every working thread reads the value its right neighbour workgroup wrote in
// phase p-1 (a real cross-workgroup dependency) and writes its own.
__global__ void k_phases(int P, double* data, unsigned* bar, int* err, int xcd_only, int nwork) {
    int wid = blockIdx.x;
    if (xcd_only) {
        if (blockIdx.x % 8 != 0) return;
        wid = blockIdx.x / 8;
    }
    const int n = nwork * blockDim.x;
    const int i = wid * blockDim.x + threadIdx.x;
    for (int p = 0; p < P; ++p) {
        const double v = data[(p & 1) * n + (i + blockDim.x) % n];
        data[((p + 1) & 1) * n + i] = v * 0.5 + p;
        grid_barrier(bar, (unsigned)(p + 1) * nwork, err);
    }
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(&bar[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nwork - 1) {
        __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&bar[1], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void k_one_phase(double* data, int n, int p) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) data[((p + 1) & 1) * n + i] = data[(p & 1) * n + (i + blockDim.x) % n] * 0.5 + p;
}

int main() {
    const int B = 256, reps = 300, P = 12;
    double* d;
    unsigned* bar;
    int* err;
    CK(hipMalloc(&d, 2 * 256 * B * sizeof(double)));
    CK(hipMemset(d, 0, 2 * 256 * B * sizeof(double)));
    CK(hipMalloc(&bar, 2 * sizeof(unsigned)));
    CK(hipMemset(bar, 0, 2 * sizeof(unsigned)));
    CK(hipMalloc(&err, sizeof(int)));
    CK(hipMemset(err, 0, sizeof(int)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](auto&& launch) {
        for (int r = 0; r < 20; ++r) launch();
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return 1000.0 * ms / reps;
    };
    for (int xcd : {1, 0}) {
        for (int nw : {8, 16, 32, 64, 128}) {
            if (xcd && nw > 32) continue;
            const int grid = xcd ? 8 * nw : nw;
            const double t0 = timed([&] { hipLaunchKernelGGL(k_phases, dim3(grid), dim3(B), 0, s, 0, d, bar, err, xcd, nw); });
            const double t1 = timed([&] { hipLaunchKernelGGL(k_phases, dim3(grid), dim3(B), 0, s, P, d, bar, err, xcd, nw); });
            int e = 0;
            CK(hipMemcpy(&e, err, sizeof(int), hipMemcpyDeviceToHost));
            std::printf("%s %3d workgroups: launch %.2f us, %d phases %.2f us -> %.2f us per barrier%s\n",
                        xcd ? "XCD0 " : "all  ", nw, t0, P, t1, (t1 - t0) / P, e ? "  [TIMEOUT]" : "");
        }
    }
    // the same P phases as P kernels captured in one graph
    for (int nw : {8, 64}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int p = 0; p < P; ++p) hipLaunchKernelGGL(k_one_phase, dim3(nw), dim3(B), 0, s, d, nw * B, p);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        const double tg = timed([&] { CK(hipGraphLaunch(ge, s)); });
        std::printf("graph of %d kernels, %3d workgroups each: %.2f us -> %.2f us per kernel\n", P, nw, tg, tg / P);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
