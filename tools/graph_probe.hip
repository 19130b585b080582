// Launch-cost probe: K tiny dependent kernels per "step", enqueued one by one vs captured once in a
// hipGraph and launched per step. Tells whether graphs pay for the launch-bound small-deck loop
// (tools/bench_small.py: 11 us/step without contact, 81 us/step with contact, host-bound).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

__global__ void k_tiny(double* p, int n, double v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 0.5 + v;
}

int main() {
    const int n = 4096, steps = 2000;
    double* d;
    CK(hipMalloc(&d, n * sizeof(double)));
    CK(hipMemset(d, 0, n * sizeof(double)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int K : {3, 20}) {
        for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_tiny, dim3(16), dim3(256), 0, s, d, n, 1.0);
        CK(hipStreamSynchronize(s));
        auto t0 = std::chrono::steady_clock::now();
        for (int st = 0; st < steps; ++st)
            for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_tiny, dim3(16), dim3(256), 0, s, d, n, (double)k);
        CK(hipStreamSynchronize(s));
        auto t1 = std::chrono::steady_clock::now();
        // one step captured, launched `steps` times; and 16 steps per graph
        for (int per : {1, 16}) {
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            for (int r = 0; r < per; ++r)
                for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_tiny, dim3(16), dim3(256), 0, s, d, n, (double)k);
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CK(hipGraphLaunch(ge, s));
            CK(hipStreamSynchronize(s));
            auto t2 = std::chrono::steady_clock::now();
            for (int st = 0; st < steps / per; ++st) CK(hipGraphLaunch(ge, s));
            auto t3 = std::chrono::steady_clock::now();
            CK(hipStreamSynchronize(s));
            auto t4 = std::chrono::steady_clock::now();
            auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
            std::printf("K=%2d kernels/step: stream %.2f us/step | graph(%2d steps/graph) %.2f us/step (host enqueue %.2f)\n",
                        K, us(t0, t1) / steps, per, us(t2, t4) / steps, us(t2, t3) / steps);
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
        }
    }
    CK(hipFree(d));
    return 0;
}
