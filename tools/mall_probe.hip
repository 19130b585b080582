// Infinity Cache (256 MiB MALL) probe for two-step temporal blocking of the element update.
// Question: if the element kernel runs step s and then step s+1 over the SAME chunk of elements
// before moving on, do the second pass's Gauss-point state reads hit the Infinity Cache, and are
// the first pass's stores absorbed there (overwritten by the second pass before write-back)?
// The state is laid out like the library's: 14 FP64 arrays of ld = 8*nE entries (stress 6,
// strain 6, eqps, yield), 896 B per element, read and written in place once per pass.
// Modes: "full" = two passes over the whole array; "chunk C" = per chunk of C elements, two
// passes over that chunk. Per-pass time = total / 2. nt selects nontemporal loads (bit 0) and
// stores (bit 1), the library's elem_gp_nt key.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

constexpr int NA = 14;
typedef double d2 __attribute__((ext_vector_type(2)));

template <int NT>
__global__ __launch_bounds__(256) void k_pass(double* __restrict__ s, long ld, long g0, long g1, double a) {
    const long stride = (long)gridDim.x * blockDim.x * 2;
    for (long g = g0 + ((long)blockIdx.x * blockDim.x + threadIdx.x) * 2; g < g1; g += stride) {
        d2 v[NA];
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            const d2* p = reinterpret_cast<const d2*>(s + k * ld + g);
            if (NT & 1)
                v[k] = __builtin_nontemporal_load(p);
            else
                v[k] = *p;
        }
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            v[k].x = v[k].x * a + 1e-9;
            v[k].y = v[k].y * a + 1e-9;
            d2* p = reinterpret_cast<d2*>(s + k * ld + g);
            if (NT & 2)
                __builtin_nontemporal_store(v[k], p);
            else
                *p = v[k];
        }
    }
}

static void launch(int nt, double* s, long ld, long g0, long g1, hipStream_t st) {
    const long n = (g1 - g0) / 2;
    int blocks = (int)std::min<long>((n + 255) / 256, 256L * 8);
    switch (nt) {
        case 0: k_pass<0><<<blocks, 256, 0, st>>>(s, ld, g0, g1, 0.999); break;
        case 1: k_pass<1><<<blocks, 256, 0, st>>>(s, ld, g0, g1, 0.999); break;
        case 2: k_pass<2><<<blocks, 256, 0, st>>>(s, ld, g0, g1, 0.999); break;
        default: k_pass<3><<<blocks, 256, 0, st>>>(s, ld, g0, g1, 0.999); break;
    }
}

int main(int argc, char** argv) {
    const long nE = argc > 1 ? atol(argv[1]) : 2000000;
    const long ld = 8 * nE;
    double* s;
    CK(hipMalloc(&s, sizeof(double) * NA * ld));
    CK(hipMemset(s, 0, sizeof(double) * NA * ld));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes_pass = 2.0 * NA * 8.0 * ld;  // read + write per pass
    std::vector<long> chunks_mb = {0, 8, 16, 32, 48, 64, 96, 128, 192, 256};
    for (int nt : {0, 3, 1, 2}) {
        for (long cmb : chunks_mb) {
            const long cE = cmb == 0 ? nE : std::max(32L, (cmb << 20) / (NA * 8 * 8) / 32 * 32);
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipEventRecord(e0, st));
                for (long e = 0; e < nE; e += cE) {
                    const long g0 = 8 * e, g1 = 8 * std::min(nE, e + cE);
                    launch(nt, s, ld, g0, g1, st);
                    launch(nt, s, ld, g0, g1, st);
                }
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep > 0 && ms < best) best = ms;
            }
            const double per_pass = best / 2.0;
            std::printf("{\"nt\": %d, \"chunk_mb\": %ld, \"chunk_elems\": %ld, \"launches\": %ld, "
                        "\"ms_per_pass\": %.4f, \"eff_TBps\": %.3f}\n",
                        nt, cmb, cE, 2 * ((nE + cE - 1) / cE), per_pass, bytes_pass / (per_pass * 1e-3) / 1e12);
            std::fflush(stdout);
        }
    }
    CK(hipFree(s));
    return 0;
}
