// LDS-DMA semantics probe (tools, not product code): where do global_load_lds_dword{,x3,x4} (SGPR base,
// instruction offset) land in LDS? Measured on gfx950: lane stride 16 B for x3 and x4, 4 B for
// dword, and the instruction offset moves the LDS address too (profiles/r03_dma_probe.log).
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(unsigned long long)(const __attribute__((address_space(3))) void*)p;
}
#define DMA(NAME, INSN)                                                                              \
    template <int OFF>                                                                               \
    __device__ __forceinline__ void NAME(unsigned voff, const void* sbase, unsigned m0) {            \
        unsigned keep;                                                                               \
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t" INSN " %1, %2 offset:%4\n\ts_mov_b32 m0, %0" \
                     : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(m0), "i"(OFF) : "memory");           \
    }
DMA(dma, "global_load_lds_dwordx3")
DMA(dma4, "global_load_lds_dwordx4")
DMA(dma1, "global_load_lds_dword")
__global__ void k(const unsigned* g, unsigned* out) {
    __shared__ unsigned s[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) s[i] = 0xFFFFFFFFu;
    __syncthreads();
    const unsigned base = lds_addr(s);
    const unsigned voff = 4u * 100u * threadIdx.x;  // lane l reads g[100 l ...]
    dma<0>(voff, g, base);                 // case A: offset 0 at s[0]
    dma<12>(voff, g, base + 4096u);        // case B: offset 12 at byte 4096 (s[1024])
    dma4<0>(voff, g, base + 8192u);        // case C: dwordx4 at s[2048]
    dma1<16>(voff, g, base + 12288u);      // case D: dword, offset 16, at byte 12288 (s[3072])
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 4096; i += 64) out[i] = s[i];
}
int main() {
    unsigned h[8000];
    for (int i = 0; i < 8000; ++i) h[i] = i;
    unsigned *dg, *dout;
    hipMalloc(&dg, sizeof h); hipMalloc(&dout, 4096 * 4);
    hipMemcpy(dg, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dg, dout);
    unsigned o[4096];
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    printf("A (offset 0, M0 = s[0]):");
    for (int i = 0; i < 12; ++i) printf(" %u", o[i]);
    printf(" ... s[189..194]:");
    for (int i = 189; i < 195; ++i) printf(" %d", (int)o[i]);
    printf("\nB (offset 12, M0 = s[1024]): s[1018..1035]:");
    for (int i = 1018; i < 1036; ++i) printf(" %d", (int)o[i]);
    printf("\nC (dwordx4, offset 0, M0 = s[2048]): s[2048..2055]:");
    for (int i = 2048; i < 2056; ++i) printf(" %d", (int)o[i]);
    printf("\nD (dword, offset 16, M0 = s[3072]): s[3074..3081]:");
    for (int i = 3074; i < 3082; ++i) printf(" %d", (int)o[i]);
    printf("\n");
    return 0;
}
