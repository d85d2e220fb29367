// Microbenchmark: throughput of the GF(2^16) butterfly (rs16_gf.hpp mul_xor +
// XOR) with the table in VGPRs, 16 rows per thread, at a given number of
// waves per SIMD.  Reports cycles per wave-butterfly at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../reed-solomon-16_amd/csrc/rs16_gf.hpp"
using namespace rs16;
#define ITER 256
template <int MODE>
__global__ void __launch_bounds__(256) k(unsigned* out, const unsigned* tab, unsigned long long* clk, unsigned seed) {
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    unsigned L[16], H[16];
    for (int i = 0; i < 16; i++) { L[i] = seed * (threadIdx.x + i + 1); H[i] = L[i] * 7 + i; }
    unsigned t[20];
    for (int i = 0; i < 20; i++) t[i] = tab[(blockIdx.x & 7) * 32 + i];
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int s = 0; s < 4; s++) {
#pragma unroll
            for (int g = 0; g < 8; g++) {
                const int rb = s, m = ((g >> rb) << (rb + 1)) + (g & ((1 << rb) - 1)), m2 = m + (1 << rb);
                if (MODE == 0) {  // FFT butterfly
                    mul_xor(L[m], H[m], L[m2], H[m2], t);
                    L[m2] ^= L[m]; H[m2] ^= H[m];
                } else {          // IFFT butterfly
                    L[m2] ^= L[m]; H[m2] ^= H[m];
                    mul_xor(L[m], H[m], L[m2], H[m2], t);
                }
            }
            asm volatile("" ::: "memory");
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    unsigned r = 0;
    for (int i = 0; i < 16; i++) r ^= L[i] ^ H[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
static unsigned long long* g_clk;
static double g_ghz = 2.4;
template <int MODE> float run(unsigned* d, const unsigned* tab, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k<MODE><<<blocks, 256>>>(d, tab, g_clk, 1);
    hipEventRecord(a);
    k<MODE><<<blocks, 256>>>(d, tab, g_clk, 1);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    unsigned long long c[2];
    hipMemcpy(c, g_clk, sizeof c, hipMemcpyDeviceToHost);
    g_ghz = c[1] ? (double)c[0] / ((double)c[1] * 10.0) : 2.4;
    return ms;
}
int main() {
    unsigned* d; unsigned* tab;
    hipMalloc(&d, 256 * 16 * 256 * 4);
    hipMalloc(&tab, 8 * 32 * 4);
    hipMalloc(&g_clk, 16);
    hipMemset(tab, 0x5a, 8 * 32 * 4);
    for (int wps = 1; wps <= 8; wps *= 2) {
        int blocks = 256 * wps;  // 256-thread blocks = 1 wave per SIMD each
        float ms0 = run<0>(d, tab, blocks), ms1 = run<1>(d, tab, blocks);
        double bf = (double)blocks * 4 * ITER * 32;  // wave-butterflies
        const double g0 = g_ghz;
        float ms1b = run<1>(d, tab, blocks);
        const double g1 = g_ghz;
        (void)ms1;
        printf("waves/SIMD %d: FFT %.3f ms @ %.2f GHz (%.1f cyc/wave-bfly/SIMD = %.2f per instr of 30)  IFFT %.3f ms @ %.2f GHz (%.1f)\n",
               wps, ms0, g0, ms0 * 1e-3 * g0 * 1e9 * 1024 / bf, ms0 * 1e-3 * g0 * 1e9 * 1024 / bf / 30, ms1b, g1,
               ms1b * 1e-3 * g1 * 1e9 * 1024 / bf);
    }
    return 0;
}
