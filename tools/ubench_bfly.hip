// Microbenchmark: throughput of the GF(2^16) butterfly (rs16_gf.hpp mul_xor +
// XOR) with the table in VGPRs, 16 rows per thread, at a given number of
// waves per SIMD.  Reports cycles per wave-butterfly at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../reed-solomon-16_amd/csrc/rs16_gf.hpp"
using namespace rs16;
// mul_xor with the selectors of L and H taken by two 64-bit shifts of the
// (L, H) pair instead of four 32-bit ones (bits shifted in from H land in
// L's top bits, which the byte masks clear)
RS16_HD void mul_xor64(uint32_t& xL, uint32_t& xH, uint32_t yL, uint32_t yH, const uint32_t* t) {
    const uint64_t y = ((uint64_t)yH << 32) | yL;
    uint64_t a, b;  // (asm: the compiler would narrow the shifts back to 32 bits)
#if defined(__HIP_DEVICE_COMPILE__)
    asm("v_lshrrev_b64 %0, 3, %1" : "=v"(a) : "v"(y));
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(b) : "v"(y));
#else
    a = y >> 3, b = y >> 6;
#endif
    const uint32_t s0 = yL & 0x07070707u, s3 = yH & 0x07070707u;
    const uint32_t s1 = (uint32_t)a & 0x07070707u, s4 = (uint32_t)(a >> 32) & 0x07070707u;
    const uint32_t s2 = (uint32_t)b & 0x03030303u, s5 = (uint32_t)(b >> 32) & 0x03030303u;
    const uint32_t l0 = perm(t[1], t[0], s0), h0 = perm(t[3], t[2], s0);
    const uint32_t l1 = perm(t[5], t[4], s1), h1 = perm(t[7], t[6], s1);
    const uint32_t l3 = perm(t[9], t[8], s3), h3 = perm(t[11], t[10], s3);
    const uint32_t l4 = perm(t[13], t[12], s4), h4 = perm(t[15], t[14], s4);
    const uint32_t l2 = perm(t[16], t[16], s2), h2 = perm(t[17], t[17], s2);
    const uint32_t l5 = perm(t[18], t[18], s5), h5 = perm(t[19], t[19], s5);
    xL = xor3(xor3(xL, l0, l1), xor3(l2, l3, l4), l5);
    xH = xor3(xor3(xH, h0, h1), xor3(h2, h3, h4), h5);
}
// the same multiply with its three instruction classes kept apart for the
// scheduler (sched_barrier): selector ops, then the 12 perms, then the XOR
// tree -- so that a wave issues long runs of one class
RS16_HD void mul_xor64g(uint32_t& xL, uint32_t& xH, uint32_t yL, uint32_t yH, const uint32_t* t) {
    const uint64_t y = ((uint64_t)yH << 32) | yL;
    uint64_t a, b;
#if defined(__HIP_DEVICE_COMPILE__)
    asm("v_lshrrev_b64 %0, 3, %1" : "=v"(a) : "v"(y));
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(b) : "v"(y));
#else
    a = y >> 3, b = y >> 6;
#endif
    const uint32_t s0 = yL & 0x07070707u, s3 = yH & 0x07070707u;
    const uint32_t s1 = (uint32_t)a & 0x07070707u, s4 = (uint32_t)(a >> 32) & 0x07070707u;
    const uint32_t s2 = (uint32_t)b & 0x03030303u, s5 = (uint32_t)(b >> 32) & 0x03030303u;
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
#endif
    const uint32_t l0 = perm(t[1], t[0], s0), h0 = perm(t[3], t[2], s0);
    const uint32_t l1 = perm(t[5], t[4], s1), h1 = perm(t[7], t[6], s1);
    const uint32_t l3 = perm(t[9], t[8], s3), h3 = perm(t[11], t[10], s3);
    const uint32_t l4 = perm(t[13], t[12], s4), h4 = perm(t[15], t[14], s4);
    const uint32_t l2 = perm(t[16], t[16], s2), h2 = perm(t[17], t[17], s2);
    const uint32_t l5 = perm(t[18], t[18], s5), h5 = perm(t[19], t[19], s5);
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
#endif
    xL = xor3(xor3(xL, l0, l1), xor3(l2, l3, l4), l5);
    xH = xor3(xor3(xH, h0, h1), xor3(h2, h3, h4), h5);
}
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
                } else if (MODE == 2) {  // FFT butterfly, 64-bit selector shifts
                    mul_xor64(L[m], H[m], L[m2], H[m2], t);
                    L[m2] ^= L[m]; H[m2] ^= H[m];
                } else if (MODE == 3) {  // the same, instruction classes grouped
                    mul_xor64g(L[m], H[m], L[m2], H[m2], t);
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
        float ms2 = run<2>(d, tab, blocks);
        const double g2 = g_ghz;
        float ms3 = run<3>(d, tab, blocks);
        const double g3 = g_ghz;
        (void)ms1;
        printf("waves/SIMD %d: FFT %.3f ms @ %.2f GHz (%.1f cyc/wave-bfly/SIMD = %.2f per instr of 30)  IFFT %.3f ms @ %.2f GHz (%.1f)\n",
               wps, ms0, g0, ms0 * 1e-3 * g0 * 1e9 * 1024 / bf, ms0 * 1e-3 * g0 * 1e9 * 1024 / bf / 30, ms1b, g1,
               ms1b * 1e-3 * g1 * 1e9 * 1024 / bf);
        printf("            FFT with 64-bit selector shifts %.3f ms @ %.2f GHz (%.1f cyc/wave-bfly/SIMD)\n", ms2, g2,
               ms2 * 1e-3 * g2 * 1e9 * 1024 / bf);
        printf("            FFT, 64-bit shifts, classes grouped %.3f ms @ %.2f GHz (%.1f cyc/wave-bfly/SIMD)\n", ms3, g3,
               ms3 * 1e-3 * g3 * 1e9 * 1024 / bf);
    }
    return 0;
}
