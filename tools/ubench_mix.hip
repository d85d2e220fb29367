// Microbenchmark: VALU issue cost of instruction mixes on gfx950, to model
// the GF(2^16) butterfly (rs16_gf.hpp): 12 v_perm_b32 + 6 v_bitop3_b32 + 12
// simple ops per 4-element butterfly.  Every pattern runs 16 independent
// chains per wave; 2, 4 and 8 waves per SIMD; cycles per wave-instruction per
// SIMD at the clock measured with s_memtime / s_memrealtime.
//   P0 perm, 3 distinct VGPR sources per instruction
//   P1 perm, hi pool byte source in an SGPR (wave-uniform table)
//   P2 bitop3 (xor3), 3 distinct VGPR sources
//   P3 xor, 2 distinct VGPR sources
//   P4 perm + xor alternating
//   P5 perm + 2 xor
//   P6 perm + bitop3 alternating
//   P7 the multiply of rs16_gf.hpp (mul_xor) with the table in VGPRs (per-lane)
//   P8 the same with the table wave-uniform (SGPR operands where the ISA allows)
//   P9 perm + and (literal mask) alternating
//   P10-P13 (round 6) grouped against interleaved perm / simple-op orders
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../reed-solomon-16_amd/csrc/rs16_gf.hpp"
using namespace rs16;
#define ITER 1024
template <int P>
__global__ void __launch_bounds__(256) k(unsigned* out, const unsigned* tab, unsigned long long* clk, unsigned seed) {
    unsigned v[16], a[16], b[16];
    for (int i = 0; i < 16; i++) {
        v[i] = seed * (threadIdx.x + i + 1);
        a[i] = v[i] * 0x9e3779b9u + i;
        b[i] = (v[i] ^ 0x5bd1e995u) & 0x07070707u;
    }
    unsigned t[20];
    for (int i = 0; i < 20; i++) t[i] = tab[(blockIdx.x & 7) * 32 + i] ^ (P == 7 ? threadIdx.x : 0u);
    if (P == 8)
        for (int i = 0; i < 20; i++) t[i] = __builtin_amdgcn_readfirstlane(t[i]);
    const unsigned su = __builtin_amdgcn_readfirstlane(seed * 77u);
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < ITER; it++) {
        if (P == 7 || P == 8) {
#pragma unroll
            for (int i = 0; i < 16; i += 2) mul_xor(v[i], v[i + 1], a[i], a[i + 1], t);
#pragma unroll
            for (int i = 0; i < 16; i++) a[i] ^= v[i];
            asm volatile("" ::: "memory");
            continue;
        }
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if (P == 0) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
            if (P == 1) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "s"(su), "v"(b[i]));
            if (P == 2) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
            if (P == 3) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(a[i]));
            if (P == 4) {
                if (i & 1) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(a[i]));
                else asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
            }
            if (P == 5) {
                if (i % 3) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(a[i]));
                else asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
            }
            if (P == 6) {
                if (i & 1) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
                else asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
            }
            if (P == 9) {
                if (i & 1) asm volatile("v_and_b32 %0, 0x7070707, %0" : "+v"(v[i]));
                else asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
            }
            if (P == 10) {  // 8 perms, then 8 xors
                if (i >= 8) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(a[i]));
                else asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
            }
            if (P == 11) {  // 4 perms, 4 xors, 4 perms, 4 xors
                if (i & 4) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(a[i]));
                else asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
            }
            if (P == 12) {  // 12 perms, 4 bitop3 (the multiply's 12 : 6 mix, grouped)
                if (i >= 12) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
                else asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
            }
            if (P == 13) {  // the same 12 : 4 mix interleaved (3 perms, 1 bitop3)
                if ((i & 3) == 3) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
                else asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a[i]), "v"(b[i]));
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    unsigned r = 0;
    for (int i = 0; i < 16; i++) r ^= v[i] ^ a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int P> void run(unsigned* d, const unsigned* tab, unsigned long long* dclk, int cus, int wps, const char* name,
                          double instr_per_iter) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int blocks = cus * wps;
    k<P><<<blocks, 256>>>(d, tab, dclk, 1);
    (void)hipEventRecord(a);
    k<P><<<blocks, 256>>>(d, tab, dclk, 1);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long clk[2];
    (void)hipMemcpy(clk, dclk, sizeof clk, hipMemcpyDeviceToHost);
    const double ghz = clk[1] ? (double)clk[0] / ((double)clk[1] * 10.0) : 2.4;
    const double simd_cycles = ms * 1e-3 * ghz * 1e9;
    const double per_iter = simd_cycles / (wps * (double)ITER);
    printf("%-34s waves/SIMD %d  %7.3f ms @ %.2f GHz  %7.1f cycles/iter  %.2f cycles/instr\n", name, wps, ms, ghz,
           per_iter, per_iter / instr_per_iter);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
}
int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *d, *tab;
    unsigned long long* dclk;
    (void)hipMalloc(&d, (size_t)cus * 8 * 256 * 4);
    (void)hipMalloc(&tab, 8 * 32 * 4);
    (void)hipMalloc(&dclk, 16);
    (void)hipMemset(tab, 0x5a, 8 * 32 * 4);
    for (int wps = 2; wps <= 8; wps *= 2) {
        run<0>(d, tab, dclk, cus, wps, "P0 perm (3 vgpr)", 16);
        run<1>(d, tab, dclk, cus, wps, "P1 perm (sgpr hi)", 16);
        run<2>(d, tab, dclk, cus, wps, "P2 bitop3 (3 vgpr)", 16);
        run<3>(d, tab, dclk, cus, wps, "P3 xor (2 vgpr)", 16);
        run<4>(d, tab, dclk, cus, wps, "P4 perm+xor", 16);
        run<5>(d, tab, dclk, cus, wps, "P5 perm+2xor", 16);
        run<6>(d, tab, dclk, cus, wps, "P6 perm+bitop3", 16);
        run<9>(d, tab, dclk, cus, wps, "P9 perm+and(lit)", 16);
        run<10>(d, tab, dclk, cus, wps, "P10 8 perm, then 8 xor", 16);
        run<11>(d, tab, dclk, cus, wps, "P11 4 perm, 4 xor (x2)", 16);
        run<12>(d, tab, dclk, cus, wps, "P12 12 perm, then 4 bitop3", 16);
        run<13>(d, tab, dclk, cus, wps, "P13 (3 perm, bitop3) x4", 16);
        run<7>(d, tab, dclk, cus, wps, "P7 mul_xor+xor (vgpr table)", 8 * 28 + 16);
        run<8>(d, tab, dclk, cus, wps, "P8 mul_xor+xor (uniform table)", 8 * 28 + 16);
    }
    return 0;
}
