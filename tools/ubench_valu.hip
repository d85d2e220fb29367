// Microbenchmark: VALU issue rate of the instructions the GF(2^16) multiply
// uses (v_perm_b32, v_bitop3_b32, v_xor_b32, v_and_b32, v_lshrrev_b32), with
// v_fma_f32 / v_add_u32 for reference, and v_lshrrev_b64 (one shift of an
// (L, H) dword pair), at 1, 2, 4 and 8 waves per SIMD.
//
// Every wave runs ITER x 16 independent instructions of one kind (16 chains,
// no dependency stalls).  Clock: wave 0 of block 0 reads s_memtime (shader
// clock) and s_memrealtime (100 MHz) around its loop, so cycles are counted
// at the clock the chip actually ran, not an assumed 2.4 GHz.
//
// Output: cycles per wave64 instruction per SIMD = SIMD cycles / (waves per
// SIMD x instructions per wave), from the kernel's hipEvent duration and the
// measured clock.  2.0 = a SIMD-32 issuing one wave64 instruction every 2
// cycles (MI355X_MICROARCH.md "SIMD-32"), 4.0 = one every 4 cycles.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 2048
template <int KIND>
__global__ void __launch_bounds__(256) k(unsigned* out, unsigned long long* clk, unsigned seed) {
    unsigned v[16];
    for (int i = 0; i < 16; i++) v[i] = seed * (threadIdx.x + i + 1);
    unsigned s = seed ^ 0x5bd1e995u, t = seed + 77;
    unsigned long long w[8];
    for (int i = 0; i < 8; i++) w[i] = ((unsigned long long)v[2 * i + 1] << 32) | v[2 * i];
    float f[16];
    for (int i = 0; i < 16; i++) f[i] = (float)v[i] * 1e-9f;
    const float fa = 1.0001f, fb = 0.5f;
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if (KIND == 0) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(s), "v"(t));
            if (KIND == 1) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(v[i]) : "v"(s), "v"(t));
            if (KIND == 2) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(s));
            if (KIND == 3) asm volatile("v_and_b32 %0, %1, %0" : "+v"(v[i]) : "v"(s));
            if (KIND == 4) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(v[i]));
            if (KIND == 5) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f[i]) : "v"(fa), "v"(fb));
            if (KIND == 6) asm volatile("v_add_u32 %0, %1, %0" : "+v"(v[i]) : "v"(s));
            if (KIND == 7) asm volatile("v_and_b32 %0, 0x7070707, %0" : "+v"(v[i]));
            if (KIND == 8 && (i & 1) == 0) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(w[i >> 1]));
            if (KIND == 9 && (i & 1) == 0) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(v[i]) : "v"(s));
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    unsigned r = 0;
    for (int i = 0; i < 16; i++) r ^= v[i] ^ __float_as_uint(f[i]) ^ (unsigned)(w[i >> 1] >> (32 * (i & 1)));
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int KIND> void run(unsigned* d, unsigned long long* dclk, int cus, int wps, const char* name) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int blocks = cus * wps;  // 256-thread blocks: one wave on each of the CU's 4 SIMDs
    k<KIND><<<blocks, 256>>>(d, dclk, 1);
    (void)hipEventRecord(a);
    k<KIND><<<blocks, 256>>>(d, dclk, 1);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long clk[2];
    (void)hipMemcpy(clk, dclk, sizeof clk, hipMemcpyDeviceToHost);
    const double ghz = clk[1] ? (double)clk[0] / ((double)clk[1] * 10.0) : 2.4;  // memrealtime: 100 MHz
    const double instr_per_wave = (double)ITER * (KIND == 8 || KIND == 9 ? 8 : 16);
    const double simd_cycles = ms * 1e-3 * ghz * 1e9;
    const double cpi = simd_cycles / (wps * instr_per_wave);
    printf("%-22s waves/SIMD %d  %8.3f ms  clock %.2f GHz  %.2f cycles per wave-instruction per SIMD\n", name, wps,
           ms, ghz, cpi);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
}
int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned* d;
    unsigned long long* dclk;
    (void)hipMalloc(&d, (size_t)cus * 8 * 256 * 4);
    (void)hipMalloc(&dclk, 16);
    printf("CUs %d\n", cus);
    for (int wps = 1; wps <= 8; wps *= 2) {
        run<0>(d, dclk, cus, wps, "v_perm_b32");
        run<1>(d, dclk, cus, wps, "v_bitop3_b32");
        run<2>(d, dclk, cus, wps, "v_xor_b32");
        run<3>(d, dclk, cus, wps, "v_and_b32 (vgpr)");
        run<7>(d, dclk, cus, wps, "v_and_b32 (literal)");
        run<4>(d, dclk, cus, wps, "v_lshrrev_b32");
        run<6>(d, dclk, cus, wps, "v_add_u32");
        run<5>(d, dclk, cus, wps, "v_fma_f32");
        run<8>(d, dclk, cus, wps, "v_lshrrev_b64 (x8)");
    }
    return 0;
}
