// Microbenchmark: VALU throughput of the instructions the GF multiply uses
// (v_perm_b32, v_bitop3_b32, v_xor_b32, v_and_b32, v_lshrrev_b32) on gfx950.
// Each wave runs ITER x 16 independent instructions of one kind.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 4096
template <int KIND>
__global__ void __launch_bounds__(256) k(unsigned* out, unsigned seed) {
    unsigned v[16];
    for (int i = 0; i < 16; i++) v[i] = seed * (threadIdx.x + i + 1);
    unsigned s = seed ^ 0x5bd1e995u, t = seed + 77;
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if (KIND == 0) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(s), "v"(t));
            if (KIND == 1) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(v[i]) : "v"(s), "v"(t));
            if (KIND == 2) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(s));
            if (KIND == 3) asm volatile("v_and_b32 %0, %1, %0" : "+v"(v[i]) : "v"(s));
            if (KIND == 4) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(v[i]));
        }
    }
    unsigned r = 0;
    for (int i = 0; i < 16; i++) r ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int KIND> float run(unsigned* d, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k<KIND><<<blocks, 256>>>(d, 1);
    hipEventRecord(a);
    k<KIND><<<blocks, 256>>>(d, 1);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
}
int main() {
    int cus = 256, blocks = cus * 8;  // 8 x 4 waves per CU = 8 waves/SIMD
    unsigned* d; hipMalloc(&d, blocks * 256 * 4);
    const char* names[] = {"v_perm_b32", "v_bitop3_b32", "v_xor_b32", "v_and_b32", "v_lshrrev_b32"};
    float ms[5] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks), run<4>(d, blocks)};
    for (int i = 0; i < 5; i++) {
        double wave_instr = (double)blocks * 4 * ITER * 16;
        double per_cu_per_ns = wave_instr / cus / (ms[i] * 1e6);
        printf("%-14s %8.3f ms  %.3f wave-instr/ns/CU  (= %.2f cycles per wave-instr per SIMD at 2.4 GHz)\n", names[i],
               ms[i], per_cu_per_ns, 4.0 * 2.4 / per_cu_per_ns);
    }
    return 0;
}
