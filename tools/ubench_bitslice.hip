// Microbenchmark: bit-sliced GF(2^16) butterflies (16 bit-planes of 32
// elements per lane, polynomial basis 0x1002D, wave-uniform twiddle c):
//   a ^= b * c  computed as XOR over set bits i of c of (b * alpha^i),
// with uniform branches on pairs of bits of c.  Compare cycles per
// 32-element butterfly with the v_perm path (ubench_bfly: per 4 elements).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITER 64
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
template <int PAIR>
__device__ __forceinline__ void mul_add(uint32_t (&a)[16], const uint32_t (&x)[16], uint32_t c) {
    uint32_t y[16];
#pragma unroll
    for (int p = 0; p < 16; p++) y[p] = x[p];
    if (PAIR) {
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            uint32_t z[16];
            // z = y * alpha
            z[0] = y[15];
#pragma unroll
            for (int p = 1; p < 16; p++) z[p] = y[p - 1];
            z[2] ^= y[15]; z[3] ^= y[15]; z[5] ^= y[15];
            const uint32_t bits = (c >> i) & 3u;
            if (bits == 1) {
#pragma unroll
                for (int p = 0; p < 16; p++) a[p] ^= y[p];
            } else if (bits == 2) {
#pragma unroll
                for (int p = 0; p < 16; p++) a[p] ^= z[p];
            } else if (bits == 3) {
#pragma unroll
                for (int p = 0; p < 16; p++) a[p] = xor3(a[p], y[p], z[p]);
            }
            if (i + 2 < 16) {
                y[0] = z[15];
#pragma unroll
                for (int p = 1; p < 16; p++) y[p] = z[p - 1];
                y[2] ^= z[15]; y[3] ^= z[15]; y[5] ^= z[15];
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if ((c >> i) & 1u) {
#pragma unroll
                for (int p = 0; p < 16; p++) a[p] ^= y[p];
            }
            const uint32_t t = y[15];
#pragma unroll
            for (int p = 15; p > 0; p--) y[p] = y[p - 1];
            y[0] = t; y[2] ^= t; y[3] ^= t; y[5] ^= t;
        }
    }
}
template <int PAIR>
__global__ void __launch_bounds__(256) k(uint32_t* out, const uint32_t* tw, uint32_t seed) {
    uint32_t r[4][16];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int p = 0; p < 16; p++) r[i][p] = seed * (threadIdx.x + 16 * i + p + 1);
    for (int it = 0; it < ITER; it++) {
        const uint32_t* t = tw + ((it * 4 + blockIdx.x) & 1023) * 4;
        const uint32_t c0 = __builtin_amdgcn_readfirstlane(t[0]), c1 = __builtin_amdgcn_readfirstlane(t[1]);
        const uint32_t c2 = __builtin_amdgcn_readfirstlane(t[2]);
        // radix-4 FFT block: layer d=2 (pairs 0-2, 1-3, twiddle c0), layer d=1 (0-1 c1, 2-3 c2)
        mul_add<PAIR>(r[0], r[2], c0);
#pragma unroll
        for (int p = 0; p < 16; p++) r[2][p] ^= r[0][p];
        mul_add<PAIR>(r[1], r[3], c0);
#pragma unroll
        for (int p = 0; p < 16; p++) r[3][p] ^= r[1][p];
        mul_add<PAIR>(r[0], r[1], c1);
#pragma unroll
        for (int p = 0; p < 16; p++) r[1][p] ^= r[0][p];
        mul_add<PAIR>(r[2], r[3], c2);
#pragma unroll
        for (int p = 0; p < 16; p++) r[3][p] ^= r[2][p];
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int p = 0; p < 16; p++) acc ^= r[i][p];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
template <int PAIR> float run(uint32_t* d, const uint32_t* tw, int blocks) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    k<PAIR><<<blocks, 256>>>(d, tw, 1);
    (void)hipEventRecord(a);
    k<PAIR><<<blocks, 256>>>(d, tw, 1);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}
int main() {
    uint32_t *d, *tw;
    (void)hipMalloc(&d, 256 * 8 * 256 * 4);
    (void)hipMalloc(&tw, 4096 * 4);
    uint32_t h[4096];
    uint32_t s = 12345;
    for (int i = 0; i < 4096; i++) { s = s * 1103515245u + 12345u; h[i] = (s >> 8) & 0xFFFF; }
    (void)hipMemcpy(tw, h, sizeof h, hipMemcpyHostToDevice);
    for (int wps = 1; wps <= 4; wps *= 2) {
        int blocks = 256 * wps;
        float m0 = run<0>(d, tw, blocks), m1 = run<1>(d, tw, blocks);
        double bf = (double)blocks * 4 * ITER * 4;  // wave-butterflies (32 elements per lane)
        printf("waves/SIMD %d: single-bit %.3f ms (%.0f cyc/wave-bfly of 32 el)  bit-pairs %.3f ms (%.0f)\n", wps, m0,
               m0 * 1e-3 * 2.4e9 * 1024 / bf, m1, m1 * 1e-3 * 2.4e9 * 1024 / bf);
    }
    return 0;
}
