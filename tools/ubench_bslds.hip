// Microbenchmark: the layout-B half of the two-direction pass done bit-sliced
// in LDS.  A tile of 256 rows x 32 quads (128
// elements = 4 chunks of 32 per row) lives in LDS as bit-planes, plane-major
// (plane p of chunk x at T[p * 1024 + x], x = row * 4 + chunk: consecutive
// lanes read consecutive dwords).  Row = set + 16 m (set = tile bits 0-3,
// m = bits 4-7).  8 layers (IFFT on m bits 0..3, FFT on m bits 3..0); a layer
// is 512 butterfly tasks of 32 element pairs, 2 per lane of a 4-wave
// workgroup; the twiddle of a task is uniform per wave (64 tasks = 16 sets x
// 4 chunks of one m pair share it).  Multiply: polynomial basis 0x1002D,
// a ^= b * c as XOR over bit pairs of c of b * x^i (uniform branches), as
// tools/ubench_bitslice.hip.  The byte <-> bit-plane transposes and Cantor
// <-> polynomial basis changes at entry / exit are modelled as CONV
// single-rate ops per chunk each way.  Timing only (the data is arbitrary).
//
// Reported: cycles per tile per CU for the 8 layers (+ conversions), against
// the v_perm baseline of the same 8 layers: 8 x 1851 = 14.8 k CU-cycles per
// tile (64 wave-quad-butterflies per layer x 115.7 cycles / 4 SIMDs,
// profiles/r03_ubench_bfly.txt).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#ifndef CONV
#define CONV 150  // single-rate ops per 32-element chunk per conversion direction
#endif

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// a ^= y * c (polynomial basis 0x1002D, bit-sliced: plane p = bit p of 32 elements)
__device__ __forceinline__ void mul_add(uint32_t (&a)[16], const uint32_t (&x)[16], uint32_t c) {
    uint32_t y[16];
#pragma unroll
    for (int p = 0; p < 16; p++) y[p] = x[p];
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
        uint32_t z[16];  // z = y * x (register renaming + 3 XORs)
        z[0] = y[15];
#pragma unroll
        for (int p = 1; p < 16; p++) z[p] = y[p - 1];
        z[2] ^= y[15];
        z[3] ^= y[15];
        z[5] ^= y[15];
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
            y[2] ^= z[15];
            y[3] ^= z[15];
            y[5] ^= z[15];
        }
    }
}

__device__ __forceinline__ void conv(uint32_t (&v)[16], uint32_t k) {
    // stand-in for a transpose + basis change: CONV dependent-free single-rate ops
#pragma unroll
    for (int i = 0; i < CONV; i++) v[i & 15] = xor3(v[i & 15], v[(i + 5) & 15], v[(i + 11) & 15] + (i == 0 ? k : 0));
}

__global__ void __launch_bounds__(256, 2) bslds(uint32_t* out, const uint32_t* tw, int reps, uint64_t* clk) {
    extern __shared__ uint32_t T[];  // 16 planes x 1024 chunks (64 KiB)
    const uint32_t t = threadIdx.x;
    for (int i = 0; i < 64; i++) T[i * 256 + t] = (t + 1) * 2654435761u ^ (i * 40503u) ^ blockIdx.x;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < reps; rep++) {
        // conversion in: the lane's 4 chunks (byte form -> planes, Cantor -> polynomial)
#pragma unroll 1
        for (int j = 0; j < 4; j++) {
            const uint32_t x = t + 256u * j;
            uint32_t v[16];
#pragma unroll
            for (int p = 0; p < 16; p++) v[p] = T[p * 1024 + x];
            conv(v, x);
#pragma unroll
            for (int p = 0; p < 16; p++) T[p * 1024 + x] = v[p];
        }
        __syncthreads();
#pragma unroll 1
        for (int l = 0; l < 8; l++) {
            const int j = l < 4 ? l : 7 - l;  // m bit of the layer
            const bool fft = l >= 4;
#pragma unroll 1
            for (int task = 0; task < 2; task++) {
                const uint32_t tid = task * 256 + t;
                const uint32_t mp = __builtin_amdgcn_readfirstlane(tid >> 6);  // m pair: uniform per wave
                const uint32_t q = tid & 63, set = q >> 2, chunk = q & 3;
                const uint32_t ma = ((mp >> j) << (j + 1)) | (mp & ((1u << j) - 1)), mb = ma + (1u << j);
                const uint32_t xa = (set + 16 * ma) * 4 + chunk, xb = (set + 16 * mb) * 4 + chunk;
                const uint32_t c = __builtin_amdgcn_readfirstlane(tw[(l * 8 + (mp >> j) + rep) & 4095]);
                uint32_t a[16], b[16];
#pragma unroll
                for (int p = 0; p < 16; p++) {
                    a[p] = T[p * 1024 + xa];
                    b[p] = T[p * 1024 + xb];
                }
                if (fft) {
                    mul_add(a, b, c);
#pragma unroll
                    for (int p = 0; p < 16; p++) b[p] ^= a[p];
                } else {
#pragma unroll
                    for (int p = 0; p < 16; p++) b[p] ^= a[p];
                    mul_add(a, b, c);
                }
#pragma unroll
                for (int p = 0; p < 16; p++) {
                    T[p * 1024 + xa] = a[p];
                    T[p * 1024 + xb] = b[p];
                }
            }
            __syncthreads();
        }
        // conversion out
#pragma unroll 1
        for (int j = 0; j < 4; j++) {
            const uint32_t x = t + 256u * j;
            uint32_t v[16];
#pragma unroll
            for (int p = 0; p < 16; p++) v[p] = T[p * 1024 + x];
            conv(v, x ^ 7u);
#pragma unroll
            for (int p = 0; p < 16; p++) T[p * 1024 + x] = v[p];
        }
        __syncthreads();
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
    for (int i = 0; i < 64; i++) acc ^= T[i * 256 + t];
    out[blockIdx.x * 256 + t] = acc;
    if (t == 0) clk[blockIdx.x] = t1 - t0;
}

int main() {
    uint32_t *d, *tw;
    uint64_t* clk;
    const int blocks = 512, reps = 20;  // 2 workgroups per CU
    (void)hipMalloc(&d, (size_t)blocks * 256 * 4);
    (void)hipMalloc(&tw, 4096 * 4);
    (void)hipMalloc(&clk, blocks * 8);
    uint32_t h[4096];
    uint32_t s = 12345;
    for (int i = 0; i < 4096; i++) {
        s = s * 1103515245u + 12345u;
        h[i] = (s >> 8) & 0xFFFF;
    }
    (void)hipMemcpy(tw, h, sizeof h, hipMemcpyHostToDevice);
    (void)hipFuncSetAttribute((const void*)bslds, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms = 0;
    for (int pass = 0; pass < 2; pass++) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(bslds, dim3(blocks), dim3(256), 65536, 0, d, tw, reps, clk);
        (void)hipEventRecord(e1, 0);
        (void)hipDeviceSynchronize();
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    uint64_t hc[blocks];
    (void)hipMemcpy(hc, clk, sizeof hc, hipMemcpyDeviceToHost);
    double sum = 0;
    for (int i = 0; i < blocks; i++) sum += (double)hc[i];
    const double per_wg = sum / blocks / reps;  // workgroup cycles per tile (2 workgroups share a CU)
    printf("bit-sliced LDS layout-B region (8 layers + 2 x %d conversion ops per chunk): %.0f cycles per tile "
           "per workgroup, %.0f CU-cycles per tile (2 per CU) vs v_perm 14808\n",
           CONV, per_wg, per_wg / 2);
    // wall clock: 512 workgroups on 256 CUs at 2 per CU = one wave of workgroups; 2.4 GHz
    printf("  event time %.3f ms -> %.0f CU-cycles per tile at 2.4 GHz\n", ms, ms * 1e-3 * 2.4e9 / reps / 2);
    return 0;
}
