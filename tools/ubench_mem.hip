// Microbenchmark: HBM copy of a 65536 x 1 KiB shard array with the access
// patterns of the pass kernels (tile = 256 rows x 32 quads, 512 threads,
// 16 rows per thread), to find the achievable rate of each pattern.
//   MODE 0: dword lo/hi loads+stores per quad, strided tile rows (DEC_MID)
//   MODE 1: same, contiguous tile rows (DEC_FIRST/LAST)
//   MODE 2: 16 B per lane row-major loads+stores, strided rows
//   MODE 3: MODE 0 + LDS exchange in 2 rounds (4 barriers)
//   MODE 4: dwordx2 (2 quads per lane, lo and hi), strided rows, 8 rows/thread
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int ROWS = 65536, S = 1024;
template <int MODE>
__global__ void __launch_bounds__(512) k(const uint8_t* __restrict__ in, uint8_t* __restrict__ out) {
    __shared__ uint2 img[256 * 16];
    const uint32_t nslab = 4;  // 1 KiB / 256 B
    const uint32_t tile = blockIdx.x / nslab, slab = blockIdx.x % nslab;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool strided = MODE != 1;
    auto row_of = [&](uint32_t kk) { return strided ? tile + (kk << 8) : tile * 256 + kk; };
    if (MODE == 0 || MODE == 1 || MODE == 3) {
        const uint32_t qt = lane & 31, s = w * 2 + (lane >> 5);
        const uint32_t Qg = slab * 32 + qt;
        const uint32_t off = (Qg >> 3) * 64 + (Qg & 7) * 4;
        uint32_t L[16], H[16];
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const uint8_t* p = in + (size_t)row_of((s << 4) + m) * S + off;
            L[m] = *(const uint32_t*)p;
            H[m] = *(const uint32_t*)(p + 32);
        }
        if (MODE == 3) {
            const uint32_t ql = qt & 15, rnd = qt >> 4;
            for (int r = 0; r < 2; r++) {
                if (rnd == r)
                    for (int m = 0; m < 16; m++) img[((s << 4) + m) * 16 + ql] = make_uint2(L[m], H[m]);
                __syncthreads();
                if (rnd == r)
                    for (int m = 0; m < 16; m++) {
                        uint2 v = img[(s + (m << 4)) * 16 + ql];
                        L[m] = v.x;
                        H[m] = v.y;
                    }
                __syncthreads();
            }
#pragma unroll
            for (int m = 0; m < 16; m++) {
                uint8_t* p = out + (size_t)row_of(s + (m << 4)) * S + off;
                *(uint32_t*)p = L[m];
                *(uint32_t*)(p + 32) = H[m];
            }
        } else {
#pragma unroll
            for (int m = 0; m < 16; m++) {
                uint8_t* p = out + (size_t)row_of((s << 4) + m) * S + off;
                *(uint32_t*)p = L[m];
                *(uint32_t*)(p + 32) = H[m];
            }
        }
    } else if (MODE == 2) {
        // 256 rows x 256 B = 4096 pieces of 16 B; 8 per thread
        uint4 v[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t piece = threadIdx.x + i * 512, r = piece >> 4, c = piece & 15;
            v[i] = *(const uint4*)(in + (size_t)row_of(r) * S + slab * 256 + c * 16);
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t piece = threadIdx.x + i * 512, r = piece >> 4, c = piece & 15;
            *(uint4*)(out + (size_t)row_of(r) * S + slab * 256 + c * 16) = v[i];
        }
    } else {
        // 2 quads per lane (dwordx2 lo + dwordx2 hi), 16 lanes per row set, 8 rows/thread
        const uint32_t qp = lane & 15, s = w * 4 + (lane >> 4);   // 32 row sets of 8 rows
        const uint32_t Qg = slab * 32 + qp * 2;
        const uint32_t off = (Qg >> 3) * 64 + (Qg & 7) * 4;
        uint2 L[8], H[8];
#pragma unroll
        for (int m = 0; m < 8; m++) {
            const uint8_t* p = in + (size_t)row_of((s << 3) + m) * S + off;
            L[m] = *(const uint2*)p;
            H[m] = *(const uint2*)(p + 32);
        }
#pragma unroll
        for (int m = 0; m < 8; m++) {
            uint8_t* p = out + (size_t)row_of((s << 3) + m) * S + off;
            *(uint2*)p = L[m];
            *(uint2*)(p + 32) = H[m];
        }
    }
}
template <int MODE> float run(const uint8_t* in, uint8_t* out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int grid = 256 * 4;
    k<MODE><<<grid, 512>>>(in, out);
    (void)hipEventRecord(a);
    for (int i = 0; i < 10; i++) k<MODE><<<grid, 512>>>(in, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 10;
}
int main() {
    uint8_t *in, *out;
    (void)hipMalloc(&in, (size_t)ROWS * S);
    (void)hipMalloc(&out, (size_t)ROWS * S);
    (void)hipMemset(in, 1, (size_t)ROWS * S);
    const char* names[] = {"dword lo/hi, strided rows", "dword lo/hi, contiguous rows", "16 B/lane, strided rows",
                           "dword + 2-round LDS exchange", "dwordx2 lo/hi (2 quads/lane)"};
    float ms[5] = {run<0>(in, out), run<1>(in, out), run<2>(in, out), run<3>(in, out), run<4>(in, out)};
    for (int i = 0; i < 5; i++)
        printf("%-32s %7.1f us  %6.0f GB/s (read+write)\n", names[i], ms[i] * 1e3, 2.0 * ROWS * S / (ms[i] * 1e-3) / 1e9);
    return 0;
}
