// rs16_colops.hpp -- in-wave radix-4 building blocks of the column codec
// (rs16_col.hip) and of the one-wave-per-quad-column tile kernels
// (rs16_pass.hip): a thread holds 4 rows of one quad column (the rows of a
// block over two row bits B0, B1 inserted into its lane index), the two
// layers of a block are butterflies between its registers, and the row bits
// of registers and lanes trade places inside the wave between blocks.
#pragma once
#include "rs16_internal.hpp"
#include "rs16_fwht.hpp"

namespace rs16 {
namespace colops {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// LDS index of row r in the image (uint2 units): bits 5 and 6 are XORed
// into bits 0-4 so that the 32 lanes of a b64 access hit 32 distinct bank
// pairs for both LDS exchanges' row patterns.
__device__ __forceinline__ uint32_t swz(uint32_t r) {
    return r ^ (((r >> 5) & 1u) * 5u) ^ (((r >> 6) & 1u) * 26u);
}

// The thread's row for register m of a block over row bits (B0, B1).
template <int B0, int B1> __device__ __forceinline__ uint32_t brow(uint32_t t, int m) {
    const uint32_t lo = t & ((1u << B0) - 1u);
    const uint32_t rest = t >> B0;
    const uint32_t mid = rest & ((1u << (B1 - B0 - 1)) - 1u);
    const uint32_t hi = rest >> (B1 - B0 - 1);
    return lo | (mid << (B0 + 1)) | (hi << (B1 + 1)) | ((uint32_t)(m & 1) << B0) | ((uint32_t)(m >> 1) << B1);
}

__device__ __forceinline__ void lds_table(uint32_t (&t)[20], const uint8_t* smem, uint32_t off) {
    const u32x4* p = (const u32x4*)(smem + off);
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const u32x4 v = p[i];
        t[4 * i] = v.x;
        t[4 * i + 1] = v.y;
        t[4 * i + 2] = v.z;
        t[4 * i + 3] = v.w;
    }
}
__device__ __forceinline__ void glb_table(uint32_t (&t)[20], const uint32_t* tabs, uint32_t entry) {
    const u32x4* p = (const u32x4*)(tabs + (size_t)entry * TAB_DWORDS);
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const u32x4 v = p[i];
        t[4 * i] = v.x;
        t[4 * i + 1] = v.y;
        t[4 * i + 2] = v.z;
        t[4 * i + 3] = v.w;
    }
}

// LDS-DMA copy of `bytes` (a multiple of 16) from src to the LDS at dst by
// all NT threads: instruction i of wave w moves bytes [(i NT + 64 w) 16, +1 KiB)
// (the LDS destination of global_load_lds is the wave's base + 16 lane).
typedef __attribute__((address_space(3))) void* lds_vp;
typedef __attribute__((address_space(1))) const void* glb_vp;
template <int NT>
__device__ __forceinline__ void dma_copy_step(const uint8_t* src, uint8_t* dst, uint32_t bytes, uint32_t i) {
    const uint32_t t = threadIdx.x, w = t >> 6;
    const uint32_t c = i * NT + t;
    if (c * 16 < bytes)
        __builtin_amdgcn_global_load_lds((glb_vp)(src + c * 16), (lds_vp)(dst + (i * NT + 64 * w) * 16), 16, 0, 0);
}
// (sizes known at compile time: fully unrolled)
template <int NT>
__device__ __forceinline__ void dma_copy(const uint8_t* src, uint8_t* dst, uint32_t bytes) {
#pragma unroll
    for (uint32_t i = 0; i * NT * 16 < bytes; i++) dma_copy_step<NT>(src, dst, bytes, i);
}
// (sizes known at run time only, e.g. mid_direct_kernel's nout x 2^hi
// tables: a plain loop -- a full-unroll request cannot be honoured there)
template <int NT>
__device__ __forceinline__ void dma_copy_rt(const uint8_t* src, uint8_t* dst, uint32_t bytes) {
    for (uint32_t i = 0; i * NT * 16 < bytes; i++) dma_copy_step<NT>(src, dst, bytes, i);
}

// Trade register bit RB (register pairs m, m | 2^RB) with lane bit LB of
// the wave: afterwards register bit RB holds the row bit lane bit LB held,
// and the other way round (lane with LB = 0 takes the partner's m into its
// m | 2^RB, lane with LB = 1 the partner's m | 2^RB into its m).
template <int RB, int LB> __device__ __forceinline__ void swap_bit(uint32_t (&X)[4]) {
#pragma unroll
    for (int m = 0; m < 4; m++) {
        if (m & (1 << RB)) continue;
        const int m1 = m | (1 << RB);
        if constexpr (LB == 4 || LB == 5) {
            // v_permlane16_swap: odd 16-lane rows of the first operand <-> even
            // rows of the second; v_permlane32_swap: upper 32 lanes <-> lower 32
            const auto r = LB == 4 ? __builtin_amdgcn_permlane16_swap(X[m], X[m1], false, false)
                                   : __builtin_amdgcn_permlane32_swap(X[m], X[m1], false, false);
            X[m] = r[0];
            X[m1] = r[1];
        } else {
            const bool hi = (threadIdx.x >> LB) & 1u;
            const uint32_t u = (uint32_t)xshfl<(1 << LB)>((int)X[m]);   // partner's m
            const uint32_t v = (uint32_t)xshfl<(1 << LB)>((int)X[m1]);  // partner's m | 2^RB
            X[m1] = hi ? X[m1] : u;
            X[m] = hi ? v : X[m];
        }
    }
}
// Block (B0, B1) -> block (C0, C1) inside the wave: register bits 0 / 1
// trade places with the lane bits that hold row bits C0 / C1.
template <int LB0, int LB1> __device__ __forceinline__ void wave_exchange(uint32_t (&XL)[4], uint32_t (&XH)[4]) {
    swap_bit<0, LB0>(XL);
    swap_bit<0, LB0>(XH);
    swap_bit<1, LB1>(XL);
    swap_bit<1, LB1>(XH);
}

// The (0, 1) block's tables, from the image (table g at g x 80 bytes).
__device__ __forceinline__ void img_table(uint32_t (&t)[20], const uint8_t* img, uint32_t g) {
    const u32x4* p = (const u32x4*)(img + (size_t)g * 80);
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const u32x4 v = p[i];
        t[4 * i] = v.x;
        t[4 * i + 1] = v.y;
        t[4 * i + 2] = v.z;
        t[4 * i + 3] = v.w;
    }
}
// The twiddle tables of one block: the layers on row bits B0 (if D0) and B1
// (if D1) of the thread's 4 rows (register m <-> bit B0 = m & 1, bit B1 =
// m >> 1).  Read from LDS one block ahead of their use.
struct BlockTabs {
    uint32_t w0[20], w2[20], w1[20];  // layer B0: pairs (0,1), (2,3); layer B1: pairs (0,2), (1,3)
};
template <bool FFT, bool D0, bool D1>
__device__ __forceinline__ void compute(uint32_t (&XL)[4], uint32_t (&XH)[4], const BlockTabs& w) {
    auto lay0 = [&]() {
        if (FFT) {
            mul_xor(XL[0], XH[0], XL[1], XH[1], w.w0);
            XL[1] ^= XL[0], XH[1] ^= XH[0];
            mul_xor(XL[2], XH[2], XL[3], XH[3], w.w2);
            XL[3] ^= XL[2], XH[3] ^= XH[2];
        } else {
            XL[1] ^= XL[0], XH[1] ^= XH[0];
            mul_xor(XL[0], XH[0], XL[1], XH[1], w.w0);
            XL[3] ^= XL[2], XH[3] ^= XH[2];
            mul_xor(XL[2], XH[2], XL[3], XH[3], w.w2);
        }
    };
    auto lay1 = [&]() {
        if (FFT) {
            mul_xor(XL[0], XH[0], XL[2], XH[2], w.w1);
            XL[2] ^= XL[0], XH[2] ^= XH[0];
            mul_xor(XL[1], XH[1], XL[3], XH[3], w.w1);
            XL[3] ^= XL[1], XH[3] ^= XH[1];
        } else {
            XL[2] ^= XL[0], XH[2] ^= XH[0];
            mul_xor(XL[0], XH[0], XL[2], XH[2], w.w1);
            XL[3] ^= XL[1], XH[3] ^= XH[1];
            mul_xor(XL[1], XH[1], XL[3], XH[3], w.w1);
        }
    };
    if (FFT) {
        if (D1) lay1();
        if (D0) lay0();
    } else {
        if (D0) lay0();
        if (D1) lay1();
    }
}

}  // namespace colops
}  // namespace rs16
