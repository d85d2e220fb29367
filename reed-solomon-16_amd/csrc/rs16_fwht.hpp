// rs16_fwht.hpp -- the 256-point FWHT in Z/65535 by one wave (device code
// shared by the eval_poly kernels, the decode passes and the column codec):
// the last H_lo of eval_poly (src/engine.rs:207-218; add/sub mod 65535 as
// NoSimd::fwht_private, src/engine/engine_nosimd.rs:153-183).
#pragma once
#include "rs16_gf.hpp"

namespace rs16 {

// x from lane (lane ^ D) of the wave, through DPP where one or two lane
// permutes do it (no LDS), ds_swizzle for 16, ds_bpermute for 32.
template <int D> __device__ __forceinline__ int xshfl(int x) {
    if constexpr (D == 1) return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    if constexpr (D == 2) return __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    if constexpr (D == 4)  // row_half_mirror (i -> 7 - i), then quad_perm [3,2,1,0]: i -> i ^ 4
        return __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false), 0x1B, 0xF, 0xF, false);
    if constexpr (D == 8) return __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, false);  // row_ror:8
    if constexpr (D == 16) return __builtin_amdgcn_ds_swizzle(x, 0x401F);              // xor 16 within 32
    if constexpr (D == 32) return __shfl_xor(x, 32);
    return x;
}
// 256-point FWHT in Z/65535 by one wave in registers: lane l holds
// v[j] = x[l + 64 j]; distances 1..32 are lane pairs (shuffles), 64 and 128
// register pairs.  No barriers.  (Residues as fwht256_lds; consumers of the
// decode's erasure logs treat 65535 and 0 alike, exp[65535] == exp[0].)
__device__ __forceinline__ void fwht256_wave(uint32_t (&v)[4]) {
    const uint32_t lane = threadIdx.x & 63;
    (void)lane;
#define RS16_L(D)                                                               \
    {                                                                           \
        const bool hi = (threadIdx.x & (D)) != 0;                               \
        _Pragma("unroll") for (int j = 0; j < 4; j++) {                         \
            const uint32_t p = (uint32_t)xshfl<(D)>((int)v[j]);                 \
            v[j] = hi ? sub_mod(p, v[j]) : add_mod(v[j], p);                    \
        }                                                                       \
    }
    RS16_L(1) RS16_L(2) RS16_L(4) RS16_L(8) RS16_L(16) RS16_L(32)
#undef RS16_L
    const uint32_t a = add_mod(v[0], v[1]), b = sub_mod(v[0], v[1]);
    const uint32_t c = add_mod(v[2], v[3]), d = sub_mod(v[2], v[3]);
    v[0] = add_mod(a, c);
    v[2] = sub_mod(a, c);
    v[1] = add_mod(b, d);
    v[3] = sub_mod(b, d);
}

}  // namespace rs16
