// rs16_gf.hpp -- GF(2^16) arithmetic for the MI355X engine (host + device).
//
// Element layout (reference src/algorithm.md:6-32): every 64-byte block of a
// shard holds 32 elements as 32 low bytes followed by 32 high bytes.  The GPU
// works on *quads*: quad q of a block = the 4 elements whose low bytes are
// the dword at byte 4q ("L") and whose high bytes are the dword at byte 32+4q
// ("H").  All FFT/IFFT/mul work is done on (L, H) dword pairs.
//
// Multiplication by a constant (reference: NoSimd::mul / mul_add with
// 4-bit nibble tables, src/engine/engine_nosimd.rs:65-79,105-119) is done
// here with CDNA's byte-permute instruction instead of table loads:
// v_perm_b32 selects 4 bytes out of an 8-byte pool using 4 per-byte 3-bit
// selectors, i.e. it is 4 lookups into an 8-entry byte table in one VALU op.
// Since x -> x*c is GF(2)-linear, x*c = XOR over bit groups of T_g[bits_g(x)].
// The 16 bits of an element are split into six groups: L[0:2], L[3:5],
// L[6:7], H[0:2], H[3:5], H[6:7]; each group has one table per output byte
// (lo / hi), 12 lookups per quad.  A product costs 6 selector extractions per
// dword pair, 12 v_perm and 4 v_bitop3 (3-input XOR), with no LDS traffic and
// no bank conflicts.
//
// Table entry layout (TAB_DWORDS dwords per log_m, see rs16_tables.cpp):
//   dword (g*2 + ob)*2 + h   g in 0..3 = {L0-2, L3-5, H0-2, H3-5},
//                            ob = output byte (0 lo, 1 hi), h = entries 0-3 / 4-7
//   dword 16 + gg*2 + ob     gg in 0..1 = {L6-7, H6-7} (4 entries, one dword)
// Entry index: log_m in 0..65535 uses reference `mul` semantics
// (tables::mul, src/engine/tables.rs:70-76; 65535 == 0 == multiply by 1);
// entry ZERO_ENTRY (65536) is the all-zero table used for the FFT/IFFT
// "no multiply" sentinel (log_m == GF_MODULUS in engine_naive.rs:64,116).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define RS16_HD __host__ __device__ __forceinline__
#else
#define RS16_HD inline
#endif

namespace rs16 {

constexpr uint32_t GF_ORDER = 65536;
constexpr uint32_t GF_MODULUS = 65535;
constexpr uint32_t ZERO_ENTRY = 65536;
constexpr uint32_t TAB_ENTRIES = 65537;
constexpr uint32_t TAB_DWORDS = 32;  // 128-byte stride: one cache line per constant

// v_perm_b32 semantics for selectors 0..7: byte i of the result is byte
// sel_i of the 64-bit value {hi:lo} (0-3 from lo, 4-7 from hi).
RS16_HD uint32_t perm_sw(uint32_t hi, uint32_t lo, uint32_t sel) {
    uint64_t pool = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; i++) {
        uint32_t s = (sel >> (8 * i)) & 0xFF;
        r |= (uint32_t)((pool >> (8 * s)) & 0xFF) << (8 * i);
    }
    return r;
}

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
#else
inline uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return perm_sw(hi, lo, sel); }
inline uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }
#endif

// (xL, xH) ^= (yL, yH) * c  where t points at the table entry of c.
RS16_HD void mul_xor(uint32_t& xL, uint32_t& xH, uint32_t yL, uint32_t yH, const uint32_t* t) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(RS16_SHIFT32)
    // The selectors of both dwords from two 64-bit shifts of the (L, H) pair
    // instead of four 32-bit ones: the bits H shifts into L's top land where
    // the byte masks clear them.  (As plain C the compiler narrows the shifts
    // back to 32 bits.)  tools/ubench_bfly: 117.7 -> 114.0 cycles per
    // wave-butterfly at 4 waves per SIMD (profiles/r06_ubench_bfly64.txt).
    const uint64_t y = ((uint64_t)yH << 32) | yL;
    uint64_t a, b;
    asm("v_lshrrev_b64 %0, 3, %1" : "=v"(a) : "v"(y));
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(b) : "v"(y));
    const uint32_t s0 = yL & 0x07070707u;
    const uint32_t s1 = (uint32_t)a & 0x07070707u;
    const uint32_t s2 = (uint32_t)b & 0x03030303u;
    const uint32_t s3 = yH & 0x07070707u;
    const uint32_t s4 = (uint32_t)(a >> 32) & 0x07070707u;
    const uint32_t s5 = (uint32_t)(b >> 32) & 0x03030303u;
#else
    const uint32_t s0 = yL & 0x07070707u;
    const uint32_t a = yL >> 3;
    const uint32_t s1 = a & 0x07070707u;
    const uint32_t s2 = (a >> 3) & 0x03030303u;
    const uint32_t s3 = yH & 0x07070707u;
    const uint32_t b = yH >> 3;
    const uint32_t s4 = b & 0x07070707u;
    const uint32_t s5 = (b >> 3) & 0x03030303u;
#endif
    const uint32_t l0 = perm(t[1], t[0], s0), h0 = perm(t[3], t[2], s0);
    const uint32_t l1 = perm(t[5], t[4], s1), h1 = perm(t[7], t[6], s1);
    const uint32_t l3 = perm(t[9], t[8], s3), h3 = perm(t[11], t[10], s3);
    const uint32_t l4 = perm(t[13], t[12], s4), h4 = perm(t[15], t[14], s4);
    const uint32_t l2 = perm(t[16], t[16], s2), h2 = perm(t[17], t[17], s2);
    const uint32_t l5 = perm(t[18], t[18], s5), h5 = perm(t[19], t[19], s5);
    xL = xor3(xor3(xL, l0, l1), xor3(l2, l3, l4), l5);
    xH = xor3(xor3(xH, h0, h1), xor3(h2, h3, h4), h5);
}

// Ones'-complement add/sub on logs (reference add_mod/sub_mod,
// src/engine.rs:90-100), in 32-bit arithmetic.
RS16_HD uint32_t add_mod(uint32_t x, uint32_t y) {
    uint32_t s = x + y;
    return (s + (s >> 16)) & 0xFFFFu;
}
RS16_HD uint32_t sub_mod(uint32_t x, uint32_t y) {
    uint32_t d = x - y;
    return (d + (d >> 16)) & 0xFFFFu;
}

}  // namespace rs16
