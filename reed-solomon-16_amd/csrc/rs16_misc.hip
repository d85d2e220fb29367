// rs16_misc.hip -- elementwise engine ops (mul, xor, formal derivative) and the
// FWHT / eval_poly kernels of the MI355X GF(2^16) Reed-Solomon engine.
#include <algorithm>

#include <cstdlib>

#include "rs16_internal.hpp"
#include "rs16_fwht.hpp"
#include "rs16_diag.hpp"

namespace rs16 {

typedef const __attribute__((address_space(4))) uint32_t* cu32p;
typedef const __attribute__((address_space(4))) uint8_t* cu8p;

// ---------------------------------------------------------------------------
// Elementwise engine ops.
// ---------------------------------------------------------------------------
// Engine::mul: x[] *= log_m (NoSimd::mul, src/engine/engine_nosimd.rs:65-79).
__global__ void __launch_bounds__(256) mul_kernel(uint8_t* x, size_t nquads, uint32_t entry, const uint32_t* mul_tab) {
    cu32p t = (cu32p)mul_tab + (size_t)entry * TAB_DWORDS;
    uint32_t tt[20];
#pragma unroll
    for (int i = 0; i < 20; i++) tt[i] = t[i];
    for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < nquads; q += (size_t)gridDim.x * blockDim.x) {
        const size_t off = (q >> 3) * 64 + (q & 7) * 4;
        uint32_t yl = *(uint32_t*)(x + off), yh = *(uint32_t*)(x + off + 32);
        uint32_t ol = 0, oh = 0;
        mul_xor(ol, oh, yl, yh, tt);
        *(uint32_t*)(x + off) = ol;
        *(uint32_t*)(x + off + 32) = oh;
    }
}
hipError_t launch_mul(uint8_t* x, size_t bytes, uint32_t entry, const uint32_t* mul_tab, hipStream_t s) {
    const size_t nq = bytes / 8;
    if (!nq) return hipSuccess;
    const unsigned grid = (unsigned)std::min<size_t>((nq + 255) / 256, 4096);
    hipLaunchKernelGGL(mul_kernel, dim3(grid), dim3(256), 0, s, x, nq, entry, mul_tab);
    return hipGetLastError();
}

// Engine::xor: x[] ^= y[] (src/engine/engine_nosimd.rs:81-88), 16 B per lane.
__global__ void __launch_bounds__(256) xor_kernel(uint4* x, const uint4* y, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        uint4 a = x[i], b = y[i];
        x[i] = make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
    }
}
hipError_t launch_xor(uint8_t* x, const uint8_t* y, size_t bytes, hipStream_t s) {
    const size_t n16 = bytes / 16;
    if (!n16) return hipSuccess;
    const unsigned grid = (unsigned)std::min<size_t>((n16 + 255) / 256, 8192);
    hipLaunchKernelGGL(xor_kernel, dim3(grid), dim3(256), 0, s, (uint4*)x, (const uint4*)y, n16);
    return hipGetLastError();
}

// Multi-chunk encodes: w[0, cb) ^= XOR of the nch - 1 chunks behind it
// (HighRateEncoder's xor_within accumulation, src/rate/rate_high.rs:56-74),
// and chunk 0 copied into chunks 1 .. nch - 1 (LowRateEncoder's per-chunk
// copy of the transformed originals, src/rate/rate_low.rs:56-74); 16 B per lane.
__global__ void __launch_bounds__(256) xor_chunks_kernel(uint4* w, size_t c16, uint32_t nch) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < c16; i += (size_t)gridDim.x * blockDim.x) {
        uint4 a = w[i];
        for (uint32_t c = 1; c < nch; c++) {
            const uint4 b = w[c * c16 + i];
            a.x ^= b.x; a.y ^= b.y; a.z ^= b.z; a.w ^= b.w;
        }
        w[i] = a;
    }
}
__global__ void __launch_bounds__(256) copy_chunks_kernel(uint4* w, size_t c16, uint32_t nch) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < c16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 a = w[i];
        for (uint32_t c = 1; c < nch; c++) w[c * c16 + i] = a;
    }
}
hipError_t launch_xor_chunks(uint8_t* w, size_t chunk_bytes, uint32_t nch, hipStream_t s) {
    const size_t c16 = chunk_bytes / 16;
    if (!c16 || nch < 2) return hipSuccess;
    const unsigned grid = (unsigned)std::min<size_t>((c16 + 255) / 256, 8192);
    hipLaunchKernelGGL(xor_chunks_kernel, dim3(grid), dim3(256), 0, s, (uint4*)w, c16, nch);
    return hipGetLastError();
}
hipError_t launch_copy_chunks(uint8_t* w, size_t chunk_bytes, uint32_t nch, hipStream_t s) {
    const size_t c16 = chunk_bytes / 16;
    if (!c16 || nch < 2) return hipSuccess;
    const unsigned grid = (unsigned)std::min<size_t>((c16 + 255) / 256, 8192);
    hipLaunchKernelGGL(copy_chunks_kernel, dim3(grid), dim3(256), 0, s, (uint4*)w, c16, nch);
    return hipGetLastError();
}

// Engine::formal_derivative (src/engine.rs:233-238), closed form, out of place:
// out[j] = in[j] ^ XOR_{b : j_b = 0, 2^b < n} in[j | 2^b]   (n a power of two).
__global__ void __launch_bounds__(256) fd_kernel(uint4* out, const uint4* in, uint32_t n, size_t row16) {
    const size_t total = (size_t)n * row16;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t j = (uint32_t)(i / row16);
        const size_t col = i - (size_t)j * row16;
        uint4 acc = in[i];
        for (uint32_t b = 1; b < n; b <<= 1)
            if (!(j & b)) {
                uint4 v = in[(size_t)(j | b) * row16 + col];
                acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
            }
        out[i] = acc;
    }
}
hipError_t launch_formal_derivative(uint8_t* out, const uint8_t* in, size_t n, size_t S, hipStream_t s) {
    const size_t row16 = S / 16, total = n * row16;
    if (!total) return hipSuccess;
    const unsigned grid = (unsigned)std::min<size_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(fd_kernel, dim3(grid), dim3(256), 0, s, (uint4*)out, (const uint4*)in, (uint32_t)n, row16);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// FWHT over Z/65535 (reference Engine::fwht, NoSimd::fwht_private
// src/engine/engine_nosimd.rs:121-183) and eval_poly (src/engine.rs:207-218).
// The 65536-point transform is two passes of 256-point transforms (row bits
// 8-15 strided, then bits 0-7 contiguous).  The butterflies are exact ring
// operations in Z/65535, so layer order does not change any residue; a value
// may come out as 65535 where the reference has 0 (same residue), which every
// consumer treats identically (mul by log 0 == mul by log 65535 == x1).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void fwht256_lds(uint32_t* s) {
    const int t = threadIdx.x;  // 256 threads
#pragma unroll
    for (int d = 1; d < 256; d <<= 1) {
        __syncthreads();
        if (t < 128) {
            const int i = (t / d) * 2 * d + (t % d), j = i + d;
            const uint32_t x = s[i], y = s[j];
            s[i] = add_mod(x, y);
            s[j] = sub_mod(x, y);
        }
    }
    __syncthreads();
}

// Stripe y = blockIdx.y of a batch with losses of its own (ErasureSpec::nstripes):
// its flags and its outputs.
__device__ __forceinline__ void stripe_spec(ErasureSpec& e) {
    const uint32_t y = blockIdx.y;
    if (y == 0) return;
    if (e.flags_a) e.flags_a += y * e.bs_fa;
    if (e.flags_b) e.flags_b += y * e.bs_fb;
    if (e.rbits) e.rbits += y * e.bs_rbits;
    if (e.zflags) e.zflags += y * e.bs_zflags;
    if (e.lostpart) e.lostpart += y * e.bs_lost;
    if (e.lostrange) e.lostrange += y * e.bs_lost;
}
__device__ __forceinline__ uint32_t erasure_at(const ErasureSpec& e, uint32_t i) {
    if (i < e.a_count) return e.flags_a ? (((cu8p)e.flags_a)[i] ? 0u : 1u) : 0u;
    if (i < e.chunk) return e.pad_fill;
    if (i - e.chunk < e.b_count) return e.flags_b ? (((cu8p)e.flags_b)[i - e.chunk] ? 0u : 1u) : 0u;
    return e.tail_fill;
}

__device__ __forceinline__ bool received_at(const ErasureSpec& e, uint32_t i) {
    if (i < e.a_count) return e.flags_a ? ((cu8p)e.flags_a)[i] != 0 : true;
    if (i >= e.chunk && i - e.chunk < e.b_count) return e.flags_b ? ((cu8p)e.flags_b)[i - e.chunk] != 0 : true;
    return false;
}
// Row i lies in the originals' segment (B for the high rate, A for the low).
__device__ __forceinline__ bool orig_row(const ErasureSpec& e, uint32_t i) {
    return e.orig_b ? (i >= e.chunk && i - e.chunk < e.b_count) : i < e.a_count;
}
// First / one past the last lost-original row of block blk (rows base +
// 64 j + bit of lmask[j]), ~0u / 0 if none, by lane 0 of the wave.
__device__ __forceinline__ void lost_part_wave(const ErasureSpec& e, uint32_t blk, uint32_t base,
                                               const uint64_t (&lmask)[4]) {
    uint32_t lo = ~0u, hi = 0;
#pragma unroll
    for (int j = 3; j >= 0; j--)
        if (lmask[j]) lo = base + 64u * j + (uint32_t)__builtin_ctzll(lmask[j]);
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (lmask[j]) hi = base + 64u * j + 64u - (uint32_t)__builtin_clzll(lmask[j]);
    if ((threadIdx.x & 63) == 0) {
        e.lostpart[2 * blk] = lo;
        e.lostpart[2 * blk + 1] = hi;
    }
}
// lostrange = [min lostpart lo, max lostpart hi) over the 256 blocks, by one wave.
__device__ __forceinline__ void lost_range_wave(const ErasureSpec& e) {
    const uint32_t lane = threadIdx.x & 63;
    const uint4 p0 = ((const uint4*)e.lostpart)[2 * lane], p1 = ((const uint4*)e.lostpart)[2 * lane + 1];
    uint32_t lo = min(min(p0.x, p0.z), min(p1.x, p1.z)), hi = max(max(p0.y, p0.w), max(p1.y, p1.w));
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, d));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, d));
    }
    if (lane == 0) {
        e.lostrange[0] = lo;
        e.lostrange[1] = hi;
    }
}
// Received rows of the 64-row chunk at row r0 by segment (A = rows < a_count),
// from the chunk's ballot: lane 0 writes rcount (ErasureSpec).
__device__ __forceinline__ void chunk_counts(const ErasureSpec& e, uint32_t r0, uint64_t rcv, uint64_t rcv_a) {
    if (e.rcount && (threadIdx.x & 63) == 0 && r0 < e.n) {
        const uint32_t ca = (uint32_t)__popcll(rcv_a);
        e.rcount[2 * (r0 >> 6)] = ca;
        e.rcount[2 * (r0 >> 6) + 1] = (uint32_t)__popcll(rcv) - ca;
    }
}
// Received-row bitmap and zero-tile flags of rows [base, base + 256) by one
// wave, from the ballots rmask[j] of rows base + 64 j + lane: rbits words,
// zflags per tile of 2^zlo rows.
__device__ __forceinline__ void block_flags_wave(const ErasureSpec& e, uint32_t base, const uint64_t (&rmask)[4]) {
    const uint32_t lane = threadIdx.x & 63;
    if (base >= e.n) return;
    if (e.rbits && lane < 8 && base + 32u * lane < e.n)
        e.rbits[(base >> 5) + lane] = (uint32_t)(rmask[lane >> 1] >> (32 * (lane & 1)));
    if (e.zflags) {
        const uint32_t ts = 1u << e.zlo, ntile = e.n >> e.zlo;
        // tile t of this block: rows [t ts, (t + 1) ts), t < 256 / ts
        for (uint32_t t = lane; t < 256u / ts; t += 64) {
            bool any = false;
            for (uint32_t r = t * ts; r < (t + 1) * ts; r += 64) {
                const uint32_t w = r >> 6, sh = r & 63, len = ts < 64 ? ts : 64;
                const uint64_t m = len == 64 ? ~0ull : ((1ull << len) - 1) << sh;
                any |= (rmask[w] & m) != 0;
            }
            if ((base >> e.zlo) + t < ntile) e.zflags[(base >> e.zlo) + t] = any ? 0 : 1;
        }
    }
}

// MODE 0: in = u32 work; MODE 1: build erasures from flags; MODE 2: in = u16 data.
// OUT 0: u32 work/out; OUT 1: u16 data.
template <int MODE, int OUT>
__global__ void __launch_bounds__(256) fwht_hi_kernel(ErasureSpec e, const uint32_t* in32, const uint16_t* in16,
                                                       uint32_t* out32, uint16_t* out16) {
    __shared__ uint32_t s[256];
    const uint32_t idx = blockIdx.x + 256u * threadIdx.x;  // bits 8-15 vary within the block
    uint32_t v;
    if (MODE == 0) v = in32[idx];
    else if (MODE == 1) v = erasure_at(e, idx);
    else v = in16[idx];
    s[threadIdx.x] = v;
    fwht256_lds(s);
    if (OUT == 0) out32[idx] = s[threadIdx.x];
    else out16[idx] = (uint16_t)s[threadIdx.x];
}

// Contiguous 256-point FWHT; if MULW, then multiply by log_walsh mod 65535 and
// do the contiguous FWHT again (the middle of eval_poly).
// (grid row y: in32 / out32 displaced by y bs_in / bs_out words -- the
// stripes of a batch with losses of their own)
template <bool MULW, int IN16, int OUT16>
__global__ void __launch_bounds__(256) fwht_lo_kernel(const uint32_t* in32, const uint16_t* in16, uint32_t* out32,
                                                       uint16_t* out16, const uint16_t* log_walsh, uint32_t bs_in = 0,
                                                       uint32_t bs_out = 0) {
    __shared__ uint32_t s[256];
    const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
    if (in32) in32 += blockIdx.y * bs_in;
    if (out32) out32 += blockIdx.y * bs_out;
    s[threadIdx.x] = IN16 ? in16[idx] : in32[idx];
    fwht256_lds(s);
    if (MULW) {
        s[threadIdx.x] = (uint32_t)(((uint64_t)s[threadIdx.x] * log_walsh[idx]) % GF_MODULUS);
        fwht256_lds(s);
    }
    if (OUT16) out16[idx] = (uint16_t)s[threadIdx.x];
    else out32[idx] = s[threadIdx.x];
}

// Contiguous 256-point FWHT of the erasure vector built from the received
// flags, one wave per 256-row block; the same wave writes the block's
// received bitmap (ballots) and zero-tile flags.
__global__ void __launch_bounds__(64) fwht_lo_flags_kernel(ErasureSpec e, uint32_t* out32) {
    const uint32_t base = blockIdx.x * 256u, lane = threadIdx.x;
    stripe_spec(e);
    out32 += blockIdx.y * e.bs_work;
    uint32_t v[4];
    uint64_t rmask[4], lmask[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t i = base + lane + 64u * j;
        v[j] = erasure_at(e, i);
        const bool rcv = i < e.n && received_at(e, i);
        rmask[j] = __ballot(rcv);
        lmask[j] = __ballot(i < e.n && orig_row(e, i) && !rcv);
        chunk_counts(e, base + 64u * j, rmask[j], __ballot(rcv && i < e.a_count));
    }
    block_flags_wave(e, base, rmask);
    if (e.lostpart) lost_part_wave(e, blockIdx.x, base, lmask);
    fwht256_wave(v);
#pragma unroll
    for (int j = 0; j < 4; j++) out32[base + lane + 64u * j] = v[j];
}
// Strided 256-point FWHT (row bits 8-15), x LogWalsh mod 65535, and again;
// one wave per column.
__global__ void __launch_bounds__(64) fwht_hi_mulw_kernel(ErasureSpec e, const uint32_t* in32, uint32_t* out32,
                                                          const uint16_t* log_walsh) {
    const uint32_t lane = threadIdx.x;
    stripe_spec(e);
    in32 += blockIdx.y * e.bs_work;
    out32 += blockIdx.y * e.bs_work;
    uint32_t v[4], lw[4];
    // LogWalsh does not depend on the previous kernel: its loads go first
#pragma unroll
    for (int j = 0; j < 4; j++) lw[j] = log_walsh[blockIdx.x + 256u * (lane + 64u * j)];
#pragma unroll
    for (int j = 0; j < 4; j++) v[j] = in32[blockIdx.x + 256u * (lane + 64u * j)];
    fwht256_wave(v);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        // v, lw <= 65535: the product fits 32 bits; two folds reduce it mod
        // 65535 (65535 may stand for 0: same residue)
        uint32_t p = v[j] * lw[j];
        p = (p & 0xFFFFu) + (p >> 16);
        v[j] = (p & 0xFFFFu) + (p >> 16);
    }
    fwht256_wave(v);
#pragma unroll
    for (int j = 0; j < 4; j++) out32[blockIdx.x + 256u * (lane + 64u * j)] = v[j];
    if (blockIdx.x == 0 && e.lostrange) lost_range_wave(e);
}

// eval_poly(e) = FWHT(LogWalsh . FWHT(e)) with FWHT = H_lo H_hi (row bits 0-7
// and 8-15; the two commute): H_lo(e) from the flags, then H_hi . LW . H_hi,
// then the last H_lo.  With last_lo == false the last H_lo is left to the
// consumer: the 65536-row decode passes (256-row tiles = one H_lo block each)
// finish it per tile in LDS (rs16_pass.hip), saving a kernel.
// One-kernel eval_poly for block-aligned segments (eval_fused_ok): workgroup
// j computes column j of H_lo(e) for all 256 blocks itself -- thread t reads
// block t's 256 flag bytes (16 x 16-byte loads, L2-resident after the first
// workgroup of an XCD) and, e being 0/1, x[t] = sum_r (-1)^|j&r| e[256t + r];
// for a flagged block (e = 1 - rcv)
//   x = sum_r sign(j, r) - sum_r sign(j, r) rcv(r),  sum_r sign(j, r) = 256 [j == 0],
// where the received part is a v_dot4_i32_i8 of the bytes' "nonzero" bits
// (0x80 = -128 as i8) with the sign bytes of the dword -- then H_hi, x LogWalsh,
// H_hi by wave 0 (exact integers, then Z/65535), as fwht_hi_mulw_kernel.
// Wave 1 writes block j's pass metadata (rbits, zflags) like
// fwht_lo_flags_kernel; workgroup 0 reduces the lost originals' row range.
// One kernel instead of two (the second waited for the first's stores).
__device__ __forceinline__ uint32_t nz80(uint32_t f) {  // 0x80 in every nonzero byte
    return __builtin_amdgcn_bitop3_b32((f & 0x7F7F7F7Fu) + 0x7F7F7F7Fu, f, 0x80808080u, 0xA8);  // (a | b) & c
}
// Region of block t (rows [256 t, 256 t + 256)) -- host-checked to be one of:
// 0 flags_a, 1 pad, 2 flags_b, 3 tail.
__device__ __forceinline__ int block_region(const ErasureSpec& e, uint32_t base) {
    if (base < e.a_count) return 0;
    if (base < e.chunk) return 1;
    if (base - e.chunk < e.b_count) return 2;
    return 3;
}
__global__ void __launch_bounds__(256) eval_fused_kernel(ErasureSpec e, uint32_t* out32, const uint16_t* log_walsh) {
    __shared__ int xs[256];
    __shared__ uint32_t lr[2][4];
    const uint32_t j = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    stripe_spec(e);
    out32 += blockIdx.y * e.bs_work;
    RS16_STAMP(e, 0);
    uint32_t lw[4];
    if (wv == 0) {
#pragma unroll
        for (int i = 0; i < 4; i++) lw[i] = log_walsh[(lane + 64u * i) * 256u + j];
    }
    // ---- x[t]: column j of H_lo(e) for block t ----
    const uint32_t base = t * 256u;
    const int reg = block_region(e, base);
    const uint8_t* fl = nullptr;  // flag bytes of the block (nullptr: no flags, all received)
    if (reg == 0 && e.flags_a) fl = e.flags_a + base;
    if (reg == 2 && e.flags_b) fl = e.flags_b + (base - e.chunk);
    const uint32_t fill = reg == 1 ? e.pad_fill : (reg == 3 ? e.tail_fill : 0u);
    // all erased rows give 256 [j == 0]; received (flagged) rows are subtracted
    const int all = (reg == 0 || reg == 2) ? (fl ? 1 : 0) : (int)fill;
    int acc = 0;  // -128 * sum_r sign(j, r) rcv(r)
    uint32_t lo = ~0u, hi = 0;  // lost rows of this block (workgroup 0, originals' segment)
    if (fl) {
        // sign bytes of a dword: byte b -> (-1)^|j & b|; dword q adds
        // (-1)^|(j >> 2) & q| = bit q of the Walsh row wm (XOR of the bit
        // patterns of the set bits of j >> 2)
        uint32_t sp = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) sp |= ((__builtin_popcount(j & b) & 1) ? 0xFFu : 0x01u) << (8 * b);
        const uint32_t sm = ~sp + 0x01010101u;  // bytewise negation of the +-1 bytes (no carries)
        constexpr uint64_t PAT[6] = {0xAAAAAAAAAAAAAAAAull, 0xCCCCCCCCCCCCCCCCull, 0xF0F0F0F0F0F0F0F0ull,
                                     0xFF00FF00FF00FF00ull, 0xFFFF0000FFFF0000ull, 0xFFFFFFFF00000000ull};
        uint64_t wm = 0;
#pragma unroll
        for (int b = 0; b < 6; b++) wm ^= ((j >> (2 + b)) & 1) ? PAT[b] : 0ull;
        const uint4* p = (const uint4*)fl;
        uint4 v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = p[i];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
            for (int c = 0; c < 4; c++)
                acc = __builtin_amdgcn_sdot4((int)nz80(w[c]), (int)(((wm >> (4 * i + c)) & 1) ? sm : sp), acc, false);
        }
        if (j == 0 && e.lostrange) {  // (uniform: workgroup 0 of a general decode)
            const bool want = e.orig_b ? reg == 2 : reg == 0;
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint32_t m = want ? ~nz80(w[c]) & 0x80808080u : 0u;  // erased bytes
                    const uint32_t r = base + 4u * (4 * i + c);
                    if (m) {
                        lo = min(lo, r + (uint32_t)(__builtin_ctz(m) >> 3));
                        hi = r + (uint32_t)((31 - __builtin_clz(m)) >> 3) + 1u;
                    }
                }
            }
        }
    }
    RS16_STAMP(e, 1);
    xs[t] = (j == 0 ? 256 * all : 0) + (acc >> 7);
    if (j == 0 && e.lostrange) {
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, d));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, d));
        }
        if (lane == 0) lr[0][wv] = lo, lr[1][wv] = hi;
    }
    // ---- wave 1: block j's received bitmap and zero-tile flags ----
    if (wv == 1) {
        const uint32_t b0 = j * 256u;
        uint64_t rmask[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t r = b0 + lane + 64u * i;
            const bool rcv = r < e.n && received_at(e, r);
            rmask[i] = __ballot(rcv);
            chunk_counts(e, b0 + 64u * i, rmask[i], __ballot(rcv && r < e.a_count));
        }
        block_flags_wave(e, b0, rmask);
    }
    __syncthreads();
    if (j == 0 && e.lostrange && t == 0) {
        e.lostrange[0] = min(min(lr[0][0], lr[0][1]), min(lr[0][2], lr[0][3]));
        e.lostrange[1] = max(max(lr[1][0], lr[1][1]), max(lr[1][2], lr[1][3]));
    }
    if (wv != 0) return;
    RS16_STAMP(e, 2);
    // ---- wave 0: y = H_hi(x) exactly, w = y * LW mod 65535, z = H_hi(w) ----
    int y[4];
#pragma unroll
    for (int i = 0; i < 4; i++) y[i] = xs[lane + 64 * i];
#define RS16_L(D)                                                               \
    {                                                                           \
        const bool up = (lane & (D)) != 0;                                      \
        _Pragma("unroll") for (int i = 0; i < 4; i++) {                         \
            const int p = xshfl<(D)>(y[i]);                                     \
            y[i] = up ? p - y[i] : y[i] + p;                                    \
        }                                                                       \
    }
    RS16_L(1) RS16_L(2) RS16_L(4) RS16_L(8) RS16_L(16) RS16_L(32)
#undef RS16_L
    {
        const int a = y[0] + y[1], b = y[0] - y[1], c = y[2] + y[3], d = y[2] - y[3];
        y[0] = a + c, y[2] = a - c, y[1] = b + d, y[3] = b - d;
    }
    uint32_t v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        // |y| <= 65536: y + 2 * 65535 >= 0, folded to [0, 65535]
        uint32_t u = (uint32_t)(y[i] + 2 * 65535);
        u = (u & 0xFFFFu) + (u >> 16);
        u = (u & 0xFFFFu) + (u >> 16);
        uint32_t p = u * lw[i];
        p = (p & 0xFFFFu) + (p >> 16);
        v[i] = (p & 0xFFFFu) + (p >> 16);
    }
    RS16_STAMP(e, 3);
    fwht256_wave(v);
    RS16_STAMP(e, 10);
#pragma unroll
    for (int i = 0; i < 4; i++) out32[(lane + 64u * i) * 256u + j] = v[i];
    RS16_STAMP_END(e);
}
// Segment boundaries on 256-row blocks and 16-byte aligned flag arrays.
static bool eval_fused_ok(const ErasureSpec& e) {
    const auto al = [](const uint8_t* p) { return ((uintptr_t)p & 15) == 0; };
    return e.a_count % 256 == 0 && e.chunk % 256 == 0 && e.b_count % 256 == 0 && al(e.flags_a) && al(e.flags_b);
}

hipError_t launch_eval_poly_from_flags(const ErasureSpec& e, uint32_t* work, uint32_t* out_elog,
                                       const uint16_t* log_walsh, hipStream_t s, bool last_lo) {
    const uint32_t ns = e.nstripes > 1 ? e.nstripes : 1;
    if (!(e.diag & DIAG_EVAL_TWO_KERNEL) && eval_fused_ok(e) && (ns == 1 || (e.bs_fa % 16 == 0 && e.bs_fb % 16 == 0))) {
        hipLaunchKernelGGL(eval_fused_kernel, dim3(256, ns), dim3(256), 0, s, e, work, log_walsh);
    } else {
        hipLaunchKernelGGL(fwht_lo_flags_kernel, dim3(256, ns), dim3(64), 0, s, e, work);
        hipLaunchKernelGGL(fwht_hi_mulw_kernel, dim3(256, ns), dim3(64), 0, s, e, work, work, log_walsh);
    }
    if (last_lo)
        hipLaunchKernelGGL((fwht_lo_kernel<false, 0, 0>), dim3(256, ns), dim3(256), 0, s, work, nullptr, out_elog, nullptr,
                           nullptr, e.bs_work, e.bs_elog);
    return hipGetLastError();
}
// eval_poly of a high-rate decode with n <= 2048 work rows:
// the erasure vector is zero from row n on (rate_high.rs:183-197, the
// truncation of the first fwht), so with H = H_lo H_hi only the NB = n/256
// blocks of row bits 8-15 below n carry input, and only rows < n of the
// output are consumed.  One 256-thread workgroup per low index j (row bits
// 0-7), thread t = row t of every block and h = t of the middle vector:
//   x[h']  = sum_t (-1)^|j&t| e[256h' + t]            (H_lo of the NB live blocks)
//   w[h]   = LW[256h + j] * sum_h' (-1)^|h&h'| x[h']   (H_hi, x LogWalsh)
//   z[h''] = sum_h (-1)^|h''&h| w[h],   h'' < NB       (H_hi, live outputs only)
// e is 0/1, so a wave's part of x[h'] is a difference of popcounts of its
// erasure ballot under the sign mask of j; (-1)^|h''&h| for h'' < NB <= 8
// depends only on h mod NB = lane mod NB, so a wave's part of z is a lane
// reduction over lane / NB followed by an NB-point transform across lanes
// 0..NB-1.  Wave parts are added through LDS.  Integer sums (|sum| < 2^28)
// reduced mod 65535 by folding (a result may be 65535 for 0: same residue,
// and every consumer of the logs treats both alike); the last H_lo over the
// NB output blocks is left to the decode passes (ework) or run by
// fwht_lo_kernel.
// (The kernel is short and runs once per CU: its time is instruction-fetch
// bound, so it is written for few executed instructions, 4 waves sharing
// each fetched line.)
__device__ __forceinline__ uint32_t fold65535(uint32_t u) {
    u = (u & 0xFFFFu) + (u >> 16);
    return (u & 0xFFFFu) + (u >> 16);
}
__device__ __forceinline__ uint32_t mod65535(int v) { return fold65535((uint32_t)(v + 65535 * 4096)); }
template <int NB>
__global__ void __launch_bounds__(256) eval_small_kernel(ErasureSpec e, const uint16_t* log_walsh, uint32_t* z) {
    __shared__ int part[2][4][NB];  // per-wave parts of x and z
    __shared__ uint32_t words[8];   // block j's received bitmap (zero-tile flags)
    const uint32_t j = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    stripe_spec(e);
    z += blockIdx.y * e.bs_work;
    RS16_STAMP(e, 0);
    const uint32_t lw = log_walsh[t * 256u + j];  // in flight from the start
    // flag bytes of rows 256 h' + t, all loads issued before the first use
    // (a row outside both segments reads a valid dummy byte)
    uint32_t f[NB];
#pragma unroll
    for (int hp = 0; hp < NB; hp++) {
        const uint32_t i = (uint32_t)hp * 256u + t;
        const bool in_a = i < e.a_count && e.flags_a, in_b = i - e.chunk < e.b_count && e.flags_b;
        const uint8_t* p = in_a ? e.flags_a + i : (in_b ? e.flags_b + (i - e.chunk) : (const uint8_t*)log_walsh);
        f[hp] = *(const __attribute__((address_space(1))) uint8_t*)p;
    }
    const uint64_t sm = __ballot(__builtin_popcount(j & t) & 1);
    __shared__ uint32_t lpart[2][4];  // workgroup 0: per-wave lost-original row range
    uint32_t wlo = ~0u, whi = 0;
#pragma unroll
    for (int hp = 0; hp < NB; hp++) {
        // erasure_at / received_at with the flag byte already loaded
        const uint32_t i = (uint32_t)hp * 256u + t;
        const bool in_a = i < e.a_count, in_b = i - e.chunk < e.b_count;
        const bool rcv = in_a ? (!e.flags_a || f[hp]) : (in_b && (!e.flags_b || f[hp]));
        const bool era = in_a || in_b ? !rcv : (i < e.chunk ? e.pad_fill : e.tail_fill) != 0;
        const uint64_t eb = __ballot(era);
        if (lane == 0) part[0][wv][hp] = __popcll(eb & ~sm) - __popcll(eb & sm);
        if (j == 0 && e.lostrange) {
            const uint64_t lb = __ballot(orig_row(e, i) && !rcv);
            const uint32_t r0 = (uint32_t)hp * 256u + wv * 64u;
            if (lb) {
                wlo = min(wlo, r0 + (uint32_t)__builtin_ctzll(lb));
                whi = max(whi, r0 + 64u - (uint32_t)__builtin_clzll(lb));
            }
        }
        if ((uint32_t)hp == j) {
            // workgroups j < NB: the pass metadata of block j (rows >= n
            // lie past both segments: never received)
            const uint64_t rb = __ballot(rcv);
            chunk_counts(e, (uint32_t)hp * 256u + wv * 64u, rb, __ballot(rcv && in_a));
            if (lane == 0) {
                words[2 * wv] = (uint32_t)rb;
                words[2 * wv + 1] = (uint32_t)(rb >> 32);
                if (e.rbits && i < e.n) {
                    e.rbits[(i >> 5)] = (uint32_t)rb;
                    e.rbits[(i >> 5) + 1] = (uint32_t)(rb >> 32);
                }
            }
        }
    }
    if (j == 0 && lane == 0) {
        lpart[0][wv] = wlo;
        lpart[1][wv] = whi;
    }
    RS16_STAMP(e, 1);
    __syncthreads();
    if (j == 0 && t == 0 && e.lostrange) {
        e.lostrange[0] = min(min(lpart[0][0], lpart[0][1]), min(lpart[0][2], lpart[0][3]));
        e.lostrange[1] = max(max(lpart[1][0], lpart[1][1]), max(lpart[1][2], lpart[1][3]));
    }
    if (j < NB && e.zflags) {
        const uint32_t base = j * 256u, ts = 1u << e.zlo, ntile = e.n >> e.zlo;
        if (t < 256u / ts && (base >> e.zlo) + t < ntile) {
            bool any = false;
            for (uint32_t r = t * ts; r < (t + 1) * ts; r += 32) {
                const uint32_t m = ts >= 32 ? 0xFFFFFFFFu : ((1u << ts) - 1) << (r & 31);
                any |= (words[r >> 5] & m) != 0;
            }
            e.zflags[(base >> e.zlo) + t] = any ? 0 : 1;
        }
    }
    // y = sum_h' (-1)^|h&h'| x[h'] for h = t (h & h' = lane & h' for h' < 8)
    int y = 0;
#pragma unroll
    for (int hp = 0; hp < NB; hp++) {
        const int x = part[0][0][hp] + part[0][1][hp] + part[0][2][hp] + part[0][3][hp];
        y += (__builtin_popcount(lane & (uint32_t)hp) & 1) ? -x : x;
    }
    int s = (int)fold65535(mod65535(y) * lw);
#pragma unroll
    for (int off = NB; off < 64; off <<= 1) s += __shfl_xor(s, off);
#pragma unroll
    for (int d = 1; d < NB; d <<= 1) {
        const int p = __shfl_xor(s, d);
        s = (lane & d) ? p - s : s + p;
    }
    if (lane < NB) part[1][wv][lane] = s;
    RS16_STAMP(e, 2);
    __syncthreads();
    if (t < NB) z[t * 256u + j] = mod65535(part[1][0][t] + part[1][1][t] + part[1][2][t] + part[1][3][t]);
    RS16_STAMP(e, 10);
    RS16_STAMP_END(e);
}

hipError_t launch_eval_poly_small(const ErasureSpec& e, uint32_t n, uint32_t* work, uint32_t* out_elog,
                                  const uint16_t* log_walsh, hipStream_t s, bool last_lo) {
    const uint32_t nb = n <= 256 ? 1 : n / 256;
    const uint32_t ns = e.nstripes > 1 ? e.nstripes : 1;
    switch (nb) {
        case 1: hipLaunchKernelGGL(eval_small_kernel<1>, dim3(256, ns), dim3(256), 0, s, e, log_walsh, work); break;
        case 2: hipLaunchKernelGGL(eval_small_kernel<2>, dim3(256, ns), dim3(256), 0, s, e, log_walsh, work); break;
        case 4: hipLaunchKernelGGL(eval_small_kernel<4>, dim3(256, ns), dim3(256), 0, s, e, log_walsh, work); break;
        case 8: hipLaunchKernelGGL(eval_small_kernel<8>, dim3(256, ns), dim3(256), 0, s, e, log_walsh, work); break;
        default: return hipErrorInvalidValue;
    }
    if (last_lo)
        hipLaunchKernelGGL((fwht_lo_kernel<false, 0, 0>), dim3(nb, ns), dim3(256), 0, s, work, nullptr, out_elog, nullptr,
                           nullptr, e.bs_work, e.bs_elog);
    return hipGetLastError();
}
// Engine-level fwht / eval_poly (the C ABI ops): the layers run in the
// reference's order -- ascending distance, H_lo (bits 0-7) before H_hi
// (bits 8-15) -- with its add_mod / sub_mod, so every output is the
// reference's u16 bit for bit (NoSimd's radix-4 fwht_4 is two plain layers,
// src/engine/engine_nosimd.rs:135-150; Naive, engine_naive.rs:75-92), not
// only the same residue.  The log_walsh product is canonical (% 65535).
template <bool MULW>
__global__ void __launch_bounds__(256) fwht_hi_exact_kernel(const uint32_t* in32, uint32_t* out32, uint16_t* out16,
                                                            const uint16_t* log_walsh) {
    __shared__ uint32_t s[256];
    const uint32_t idx = blockIdx.x + 256u * threadIdx.x;
    s[threadIdx.x] = in32[idx];
    fwht256_lds(s);
    uint32_t v = s[threadIdx.x];
    if (MULW) v = (uint32_t)(((uint64_t)v * log_walsh[idx]) % GF_MODULUS);
    if (out16) out16[idx] = (uint16_t)v;
    else out32[idx] = v;
}
hipError_t launch_eval_poly_u16(uint16_t* data, uint32_t* work, const uint16_t* log_walsh, hipStream_t s) {
    hipLaunchKernelGGL((fwht_lo_kernel<false, 1, 0>), dim3(256), dim3(256), 0, s, nullptr, data, work, nullptr, nullptr);
    hipLaunchKernelGGL(fwht_hi_exact_kernel<true>, dim3(256), dim3(256), 0, s, work, work, nullptr, log_walsh);
    hipLaunchKernelGGL((fwht_lo_kernel<false, 0, 0>), dim3(256), dim3(256), 0, s, work, nullptr, work, nullptr, nullptr);
    hipLaunchKernelGGL(fwht_hi_exact_kernel<false>, dim3(256), dim3(256), 0, s, work, nullptr, data, nullptr);
    return hipGetLastError();
}
hipError_t launch_fwht_u16(uint16_t* data, uint32_t* work, hipStream_t s) {
    hipLaunchKernelGGL((fwht_lo_kernel<false, 1, 0>), dim3(256), dim3(256), 0, s, nullptr, data, work, nullptr, nullptr);
    hipLaunchKernelGGL(fwht_hi_exact_kernel<false>, dim3(256), dim3(256), 0, s, work, nullptr, data, nullptr);
    return hipGetLastError();
}

}  // namespace rs16
