// rs16_kernels.hip -- HIP kernels of the MI355X GF(2^16) Reed-Solomon engine.
//
// Hot path (reference `Engine` FFT/IFFT butterflies, src/engine/engine_nosimd.rs
// :190-384, spec src/engine/engine_naive.rs:43-124, driven by the Rate code
// src/rate/rate_high.rs:44-83, 168-247):
//
//   A transform of 2^L rows is done in ceil(L/8) HBM passes.  Each pass loads
//   a tile of 2^T rows x 64 quads (512 B of every row; a quad = 4 elements =
//   one lo dword + one hi dword, see rs16_gf.hpp) into registers, applies T
//   layers, and stores it.  A workgroup has 2^(T-4) waves; lane = quad, so
//   every twiddle (which depends only on the row index) is wave-uniform and
//   its multiply table is fetched with scalar loads into SGPRs.  Each thread
//   holds 16 rows of one quad in VGPRs; the 4 layers whose row bits are in
//   registers are radix-16 butterfly networks with no data movement, and the
//   other (T-4) layers are reached by one LDS transpose (layout A: k bits
//   0-3 in registers, layout B: k bits T-4..T-1 in registers).
//
//   Butterflies (identical to the reference, which is the bit-exact spec):
//     FFT  layer d: a ^= b * skew[r + d + skew_delta - 1];  b ^= a
//     IFFT layer d: b ^= a;  a ^= b * skew[r + d + skew_delta - 1]
//   with r = group start (row & ~(2d-1)) and the GF_MODULUS sentinel meaning
//   "no multiply" (table entry ZERO_ENTRY multiplies by zero).
#include <algorithm>

#include "rs16_internal.hpp"

namespace rs16 {

typedef const __attribute__((address_space(4))) uint32_t* cu32p;
typedef const __attribute__((address_space(4))) uint8_t* cu8p;

enum LoadMode { LD_PLAIN = 0, LD_GATHER_ENC, LD_GATHER_DEC, LD_DEC_LAST };
enum StoreMode { ST_PLAIN = 0, ST_RECOVERY, ST_RESTORE };

template <int P> struct ProgTraits;
#define RS16_PROG(P, LD, I, F, FF, ST)                                                  \
    template <> struct ProgTraits<P> {                                                 \
        static constexpr int LOAD = LD;                                                \
        static constexpr bool IFFT = I, FD = F, FFT = FF;                              \
        static constexpr int STORE = ST;                                               \
    };
RS16_PROG(GEN_FFT, LD_PLAIN, false, false, true, ST_PLAIN)
RS16_PROG(GEN_IFFT, LD_PLAIN, true, false, false, ST_PLAIN)
RS16_PROG(ENC_FIRST, LD_GATHER_ENC, true, false, false, ST_PLAIN)
RS16_PROG(ENC_MID, LD_PLAIN, true, false, true, ST_PLAIN)
RS16_PROG(ENC_LAST, LD_PLAIN, false, false, true, ST_RECOVERY)
RS16_PROG(ENC_SINGLE, LD_GATHER_ENC, true, false, true, ST_RECOVERY)
RS16_PROG(DEC_FIRST, LD_GATHER_DEC, true, false, false, ST_PLAIN)
RS16_PROG(DEC_MID, LD_PLAIN, true, true, true, ST_PLAIN)
RS16_PROG(DEC_LAST, LD_DEC_LAST, false, false, true, ST_RESTORE)
RS16_PROG(DEC_SINGLE, LD_GATHER_DEC, true, true, true, ST_RESTORE)
#undef RS16_PROG

template <int T> struct Geo {
    static constexpr int R = T > 4 ? 4 : T;       // row bits held in registers
    static constexpr int NR = 1 << R;             // rows per thread
    static constexpr int W = T > 4 ? (1 << (T - 4)) : 1;  // waves per workgroup
    static constexpr int SHB = T - R;             // layout B: k = w + (m << SHB)
    static constexpr int THREADS = 64 * W;
};

template <int P, int T> constexpr bool uses_lds() {
    return T > 4 || ProgTraits<P>::FD || ProgTraits<P>::LOAD == LD_DEC_LAST;
}

struct Thr {
    uint32_t lane, w, b_low, b_high, offL;
    bool active;
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

template <int T, bool LB> __device__ __forceinline__ uint32_t kidx(const Thr& c, int m) {
    return LB ? c.w + ((uint32_t)m << Geo<T>::SHB) : (c.w << Geo<T>::R) + (uint32_t)m;
}

template <int T> __device__ __forceinline__ uint32_t row_rel(const Thr& c, const PassArgs& a, uint32_t k) {
    return c.b_low + (k << a.lo) + (c.b_high << (a.lo + T));
}

__device__ __forceinline__ void ld_quad(const uint8_t* row, const Thr& c, uint32_t& L, uint32_t& H) {
    if (c.active) {
        L = *(const uint32_t*)(row + c.offL);
        H = *(const uint32_t*)(row + c.offL + 32);
    } else {
        L = H = 0;
    }
}
__device__ __forceinline__ void st_quad(uint8_t* row, const Thr& c, uint32_t L, uint32_t H) {
    if (c.active) {
        *(uint32_t*)(row + c.offL) = L;
        *(uint32_t*)(row + c.offL + 32) = H;
    }
}

// Apply layers for k-bits [KB0, KB1) held in registers of layout LB.
template <int T, bool LB, int KB0, int KB1, bool FFT>
__device__ __forceinline__ void layers(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                       const PassArgs& a, uint32_t skew) {
    constexpr int SH = LB ? Geo<T>::SHB : 0;
    cu32p sk = (cu32p)a.skew_entry;
    cu32p tb = (cu32p)a.mul_tab;
#pragma unroll
    for (int s = 0; s < KB1 - KB0; s++) {
        const int kb = FFT ? KB1 - 1 - s : KB0 + s;
        const int rb = kb - SH;
        const uint32_t d = 1u << (a.lo + kb);
#pragma unroll
        for (int m = 0; m < Geo<T>::NR; m++) {
            if ((m >> rb) & 1) continue;
            const int m2 = m | (1 << rb);
            const uint32_t r = row_rel<T>(c, a, kidx<T, LB>(c, m));
            const uint32_t g = r & ~(2 * d - 1);
            const uint32_t e = uni(sk[g + d + skew - 1]);
            cu32p t = tb + e * TAB_DWORDS;
            uint32_t tt[20];
#pragma unroll
            for (int i = 0; i < 20; i++) tt[i] = t[i];
            if (FFT) {
                mul_xor(L[m], H[m], L[m2], H[m2], tt);
                L[m2] ^= L[m];
                H[m2] ^= H[m];
            } else {
                L[m2] ^= L[m];
                H[m2] ^= H[m];
                mul_xor(L[m], H[m], L[m2], H[m2], tt);
            }
        }
    }
}

template <int T, bool FROM_B>
__device__ __forceinline__ void exchange(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                         uint2* lds) {
#pragma unroll
    for (int m = 0; m < Geo<T>::NR; m++) lds[kidx<T, FROM_B>(c, m) * 64 + c.lane] = make_uint2(L[m], H[m]);
    __syncthreads();
#pragma unroll
    for (int m = 0; m < Geo<T>::NR; m++) {
        uint2 v = lds[kidx<T, !FROM_B>(c, m) * 64 + c.lane];
        L[m] = v.x;
        H[m] = v.y;
    }
    __syncthreads();
}

// y[k] = (SELF ? x[k] : base[k]) ^ XOR_{b < T, k_b = 0} x[k | 2^b], x read from LDS.
// This is the formal derivative restricted to the tile's row bits
// (reference Engine::formal_derivative, src/engine.rs:233-238, in closed form:
// step i = (j & ~(2^b-1)) | 2^b XORs row j|2^b into row j, and that source row
// is never written before it is read).
template <int T, bool LB>
__device__ __forceinline__ void fd_from_lds(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                            const uint2* lds) {
#pragma unroll
    for (int m = 0; m < Geo<T>::NR; m++) {
        const uint32_t k = kidx<T, LB>(c, m);
        uint32_t xl = L[m], xh = H[m];
#pragma unroll
        for (int b = 0; b < T; b++) {
            if (!((k >> b) & 1)) {
                uint2 v = lds[(k | (1u << b)) * 64 + c.lane];
                xl ^= v.x;
                xh ^= v.y;
            }
        }
        L[m] = xl;
        H[m] = xh;
    }
}

template <int P, int T>
__global__ void __launch_bounds__(Geo<T>::THREADS) pass_kernel(PassArgs a) {
    using PT = ProgTraits<P>;
    constexpr int NR = Geo<T>::NR;
    constexpr int R = Geo<T>::R;
    extern __shared__ uint2 lds[];

    Thr c;
    c.lane = threadIdx.x & 63;
    c.w = uni(threadIdx.x >> 6);
    const uint32_t slab = blockIdx.x % a.nslab;
    const uint32_t tile = blockIdx.x / a.nslab + a.tile_base;
    c.b_low = tile & ((1u << a.lo) - 1);
    c.b_high = tile >> a.lo;
    const uint32_t Q = slab * 64 + c.lane;
    c.active = Q < a.qrow;
    c.offL = (Q >> 3) * 64 + (Q & 7) * 4;
    cu32p elog = (cu32p)a.elog;
    cu32p tb = (cu32p)a.mul_tab;

    uint32_t L[NR], H[NR];
    // Layout of the first transform phase: IFFT starts with the low k bits
    // (layout A), FFT with the high ones (layout B).
    constexpr bool START_B = !PT::IFFT;

    // ---------------- load ----------------
    if (PT::LOAD == LD_PLAIN) {
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t r = row_rel<T>(c, a, kidx<T, START_B>(c, m));
            ld_quad(a.in + (uint64_t)r * a.S, c, L[m], H[m]);
        }
    } else if (PT::LOAD == LD_GATHER_ENC) {
        // HighRateEncoder::encode: work[0..k) = originals, rest zero (rate_high.rs:50-54)
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t r = row_rel<T>(c, a, kidx<T, START_B>(c, m));
            if (r < a.a_count) ld_quad(a.seg_a + (uint64_t)r * a.S, c, L[m], H[m]);
            else L[m] = H[m] = 0;
        }
    } else if (PT::LOAD == LD_GATHER_DEC) {
        // "MULTIPLY SHARDS" of rate_high.rs:203-228 / rate_low.rs:203-228:
        // received rows * erasure log, everything else zero.
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t r = row_rel<T>(c, a, kidx<T, START_B>(c, m));
            const uint8_t* src = nullptr;
            if (r < a.a_count) {
                if (!a.flags_a || uni(((cu8p)a.flags_a)[r])) src = a.seg_a + (uint64_t)r * a.S;
            } else if (r >= a.chunk && r - a.chunk < a.b_count) {
                const uint32_t i = r - a.chunk;
                if (!a.flags_b || uni(((cu8p)a.flags_b)[i])) src = a.seg_b + (uint64_t)i * a.S;
            }
            L[m] = H[m] = 0;
            if (src) {
                uint32_t yl, yh;
                ld_quad(src, c, yl, yh);
                const uint32_t e = uni(elog[r]);
                cu32p t = tb + e * TAB_DWORDS;
                uint32_t tt[20];
#pragma unroll
                for (int i = 0; i < 20; i++) tt[i] = t[i];
                mul_xor(L[m], H[m], yl, yh, tt);
            }
        }
    } else {  // LD_DEC_LAST: y = u + L(z)  (L = formal-derivative part over the tile's bits)
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t k = kidx<T, START_B>(c, m);
            const uint32_t r = row_rel<T>(c, a, k);
            uint32_t zl, zh;
            ld_quad(a.in + (uint64_t)r * a.S, c, zl, zh);
            lds[k * 64 + c.lane] = make_uint2(zl, zh);
            ld_quad(a.in2 + (uint64_t)r * a.S, c, L[m], H[m]);
        }
        __syncthreads();
        fd_from_lds<T, START_B>(L, H, c, lds);
        __syncthreads();
    }

    // ---------------- IFFT ----------------
    bool in_b = START_B;
    if (PT::IFFT) {
        layers<T, false, 0, R, false>(L, H, c, a, a.skew_ifft);
        if (T > 4) {
            exchange<T, false>(L, H, c, lds);
            layers<T, true, 4, (T > 4 ? T : 4), false>(L, H, c, a, a.skew_ifft);
            in_b = true;
        }
    }
    // ---------------- formal derivative (tile bits) ----------------
    if (PT::FD) {
        if (in_b) {
#pragma unroll
            for (int m = 0; m < NR; m++) lds[kidx<T, true>(c, m) * 64 + c.lane] = make_uint2(L[m], H[m]);
            __syncthreads();
            fd_from_lds<T, true>(L, H, c, lds);
        } else {
#pragma unroll
            for (int m = 0; m < NR; m++) lds[kidx<T, false>(c, m) * 64 + c.lane] = make_uint2(L[m], H[m]);
            __syncthreads();
            fd_from_lds<T, false>(L, H, c, lds);
        }
        __syncthreads();
    }
    // ---------------- FFT ----------------
    if (PT::FFT) {
        if (T > 4) {
            layers<T, true, 4, (T > 4 ? T : 4), true>(L, H, c, a, a.skew_fft);
            exchange<T, true>(L, H, c, lds);
            in_b = false;
        }
        layers<T, false, 0, R, true>(L, H, c, a, a.skew_fft);
    }

    // ---------------- store ----------------
    // Final layout: after FFT -> A; after IFFT only -> B (T > 4) ; T <= 4: A == B.
    constexpr bool END_B = !PT::FFT && T > 4;
#pragma unroll
    for (int m = 0; m < NR; m++) {
        const uint32_t r = row_rel<T>(c, a, kidx<T, END_B>(c, m));
        if (PT::STORE == ST_PLAIN) {
            st_quad(a.out + (uint64_t)r * a.S, c, L[m], H[m]);
        } else if (PT::STORE == ST_RECOVERY) {
            if (r < a.out_rows) st_quad(a.out + (uint64_t)r * a.S, c, L[m], H[m]);
        } else {
            // REVEAL ERASURES (rate_high.rs:236-242 / rate_low.rs:236-242):
            // lost original i -> work[i] * (GF_MODULUS - erasures[i]).
            const uint32_t base = a.rest_seg_b ? a.chunk : 0;
            const uint32_t cnt = a.rest_seg_b ? a.b_count : a.a_count;
            const uint8_t* fl = a.rest_seg_b ? a.flags_b : a.flags_a;
            if (r >= base && r - base < cnt) {
                const uint32_t i = r - base;
                const bool received = !fl || uni(((cu8p)fl)[i]);
                if (!received) {
                    const uint32_t e = GF_MODULUS - uni(elog[r]);
                    cu32p t = tb + e * TAB_DWORDS;
                    uint32_t tt[20];
#pragma unroll
                    for (int j = 0; j < 20; j++) tt[j] = t[j];
                    uint32_t ol = 0, oh = 0;
                    mul_xor(ol, oh, L[m], H[m], tt);
                    st_quad(a.rest + (uint64_t)i * a.S, c, ol, oh);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Dispatch table [prog][T].
// ---------------------------------------------------------------------------
typedef void (*PassFn)(PassArgs);

#define RS16_ROW(P) {pass_kernel<P, 0>, pass_kernel<P, 1>, pass_kernel<P, 2>, pass_kernel<P, 3>, pass_kernel<P, 4>, \
                     pass_kernel<P, 5>, pass_kernel<P, 6>, pass_kernel<P, 7>, pass_kernel<P, 8>}
static const PassFn kPass[NUM_PROGS][9] = {
    RS16_ROW(GEN_FFT),  RS16_ROW(GEN_IFFT),  RS16_ROW(ENC_FIRST), RS16_ROW(ENC_MID),  RS16_ROW(ENC_LAST),
    RS16_ROW(ENC_SINGLE), RS16_ROW(DEC_FIRST), RS16_ROW(DEC_MID),  RS16_ROW(DEC_LAST), RS16_ROW(DEC_SINGLE),
};
#undef RS16_ROW

static bool prog_uses_lds(int prog, int T) {
    bool fd = prog == DEC_MID || prog == DEC_SINGLE;
    return T > 4 || fd || prog == DEC_LAST;
}

hipError_t launch_pass(int prog, int T, const PassArgs& a, uint32_t num_tiles, hipStream_t s) {
    if (prog < 0 || prog >= NUM_PROGS || T < 0 || T > 8) return hipErrorInvalidValue;
    if (num_tiles == 0) return hipSuccess;
    const int W = T > 4 ? (1 << (T - 4)) : 1;
    const size_t lds = prog_uses_lds(prog, T) ? ((size_t)1 << T) * 64 * sizeof(uint2) : 0;
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)kPass[prog][T], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    dim3 grid(num_tiles * a.nslab), block(64 * W);
    hipLaunchKernelGGL(kPass[prog][T], grid, block, lds, s, a);
    return hipGetLastError();
}

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

__device__ __forceinline__ uint32_t erasure_at(const ErasureSpec& e, uint32_t i) {
    if (i < e.a_count) return e.flags_a ? (((cu8p)e.flags_a)[i] ? 0u : 1u) : 0u;
    if (i < e.chunk) return e.pad_fill;
    if (i - e.chunk < e.b_count) return e.flags_b ? (((cu8p)e.flags_b)[i - e.chunk] ? 0u : 1u) : 0u;
    return e.tail_fill;
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
template <bool MULW, int IN16, int OUT16>
__global__ void __launch_bounds__(256) fwht_lo_kernel(const uint32_t* in32, const uint16_t* in16, uint32_t* out32,
                                                       uint16_t* out16, const uint16_t* log_walsh) {
    __shared__ uint32_t s[256];
    const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
    s[threadIdx.x] = IN16 ? in16[idx] : in32[idx];
    fwht256_lds(s);
    if (MULW) {
        s[threadIdx.x] = (uint32_t)(((uint64_t)s[threadIdx.x] * log_walsh[idx]) % GF_MODULUS);
        fwht256_lds(s);
    }
    if (OUT16) out16[idx] = (uint16_t)s[threadIdx.x];
    else out32[idx] = s[threadIdx.x];
}

hipError_t launch_eval_poly_from_flags(const ErasureSpec& e, uint32_t* work, uint32_t* out_elog,
                                       const uint16_t* log_walsh, hipStream_t s) {
    hipLaunchKernelGGL((fwht_hi_kernel<1, 0>), dim3(256), dim3(256), 0, s, e, nullptr, nullptr, work, nullptr);
    hipLaunchKernelGGL((fwht_lo_kernel<true, 0, 0>), dim3(256), dim3(256), 0, s, work, nullptr, work, nullptr, log_walsh);
    hipLaunchKernelGGL((fwht_hi_kernel<0, 0>), dim3(256), dim3(256), 0, s, e, work, nullptr, out_elog, nullptr);
    return hipGetLastError();
}
hipError_t launch_eval_poly_u16(uint16_t* data, uint32_t* work, const uint16_t* log_walsh, hipStream_t s) {
    ErasureSpec e{};
    hipLaunchKernelGGL((fwht_hi_kernel<2, 0>), dim3(256), dim3(256), 0, s, e, nullptr, data, work, nullptr);
    hipLaunchKernelGGL((fwht_lo_kernel<true, 0, 0>), dim3(256), dim3(256), 0, s, work, nullptr, work, nullptr, log_walsh);
    hipLaunchKernelGGL((fwht_hi_kernel<0, 1>), dim3(256), dim3(256), 0, s, e, work, nullptr, nullptr, data);
    return hipGetLastError();
}
hipError_t launch_fwht_u16(uint16_t* data, uint32_t* work, hipStream_t s) {
    ErasureSpec e{};
    hipLaunchKernelGGL((fwht_hi_kernel<2, 0>), dim3(256), dim3(256), 0, s, e, nullptr, data, work, nullptr);
    hipLaunchKernelGGL((fwht_lo_kernel<false, 0, 1>), dim3(256), dim3(256), 0, s, work, nullptr, nullptr, data, nullptr);
    return hipGetLastError();
}

}  // namespace rs16
