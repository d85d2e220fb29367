// rs16_pass.hip -- the HBM-pass kernels of the MI355X GF(2^16) Reed-Solomon
// engine: the FFT/IFFT butterflies of the reference `Engine`
// (src/engine/engine_nosimd.rs:190-384, spec src/engine/engine_naive.rs:43-124)
// fused with the Rate-level steps around them (src/rate/rate_high.rs:44-83,
// 168-247; src/rate/rate_low.rs:168-247).
//
// Structure of one pass
// ---------------------
//   A transform of 2^L rows runs in ceil(L/8) HBM passes.  A pass loads a
//   tile of 2^T rows (T <= 8) x 64 quads (512 B of each row; a quad = 4
//   elements = one lo dword + one hi dword, rs16_gf.hpp), applies T layers
//   and stores it.  Tile t covers rows  b_low + (k << lo) + (b_high << (lo+T)),
//   k in [0, 2^T): lo = 0 gives contiguous tiles, lo > 0 strided ones.
//
//   Workgroup = 2^(T-4) waves, lane = quad, so every twiddle (a function of
//   the row index only) is wave-uniform.  Each thread keeps 16 rows of its
//   quad in VGPRs: the 4 layers whose row bits are in registers are radix-16
//   butterfly networks with no data movement; one LDS transpose switches
//   between layout A (k bits 0-3 in registers) and layout B (k bits T-4..T-1).
//
//   Twiddle tables: a tile needs 2^T - 1 distinct twiddles per transform
//   direction (one per (layer, group)).  Their 80-byte v_perm multiply tables
//   are staged into LDS once per workgroup and read with broadcast
//   ds_read_b128 (5 per group), one group ahead of use.  Groups are compiled
//   as a straight-line sequence separated by register pins, so a wave holds
//   at most two tables.
//
//   Butterflies (bit-exact spec, the reference's):
//     FFT  layer d: a ^= b * skew[r + d + skew_delta - 1];  b ^= a
//     IFFT layer d: b ^= a;  a ^= b * skew[r + d + skew_delta - 1]
//   r = group start (row & ~(2d-1)); the GF_MODULUS sentinel ("no multiply",
//   engine_naive.rs:64,116) maps to the all-zero table ZERO_ENTRY.
#include "rs16_internal.hpp"

namespace rs16 {

typedef const __attribute__((address_space(4))) uint32_t* cu32p;
typedef const __attribute__((address_space(4))) uint8_t* cu8p;

enum LoadMode { LD_PLAIN = 0, LD_GATHER_ENC, LD_GATHER_DEC, LD_DEC_LAST };
enum StoreMode { ST_PLAIN = 0, ST_RECOVERY, ST_RESTORE };

template <int P> struct ProgTraits;
#define RS16_PROG(P, LD, I, F, FF, ST)          \
    template <> struct ProgTraits<P> {         \
        static constexpr int LOAD = LD;        \
        static constexpr bool IFFT = I;        \
        static constexpr bool FD = F;          \
        static constexpr bool FFT = FF;        \
        static constexpr int STORE = ST;       \
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
    static constexpr int R = T > 4 ? 4 : T;               // row bits held in registers
    static constexpr int NR = 1 << R;                     // rows per thread
    static constexpr int W = T > 4 ? (1 << (T - 4)) : 1;  // waves per workgroup
    static constexpr int SHB = T - R;                     // layout B: k = w + (m << SHB)
    static constexpr int THREADS = 64 * W;
    static constexpr int NTAB = (1 << T) - 1;             // twiddle groups per direction
    // Tables of layers kb >= 4 (layout-B phase) come last: t >= TSPLIT.
    static constexpr int TSPLIT = T > 4 ? (1 << T) - (1 << (T - 4)) : 0;
};

// Dynamic LDS layout of program P at tile bits T (bytes):
//   [data tile: 2^T x 64 x 8][tab1: NTAB x 80][tab2: (NTAB - TSPLIT) x 80]
// tab1 holds the first direction's tables; in two-direction programs tab2
// holds the second direction's layout-B tables and its layout-A tables are
// restaged into tab1 once the first direction's layout-A phase is done.
template <int P, int T> struct Smem {
    using PT = ProgTraits<P>;
    static constexpr bool TWO = PT::IFFT && PT::FFT;
    static constexpr bool DATA = T > 4 || PT::FD || PT::LOAD == LD_DEC_LAST;
    static constexpr int DATA_BYTES = DATA ? (1 << T) * 64 * 8 : 0;
    static constexpr int TAB1_BYTES = Geo<T>::NTAB * 80;
    static constexpr int TAB2_BYTES = TWO ? (Geo<T>::NTAB - Geo<T>::TSPLIT) * 80 : 0;
    static constexpr int BYTES = DATA_BYTES + TAB1_BYTES + TAB2_BYTES;
};

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

__device__ __forceinline__ void ld_quad(const uint8_t* row, const Thr& c, uint32_t& L, uint32_t& H);
__device__ __forceinline__ void st_quad(uint8_t* row, const Thr& c, uint32_t L, uint32_t H);
__device__ __forceinline__ void ld_quad(const uint8_t* row, const Thr& c, uint32_t& L, uint32_t& H) {
#if defined(RS16_ABLATE) && RS16_ABLATE == 2
    L = (uint32_t)(uintptr_t)row ^ c.offL;
    H = L * 3u;
    return;
#endif
    if (c.active) {
        L = *(const uint32_t*)(row + c.offL);
        H = *(const uint32_t*)(row + c.offL + 32);
    } else {
        L = H = 0;
    }
}
__device__ __forceinline__ void st_quad(uint8_t* row, const Thr& c, uint32_t L, uint32_t H) {
#if defined(RS16_ABLATE) && RS16_ABLATE == 2
    if ((L ^ H) != 0x9e3779b9u) return;  // keeps the results live, (almost) never stores
#endif
    if (c.active) {
        *(uint32_t*)(row + c.offL) = L;
        *(uint32_t*)(row + c.offL + 32) = H;
    }
}

// Table of a twiddle from global memory into SGPRs (used for the per-row
// erasure multiplies, which are few).
__device__ __forceinline__ void load_table_global(uint32_t (&t)[20], const PassArgs& a, uint32_t e) {
    cu32p p = (cu32p)a.mul_tab + e * TAB_DWORDS;
#pragma unroll
    for (int i = 0; i < 20; i++) t[i] = p[i];
}

__device__ __forceinline__ void load_table_lds(uint32_t (&t)[20], const uint4* p) {
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const uint4 v = p[i];
        t[4 * i] = v.x;
        t[4 * i + 1] = v.y;
        t[4 * i + 2] = v.z;
        t[4 * i + 3] = v.w;
    }
}

// ---------------------------------------------------------------------------
// Twiddle-table staging.  Group id t in [0, 2^T-1): layer kb with
// offset(kb) = 2^T - 2^(T-kb) <= t < offset(kb+1), group j = t - offset(kb)
// covering tile rows k with k >> (kb+1) == j.
// ---------------------------------------------------------------------------
// Staging is split into issue (global loads into registers, issued next to
// the tile's own loads so their latencies overlap) and commit (ds_write,
// before the barrier that publishes the tables).  N = number of groups.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int T, int N> struct Stager {
    static constexpr int PER = (N * 5 + Geo<T>::THREADS - 1) / Geo<T>::THREADS;
    u32x4 v[PER > 0 ? PER : 1];
    int di[PER > 0 ? PER : 1];

    __device__ __forceinline__ void issue(int t_begin, int t_base, uint32_t skew, const Thr& c, const PassArgs& a) {
        const uint32_t* sk = a.skew_entry;
        const u32x4* tab = (const u32x4*)a.mul_tab;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int idx = (int)threadIdx.x + i * Geo<T>::THREADS;
            di[i] = -1;
            if (idx < N * 5) {
                const int t = t_begin + idx / 5, part = idx % 5;
                int kb = 0;
                while (t >= (1 << T) - (1 << (T - kb - 1))) kb++;
                const uint32_t j = (uint32_t)(t - ((1 << T) - (1 << (T - kb))));
                const uint32_t d = 1u << (a.lo + kb);
                const uint32_t g = (c.b_high << (a.lo + T)) + (j << (kb + 1 + a.lo));
                const uint32_t e = sk[g + d + skew - 1];
                v[i] = tab[(size_t)e * (TAB_DWORDS / 4) + part];
                di[i] = (t - t_base) * 5 + part;
            }
        }
    }
    __device__ __forceinline__ void commit(uint4* dst) const {
        u32x4* d = (u32x4*)dst;
#pragma unroll
        for (int i = 0; i < PER; i++)
            if (di[i] >= 0) d[di[i]] = v[i];
    }
};

// Layers for k-bits [KB0, KB1) held in registers of layout LB, as a
// compile-time sequence of twiddle groups (step s, index gi).
template <int T, bool LB, int KB0, int KB1, bool FFT> struct LayerSeq {
    static constexpr int SH = LB ? Geo<T>::SHB : 0;
    static constexpr int NR = Geo<T>::NR;
    static constexpr int kb_of(int s) { return FFT ? KB1 - 1 - s : KB0 + s; }
    static constexpr int groups_of(int s) { return NR >> (kb_of(s) - SH + 1); }
    static constexpr int total() {
        int n = 0;
        for (int s = 0; s < KB1 - KB0; s++) n += groups_of(s);
        return n;
    }
    static constexpr int step_of(int g) {
        int s = 0;
        while (g >= groups_of(s)) g -= groups_of(s), s++;
        return s;
    }
    static constexpr int index_of(int g) {
        int s = 0;
        while (g >= groups_of(s)) g -= groups_of(s), s++;
        return g;
    }
};

// Where group G's table lives: tile group id t = offset(kb) + j, with
// j = k >> (kb+1) of the group's rows; in two-direction kernels the second
// direction's layout-B tables are in tab2.
template <int T, bool LB, int KB0, int KB1, bool FFT, int G, bool IN_TAB2>
__device__ __forceinline__ const uint4* group_table(const Thr& c, const uint4* tab1, const uint4* tab2) {
    using S = LayerSeq<T, LB, KB0, KB1, FFT>;
    constexpr int s = S::step_of(G), gi = S::index_of(G);
    constexpr int kb = S::kb_of(s);
    constexpr int off = (1 << T) - (1 << (T - kb));
    // layout A: k = (w << R) + m  ->  j = (w << (R-1-kb)) + gi ; layout B: j = gi
    const uint32_t j = LB ? (uint32_t)gi : (c.w << (Geo<T>::R - 1 - kb)) + gi;
    const uint32_t t = off + j;
    if (IN_TAB2) return tab2 + (t - Geo<T>::TSPLIT) * 5;
    return tab1 + t * 5;
}

// Empty volatile asm that "redefines" the data registers: ALU work cannot
// cross it, so group boundaries are real scheduling boundaries.
template <int NR> __device__ __forceinline__ void pin_rows(uint32_t (&L)[NR], uint32_t (&H)[NR]) {
    if constexpr (NR >= 4) {
#pragma unroll
        for (int i = 0; i < NR; i += 4)
            asm volatile("" : "+v"(L[i]), "+v"(L[i + 1]), "+v"(L[i + 2]), "+v"(L[i + 3]), "+v"(H[i]), "+v"(H[i + 1]),
                         "+v"(H[i + 2]), "+v"(H[i + 3]));
    } else {
#pragma unroll
        for (int i = 0; i < NR; i++) asm volatile("" : "+v"(L[i]), "+v"(H[i]));
    }
}

template <int T, bool LB, int KB0, int KB1, bool FFT, bool IN_TAB2, int G> struct GroupLoop {
    static __device__ __forceinline__ void run(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                               const uint4* tab1, const uint4* tab2, const uint32_t (&cur)[20]) {
        using S = LayerSeq<T, LB, KB0, KB1, FFT>;
        constexpr int s = S::step_of(G), gi = S::index_of(G);
        constexpr int rb = S::kb_of(s) - S::SH;
        constexpr bool more = G + 1 < S::total();
        uint32_t nxt[20];
        if constexpr (more)
            load_table_lds(nxt, group_table<T, LB, KB0, KB1, FFT, G + 1, IN_TAB2>(c, tab1, tab2));
#pragma unroll
        for (int j = 0; j < (1 << rb); j++) {
            const int m = (gi << (rb + 1)) + j, m2 = m + (1 << rb);
            if (FFT) {
                mul_xor(L[m], H[m], L[m2], H[m2], cur);
                L[m2] ^= L[m];
                H[m2] ^= H[m];
            } else {
                L[m2] ^= L[m];
                H[m2] ^= H[m];
                mul_xor(L[m], H[m], L[m2], H[m2], cur);
            }
        }
        pin_rows<Geo<T>::NR>(L, H);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (more) GroupLoop<T, LB, KB0, KB1, FFT, IN_TAB2, G + 1>::run(L, H, c, tab1, tab2, nxt);
    }
};

// Apply the layers for k-bits [KB0, KB1) held in registers of layout LB.
// Diagnostic ablation builds (never the shipped library):
//   -DRS16_ABLATE=1  compile the butterfly layers out (memory + staging only)
//   -DRS16_ABLATE=2  compile HBM loads/stores out (compute only)
#ifndef RS16_ABLATE
#define RS16_ABLATE 0
#endif
template <int T, bool LB, int KB0, int KB1, bool FFT, bool IN_TAB2>
__device__ __forceinline__ void layers(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                       const uint4* tab1, const uint4* tab2) {
    if constexpr (KB1 > KB0 && RS16_ABLATE != 1) {
        uint32_t t0[20];
        load_table_lds(t0, group_table<T, LB, KB0, KB1, FFT, 0, IN_TAB2>(c, tab1, tab2));
        GroupLoop<T, LB, KB0, KB1, FFT, IN_TAB2, 0>::run(L, H, c, tab1, tab2, t0);
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

// y[k] ^= XOR_{b < T, k_b = 0} x[k | 2^b] with x read from LDS: the formal
// derivative restricted to the tile's row bits (Engine::formal_derivative,
// src/engine.rs:233-238, in closed form -- step i = (j & ~(2^b-1)) | 2^b XORs
// row j|2^b into row j, and that source row is never written before it is read).
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
    using SM = Smem<P, T>;
    constexpr int NR = Geo<T>::NR;
    constexpr int R = Geo<T>::R;
    constexpr bool TWO = SM::TWO;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint2* lds = (uint2*)smem;
    uint4* tab1 = (uint4*)(smem + SM::DATA_BYTES);
    uint4* tab2 = (uint4*)(smem + SM::DATA_BYTES + SM::TAB1_BYTES);

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

    uint32_t L[NR], H[NR];
    // IFFT starts with the low k bits (layout A), FFT with the high ones (B).
    constexpr bool START_B = !PT::IFFT;

    // ---------------- load ----------------
    if constexpr (PT::LOAD == LD_PLAIN) {
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t r = row_rel<T>(c, a, kidx<T, START_B>(c, m));
            ld_quad(a.in + (uint64_t)r * a.S, c, L[m], H[m]);
        }
    } else if constexpr (PT::LOAD == LD_GATHER_ENC) {
        // HighRateEncoder::encode: work[0..k) = originals, rest zero (rate_high.rs:50-54)
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t r = row_rel<T>(c, a, kidx<T, START_B>(c, m));
            if (r < a.a_count) ld_quad(a.seg_a + (uint64_t)r * a.S, c, L[m], H[m]);
            else L[m] = H[m] = 0;
        }
    } else if constexpr (PT::LOAD == LD_GATHER_DEC) {
        // "MULTIPLY SHARDS" of rate_high.rs:203-228 / rate_low.rs:203-228:
        // received rows * erasure log, everything else zero.
        uint32_t Y[NR][2];
        bool got[NR];
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
            got[m] = src != nullptr;
            if (src) ld_quad(src, c, Y[m][0], Y[m][1]);
            else Y[m][0] = Y[m][1] = 0;
        }
#pragma unroll
        for (int m = 0; m < NR; m++) {
            L[m] = H[m] = 0;
            if (got[m]) {
                const uint32_t r = row_rel<T>(c, a, kidx<T, START_B>(c, m));
                uint32_t tt[20];
                load_table_global(tt, a, uni(elog[r]));
                mul_xor(L[m], H[m], Y[m][0], Y[m][1], tt);
            }
        }
    } else {  // LD_DEC_LAST: y = u + L(z)  (formal-derivative part over the tile's bits)
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t k = kidx<T, START_B>(c, m);
            const uint32_t r = row_rel<T>(c, a, k);
            uint32_t zl, zh;
            ld_quad(a.in + (uint64_t)r * a.S, c, zl, zh);
            lds[k * 64 + c.lane] = make_uint2(zl, zh);
            ld_quad(a.in2 + (uint64_t)r * a.S, c, L[m], H[m]);
        }
    }
    // Stage the first direction's tables (and, in two-direction programs,
    // the second direction's layout-B tables); their loads overlap the tile's.
    {
        const uint32_t skew1 = PT::IFFT ? a.skew_ifft : a.skew_fft;
        Stager<T, Geo<T>::NTAB> s1;
        s1.issue(0, 0, skew1, c, a);
        if constexpr (TWO) {
            Stager<T, Geo<T>::NTAB - Geo<T>::TSPLIT> s2;
            s2.issue(Geo<T>::TSPLIT, Geo<T>::TSPLIT, a.skew_fft, c, a);
            s2.commit(tab2);
        }
        s1.commit(tab1);
    }
    __syncthreads();  // staged tables (and DEC_LAST's z tile) visible
    if constexpr (PT::LOAD == LD_DEC_LAST) {
        fd_from_lds<T, START_B>(L, H, c, lds);
        __syncthreads();
    }

    // ---------------- IFFT ----------------
    bool in_b = START_B;
    if constexpr (PT::IFFT) {
        layers<T, false, 0, R, false, false>(L, H, c, tab1, tab2);
        if constexpr (T > 4) {
            // stores A -> LDS, barrier, loads B (exchange writes first, so the
            // layout-A tables are dead after its first barrier)
            // Second direction's layout-A tables replace the first's (dead
            // once every wave has passed the exchange barrier below).
            Stager<T, (TWO ? Geo<T>::TSPLIT : 0)> s3;
            if constexpr (TWO) s3.issue(0, 0, a.skew_fft, c, a);
#pragma unroll
            for (int m = 0; m < NR; m++) lds[kidx<T, false>(c, m) * 64 + c.lane] = make_uint2(L[m], H[m]);
            __syncthreads();
            if constexpr (TWO) s3.commit(tab1);
#pragma unroll
            for (int m = 0; m < NR; m++) {
                uint2 v = lds[kidx<T, true>(c, m) * 64 + c.lane];
                L[m] = v.x;
                H[m] = v.y;
            }
            __syncthreads();
            layers<T, true, 4, (T > 4 ? T : 4), false, false>(L, H, c, tab1, tab2);
            in_b = true;
        }
    }
    // ---------------- formal derivative (tile bits) ----------------
    if constexpr (PT::FD) {
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
    if constexpr (PT::FFT) {
        if constexpr (T > 4) {
            layers<T, true, 4, (T > 4 ? T : 4), true, TWO>(L, H, c, tab1, tab2);
            exchange<T, true>(L, H, c, lds);
            in_b = false;
        }
        // two-direction, T <= 4: the whole second direction is in tab2
        layers<T, false, 0, R, true, (TWO && T <= 4)>(L, H, c, tab1, tab2);
    }

    // ---------------- store ----------------
    // Final layout: after FFT -> A; after IFFT only -> B (T > 4); T <= 4: A == B.
    constexpr bool END_B = !PT::FFT && T > 4;
#pragma unroll
    for (int m = 0; m < NR; m++) {
        const uint32_t r = row_rel<T>(c, a, kidx<T, END_B>(c, m));
        if constexpr (PT::STORE == ST_PLAIN) {
            st_quad(a.out + (uint64_t)r * a.S, c, L[m], H[m]);
        } else if constexpr (PT::STORE == ST_RECOVERY) {
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
                    uint32_t tt[20];
                    load_table_global(tt, a, GF_MODULUS - uni(elog[r]));
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

#define RS16_ROW(P)                                                                                            \
    {pass_kernel<P, 0>, pass_kernel<P, 1>, pass_kernel<P, 2>, pass_kernel<P, 3>, pass_kernel<P, 4>,             \
     pass_kernel<P, 5>, pass_kernel<P, 6>, pass_kernel<P, 7>, pass_kernel<P, 8>}
static const PassFn kPass[NUM_PROGS][9] = {
    RS16_ROW(GEN_FFT),    RS16_ROW(GEN_IFFT),  RS16_ROW(ENC_FIRST), RS16_ROW(ENC_MID),  RS16_ROW(ENC_LAST),
    RS16_ROW(ENC_SINGLE), RS16_ROW(DEC_FIRST), RS16_ROW(DEC_MID),   RS16_ROW(DEC_LAST), RS16_ROW(DEC_SINGLE),
};
#undef RS16_ROW

#define RS16_SM(P)                                                                                             \
    {Smem<P, 0>::BYTES, Smem<P, 1>::BYTES, Smem<P, 2>::BYTES, Smem<P, 3>::BYTES, Smem<P, 4>::BYTES,             \
     Smem<P, 5>::BYTES, Smem<P, 6>::BYTES, Smem<P, 7>::BYTES, Smem<P, 8>::BYTES}
static const int kSmem[NUM_PROGS][9] = {
    RS16_SM(GEN_FFT),    RS16_SM(GEN_IFFT),  RS16_SM(ENC_FIRST), RS16_SM(ENC_MID),  RS16_SM(ENC_LAST),
    RS16_SM(ENC_SINGLE), RS16_SM(DEC_FIRST), RS16_SM(DEC_MID),   RS16_SM(DEC_LAST), RS16_SM(DEC_SINGLE),
};
#undef RS16_SM

hipError_t launch_pass(int prog, int T, const PassArgs& a, uint32_t num_tiles, hipStream_t s) {
    if (prog < 0 || prog >= NUM_PROGS || T < 0 || T > 8) return hipErrorInvalidValue;
    if (num_tiles == 0) return hipSuccess;
    const int W = T > 4 ? (1 << (T - 4)) : 1;
    const size_t lds = (size_t)kSmem[prog][T];
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)kPass[prog][T], hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
        if (e != hipSuccess) return e;
    }
    dim3 grid(num_tiles * a.nslab), block(64 * W);
    hipLaunchKernelGGL(kPass[prog][T], grid, block, lds, s, a);
    return hipGetLastError();
}

}  // namespace rs16
