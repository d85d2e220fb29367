// rs16_pass.hip -- the HBM-pass kernels of the MI355X GF(2^16) Reed-Solomon
// engine: the FFT/IFFT butterflies of the reference `Engine`
// (src/engine/engine_nosimd.rs:190-384, spec src/engine/engine_naive.rs:43-124)
// fused with the Rate-level steps around them (src/rate/rate_high.rs:44-83,
// 168-247; src/rate/rate_low.rs:168-247).
//
// Structure of one pass
// ---------------------
//   A transform of 2^L rows runs in ceil(L/8) HBM passes.  A pass loads a
//   tile of 2^T rows (T <= 8) x Q quads (a quad = 4 elements = one lo dword
//   + one hi dword, rs16_gf.hpp; Q = 32 for T > 4, else 64), applies T layers
//   and stores it.  Tile t covers rows  b_low + (k << lo) + (b_high << (lo+T)),
//   k in [0, 2^T): lo = 0 gives contiguous tiles, lo > 0 strided ones.
//
//   Lane = quad.  Each thread keeps 16 rows ("a row set") of its quad in
//   VGPRs; a wave holds 64/Q row sets.  The 4 layers whose row bits are in
//   registers are radix-16 butterfly networks with no data movement; LDS
//   transposes switch between layout A (k bits 0-3 in registers) and layout B
//   (k bits T-4..T-1).  The transpose runs in NQR rounds of QL quads; NQR is
//   chosen per program (Rnd below) to bound a workgroup's LDS so that several
//   workgroups share a CU: one workgroup's HBM loads and stores overlap
//   another's butterflies.
//
//   Twiddle tables: a tile needs 2^T - 1 distinct twiddles per transform
//   direction (one per (layer, group)).  Their 80-byte v_perm multiply tables
//   are staged into LDS once per workgroup and read with ds_read_b128
//   (5 per group, broadcast within each row set), one group ahead of use.
//   Groups are compiled as a straight-line sequence separated by register
//   pins, so a wave holds at most two tables.  The decoder's per-row erasure
//   multipliers (gather and reveal) are staged the same way.
//
//   Butterflies (bit-exact spec, the reference's):
//     FFT  layer d: a ^= b * skew[r + d + skew_delta - 1];  b ^= a
//     IFFT layer d: b ^= a;  a ^= b * skew[r + d + skew_delta - 1]
//   r = group start (row & ~(2d-1)); the GF_MODULUS sentinel ("no multiply",
//   engine_naive.rs:64,116) maps to the all-zero table ZERO_ENTRY.
//
//   Decode zero tiles: a DEC_FIRST tile none of whose rows was received is
//   all zero after the erasure multiply (rate_high.rs:210-228 zero-fills
//   every row it does not multiply) and stays zero through its IFFT layers.
//   It is neither computed nor stored; its flag zflags[tile] = 1 tells
//   DEC_MID to read those rows as zero and to skip the IFFT groups whose rows
//   all are, and DEC_LAST that its z term is zero (y = u + L(z) = u).  At
//   100 % original loss this is the whole original half of the decode work.
#include "rs16_internal.hpp"

namespace rs16 {

typedef const __attribute__((address_space(4))) uint32_t* cu32p;

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

// Quads per tile row for T > 4 (32: a wave holds two 16-row sets of 32
// quads; 16: four row sets of 16 quads, half-size workgroups).
#ifndef RS16_QW
#define RS16_QW 32
#endif
template <int T> struct Geo {
    static constexpr int R = T > 4 ? 4 : T;               // row bits held in registers
    static constexpr int NR = 1 << R;                     // rows per thread (a row set)
    // quads per tile row (a workgroup needs SETS >= HWS: RS16_QW < 32 from T = 6)
    static constexpr int Q = T > 5 ? RS16_QW : (T > 4 ? 32 : 64);
    static constexpr int HWS = 64 / Q;                    // row sets per wave
    static constexpr int SETS = 1 << (T - R);             // row sets per tile
    static constexpr int W = SETS / HWS > 0 ? SETS / HWS : 1;  // waves per workgroup
    static constexpr int SHB = T - R;                     // layout B: k = s + (m << SHB)
    static constexpr int THREADS = 64 * W;
    static constexpr int NTAB = (1 << T) - 1;             // twiddle groups per direction
    // Tables of layers kb >= 4 (layout-B phase) come last: t >= TSPLIT.
    static constexpr int TSPLIT = T > 4 ? (1 << T) - (1 << (T - 4)) : 0;
};

// LDS rounds of the layout switches at T = 8 / T = 7 (diagnostic builds may
// override them).  The programs that stage reveal tables (DEC_LAST,
// DEC_SINGLE) keep 2 rounds at T = 8.
#ifndef RS16_NQR8
#define RS16_NQR8 2
#endif
#ifndef RS16_NQR7
#define RS16_NQR7 2
#endif
template <int P, int T> struct Rnd {
    static constexpr int NQR = T == 8 ? (ProgTraits<P>::STORE == ST_RESTORE ? 2 : RS16_NQR8)
                                      : (T == 7 ? RS16_NQR7 : 1);
    static constexpr int QL = Geo<T>::Q / NQR;
};

// Dynamic LDS layout of program P at tile bits T (bytes):
//   [region 0: data image 2^T x QL x 8 | gather multipliers 2^T x 80]
//   [tab1: NTAB x 80][tab2: (NTAB - TSPLIT) x 80]
//   [rvt: 2^T x 80 (reveal multipliers)][lost: 2^T x u32 (row is a lost original)]
// The gather multipliers are consumed right after the load, before the first
// layout switch writes the image (a barrier separates the two).  tab1 holds
// the first direction's tables; in two-direction programs tab2 holds the
// second direction's layout-B tables and its layout-A tables are restaged
// into tab1 once the first direction's layout-A phase is done.
template <int P, int T> struct Smem {
    using PT = ProgTraits<P>;
    static constexpr bool TWO = PT::IFFT && PT::FFT;
    static constexpr int IMG_BYTES = T > 4 ? (1 << T) * Rnd<P, T>::QL * 8 : 0;
    static constexpr int ERT_BYTES = PT::LOAD == LD_GATHER_DEC ? (1 << T) * 80 : 0;
    static constexpr int R0_BYTES = IMG_BYTES > ERT_BYTES ? IMG_BYTES : ERT_BYTES;
    static constexpr int TAB1_BYTES = Geo<T>::NTAB * 80;
    static constexpr int TAB2_BYTES = TWO ? (Geo<T>::NTAB - Geo<T>::TSPLIT) * 80 : 0;
    static constexpr int RVT_BYTES = PT::STORE == ST_RESTORE ? (1 << T) * 80 : 0;
    static constexpr int LOST_BYTES = PT::STORE == ST_RESTORE ? (1 << T) * 4 : 0;
    static constexpr int ERT_OFF = 0;
    static constexpr int TAB1_OFF = R0_BYTES;
    static constexpr int TAB2_OFF = TAB1_OFF + TAB1_BYTES;
    static constexpr int RVT_OFF = TAB2_OFF + TAB2_BYTES;
    static constexpr int LOST_OFF = RVT_OFF + RVT_BYTES;
    // erasure logs of the tile's rows when the pass finishes eval_poly (ework)
    static constexpr int ELOG_BYTES = ((P == DEC_FIRST || P == DEC_LAST) && T == 8) ? 256 * 4 : 0;
    static constexpr int ELOG_OFF = LOST_OFF + LOST_BYTES;
    static constexpr int BYTES = ELOG_OFF + ELOG_BYTES;
};

struct Thr {
    uint32_t lane, w, s;   // lane, wave, row set
    uint32_t qt;           // quad within the tile row
    uint32_t ql, round;    // quad within the LDS round, LDS round
    uint32_t b_low, b_high, offL;
    bool active;
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

template <int T, bool LB> __device__ __forceinline__ uint32_t kidx(const Thr& c, int m) {
    return LB ? c.s + ((uint32_t)m << Geo<T>::SHB) : (c.s << Geo<T>::R) + (uint32_t)m;
}

template <int T> __device__ __forceinline__ uint32_t row_rel(const Thr& c, const PassArgs& a, uint32_t k) {
    return c.b_low + (k << a.lo) + (c.b_high << (a.lo + T));
}

// Diagnostic ablation builds (never the shipped library):
//   -DRS16_ABLATE=1  compile the butterfly layers out (memory + staging only)
//   -DRS16_ABLATE=2  compile HBM loads/stores out (compute only)
//   -DRS16_ABLATE=3  as 1, and no table staging
//   -DRS16_ABLATE=4  as 1, and no LDS exchanges / formal derivative
#ifndef RS16_ABLATE
#define RS16_ABLATE 0
#endif
#ifndef RS16_NO_PIN
#define RS16_NO_PIN 0
#endif

__device__ __forceinline__ void ld_quad(const uint8_t* row, const Thr& c, uint32_t& L, uint32_t& H) {
#if RS16_ABLATE == 2
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
#if RS16_ABLATE == 2
    if ((L ^ H) != 0x9e3779b9u) return;  // keeps the results live, (almost) never stores
#endif
    if (c.active) {
        *(uint32_t*)(row + c.offL) = L;
        *(uint32_t*)(row + c.offL + 32) = H;
    }
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
// Table staging.  N tables of 5 x 16 B, table i taken from mul_tab entry
// entry(i), spread over the workgroup's threads.  Split into issue (global
// loads into registers, issued next to the tile's own loads so that their
// latencies overlap) and commit (ds_write, before the barrier that
// publishes the tables).
// ---------------------------------------------------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int T, int N> struct Stager {
    static constexpr int PER = (N * 5 + Geo<T>::THREADS - 1) / Geo<T>::THREADS;
    u32x4 v[PER > 0 ? PER : 1];

    template <class F> __device__ __forceinline__ void issue(const PassArgs& a, F entry) {
        if (RS16_ABLATE == 3) return;
        const u32x4* tab = (const u32x4*)a.mul_tab;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int idx = (int)threadIdx.x + i * Geo<T>::THREADS;
            if (idx < N * 5) v[i] = tab[(size_t)entry(idx / 5) * (TAB_DWORDS / 4) + idx % 5];
        }
    }
    __device__ __forceinline__ void commit(uint4* dst) const {
        if (RS16_ABLATE == 3) return;
        u32x4* d = (u32x4*)dst;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int idx = (int)threadIdx.x + i * Geo<T>::THREADS;
            if (idx < N * 5) d[idx] = v[i];
        }
    }
};

// Twiddle of tile group t (t in [0, 2^T - 1)): layer kb with
// offset(kb) = 2^T - 2^(T-kb) <= t < offset(kb+1), group j = t - offset(kb)
// covering tile rows k with k >> (kb+1) == j.
template <int T> struct TwiddleEntry {
    const PassArgs& a;
    const Thr& c;
    int t_begin;
    uint32_t skew;
    __device__ __forceinline__ uint32_t operator()(int i) const {
        const int t = t_begin + i;
        int kb = 0;
        while (t >= (1 << T) - (1 << (T - kb - 1))) kb++;
        const uint32_t j = (uint32_t)(t - ((1 << T) - (1 << (T - kb))));
        const uint32_t d = 1u << (a.lo + kb);
        const uint32_t g = (c.b_high << (a.lo + T)) + (j << (kb + 1 + a.lo));
        return a.skew_entry[g + d + skew - 1];
    }
};

// Received?  Rows [0, a_count) are segment A, [chunk, chunk + b_count)
// segment B; anything else is an absent (zero) row.
__device__ __forceinline__ bool row_received(const PassArgs& a, uint32_t r) {
    if (r < a.a_count) return !a.flags_a || a.flags_a[r];
    if (r >= a.chunk && r - a.chunk < a.b_count) return !a.flags_b || a.flags_b[r - a.chunk];
    return false;
}
// Lost original?  (the rows the decoder reveals)
__device__ __forceinline__ bool row_lost_original(const PassArgs& a, uint32_t r) {
    const uint32_t base = a.rest_seg_b ? a.chunk : 0;
    const uint32_t cnt = a.rest_seg_b ? a.b_count : a.a_count;
    const uint8_t* fl = a.rest_seg_b ? a.flags_b : a.flags_a;
    return r >= base && r - base < cnt && fl && !fl[r - base];
}

// "MULTIPLY SHARDS" of rate_high.rs:203-228 / rate_low.rs:203-228: received
// row r is multiplied by erasure log e[r]; absent rows by zero.
// e[r]: from the tile's LDS copy when the pass finished eval_poly itself
// (el = the tile's 2^T logs), else from HBM.
template <int T> struct GatherEntry {
    const PassArgs& a;
    const Thr& c;
    const uint32_t* el;
    __device__ __forceinline__ uint32_t operator()(int k) const {
        const uint32_t r = row_rel<T>(c, a, (uint32_t)k);
        return row_received(a, r) ? (el ? el[k] : a.elog[r]) : ZERO_ENTRY;
    }
};
// REVEAL ERASURES (rate_high.rs:236-242 / rate_low.rs:236-242): lost
// original row r -> work[r] * (GF_MODULUS - e[r]).
template <int T> struct RevealEntry {
    const PassArgs& a;
    const Thr& c;
    const uint32_t* el;
    __device__ __forceinline__ uint32_t operator()(int k) const {
        const uint32_t r = row_rel<T>(c, a, (uint32_t)k);
        return row_lost_original(a, r) ? GF_MODULUS - (el ? el[k] : a.elog[r]) : ZERO_ENTRY;
    }
};

// The last 256-point FWHT of eval_poly (src/engine.rs:207-218; row bits 0-7,
// add/sub mod 65535 as NoSimd::fwht_private, src/engine/engine_nosimd.rs:153-183)
// over a 256-row tile's values in LDS; every thread of the workgroup calls it.
__device__ __forceinline__ void fwht256_tile(uint32_t* s) {
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (uint32_t d = 1; d < 256; d <<= 1) {
        __syncthreads();
        if (t < 128) {
            const uint32_t i = (t / d) * 2 * d + (t % d), j = i + d;
            const uint32_t x = s[i], y = s[j];
            s[i] = add_mod(x, y);
            s[j] = sub_mod(x, y);
        }
    }
    __syncthreads();
}

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
// j = k >> (kb+1) of the group's rows (per row set in layout A, uniform in
// layout B); in two-direction kernels the second direction's layout-B
// tables are in tab2.
template <int T, bool LB, int KB0, int KB1, bool FFT, int G, bool IN_TAB2>
__device__ __forceinline__ const uint4* group_table(const Thr& c, const uint4* tab1, const uint4* tab2) {
    using S = LayerSeq<T, LB, KB0, KB1, FFT>;
    constexpr int s = S::step_of(G), gi = S::index_of(G);
    constexpr int kb = S::kb_of(s);
    constexpr int off = (1 << T) - (1 << (T - kb));
    // layout A: k = (s << R) + m  ->  j = (s << (R-1-kb)) + gi ; layout B: j = gi
    const uint32_t j = LB ? (uint32_t)gi : (c.s << (Geo<T>::R - 1 - kb)) + gi;
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

// PRUNE (layout-B groups of DEC_MID; the conditions are uniform):
//   PR_OUT  FFT: a group whose rows [gi << (kb+1), (gi+1) << (kb+1)) miss
//           [need_lo, need_hi) feeds no consumed output and is skipped;
//   PR_ZERO IFFT: a group whose rows are all zero on input stays zero and is
//           skipped.  zmask bit j = tile rows [16j, 16j+16) are all zero.
enum { PR_NONE = 0, PR_OUT, PR_ZERO };
template <int T, bool LB, int KB0, int KB1, bool FFT, bool IN_TAB2, int PRUNE, int G> struct GroupLoop {
    static __device__ __forceinline__ void run(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                               const PassArgs& a, const uint4* tab1, const uint4* tab2,
                                               const uint32_t (&cur)[20], uint32_t zmask) {
        using S = LayerSeq<T, LB, KB0, KB1, FFT>;
        constexpr int s = S::step_of(G), gi = S::index_of(G);
        constexpr int kb = S::kb_of(s);
        constexpr int rb = kb - S::SH;
        constexpr bool more = G + 1 < S::total();
        uint32_t nxt[20];
        if constexpr (more)
            load_table_lds(nxt, group_table<T, LB, KB0, KB1, FFT, G + 1, IN_TAB2>(c, tab1, tab2));
        __builtin_amdgcn_sched_barrier(0);  // the prefetch is issued before this group's work
        bool need = true;
        if constexpr (PRUNE == PR_OUT)
            need = ((uint32_t)gi << (kb + 1)) < a.need_hi && ((uint32_t)(gi + 1) << (kb + 1)) > a.need_lo;
        if constexpr (PRUNE == PR_ZERO) {
            static_assert(LB && kb >= 4, "zero pruning works on 16-row blocks of layout B");
            constexpr int nb = 1 << (kb - 3);  // 16-row blocks covered by the group
            constexpr uint32_t all = (uint32_t)((1ull << nb) - 1);
            need = ((zmask >> (gi * nb)) & all) != all;
        }
        if (need) {
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
        }
#if !RS16_NO_PIN
        pin_rows<Geo<T>::NR>(L, H);
#endif
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (more)
            GroupLoop<T, LB, KB0, KB1, FFT, IN_TAB2, PRUNE, G + 1>::run(L, H, c, a, tab1, tab2, nxt, zmask);
    }
};

// Apply the layers for k-bits [KB0, KB1) held in registers of layout LB.
template <int T, bool LB, int KB0, int KB1, bool FFT, bool IN_TAB2, int PRUNE = PR_NONE>
__device__ __forceinline__ void layers(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                       const PassArgs& a, const uint4* tab1, const uint4* tab2,
                                       uint32_t zmask = 0) {
    if constexpr (KB1 > KB0 && (RS16_ABLATE == 0 || RS16_ABLATE == 2)) {
        uint32_t t0[20];
        load_table_lds(t0, group_table<T, LB, KB0, KB1, FFT, 0, IN_TAB2>(c, tab1, tab2));
        GroupLoop<T, LB, KB0, KB1, FFT, IN_TAB2, PRUNE, 0>::run(L, H, c, a, tab1, tab2, t0, zmask);
    }
}

// LDS image of the data: row k, quad ql of the current round, as two planes
// (lo dwords, then hi dwords, PLANE dwords apart) so that a row's two dwords
// go through one ds_write2st64_b32 / ds_read2st64_b32 from independent
// registers (an interleaved uint2 image needs register pairs: v_mov copies).
template <int T, int QL> struct Img {
    static constexpr int PLANE = (1 << T) * QL;
    static __device__ __forceinline__ uint32_t* at(uint2* lds, const Thr& c, uint32_t k) {
        return (uint32_t*)lds + k * QL + c.ql;
    }
};

template <int NQR> __device__ __forceinline__ bool my_round(const Thr& c, int r) {
    return NQR == 1 || c.round == (uint32_t)r;
}

template <int T, int QL, bool LB>
__device__ __forceinline__ void put_rows(const uint32_t (&L)[Geo<T>::NR], const uint32_t (&H)[Geo<T>::NR],
                                         const Thr& c, uint2* lds) {
#pragma unroll
    for (int m = 0; m < Geo<T>::NR; m++) {
        uint32_t* p = Img<T, QL>::at(lds, c, kidx<T, LB>(c, m));
        p[0] = L[m];
        p[Img<T, QL>::PLANE] = H[m];
    }
}
template <int T, int QL, bool LB>
__device__ __forceinline__ void get_rows(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                         uint2* lds) {
#pragma unroll
    for (int m = 0; m < Geo<T>::NR; m++) {
        const uint32_t* p = Img<T, QL>::at(lds, c, kidx<T, LB>(c, m));
        L[m] = p[0];
        H[m] = p[Img<T, QL>::PLANE];
    }
}

// y[k] ^= XOR_{b < T, k_b = 0} x[k | 2^b]: the formal derivative restricted
// to the tile's row bits (Engine::formal_derivative, src/engine.rs:233-238,
// in closed form -- step i = (j & ~(2^b-1)) | 2^b XORs row j|2^b into row j,
// and that source row is never written before it is read).
// Terms of row bits held in registers come straight from registers: rows are
// updated in ascending m and a term's source row m | 2^b lies above m, so it
// is read before it is updated and y may alias x.  Terms of row-set bits
// differ between lanes: they are read from the LDS image of x
// unconditionally (for k_b = 1 the address is the row itself) and masked
// with a select, so all reads of a row issue back to back.
template <int T, int QL, bool LB>
__device__ __forceinline__ void fd_rows(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR],
                                        const uint32_t (&SL)[Geo<T>::NR], const uint32_t (&SH)[Geo<T>::NR],
                                        const Thr& c, uint2* lds) {
    constexpr int R = Geo<T>::R, SHB = Geo<T>::SHB;
#pragma unroll
    for (int m = 0; m < Geo<T>::NR; m++) {
        const uint32_t k = kidx<T, LB>(c, m);
        uint32_t xl = L[m], xh = H[m];
#pragma unroll
        for (int b = 0; b < T; b++) {
            // is bit b of k a register (compile-time) bit?
            const bool reg_bit = LB ? (b >= SHB) : (b < R);
            if (reg_bit) {
                const int mb = LB ? b - SHB : b;
                if (!((m >> mb) & 1)) {
                    xl ^= SL[m | (1 << mb)];
                    xh ^= SH[m | (1 << mb)];
                }
            } else {
                // bit sb of the row set s: above the lane-half bit it is a bit
                // of the (uniform) wave index, and a term not taken is skipped
                constexpr int LOG_HWS = Geo<T>::HWS == 4 ? 2 : (Geo<T>::HWS == 2 ? 1 : 0);
                const int sb = LB ? b : b - R;
                if (sb >= LOG_HWS) {
                    if (!((c.w >> (sb - LOG_HWS)) & 1)) {
                        const uint32_t* p = Img<T, QL>::at(lds, c, k | (1u << b));
                        xl ^= p[0];
                        xh ^= p[Img<T, QL>::PLANE];
                    }
                } else {
                    const uint32_t* p = Img<T, QL>::at(lds, c, k | (1u << b));
                    const uint32_t vl = p[0], vh = p[Img<T, QL>::PLANE];
                    const bool take = !((k >> b) & 1);
                    xl ^= take ? vl : 0u;
                    xh ^= take ? vh : 0u;
                }
            }
        }
        L[m] = xl;
        H[m] = xh;
    }
}

// Layout switch through LDS, in rounds.  `mid` runs after the first barrier
// (every wave is past its previous phase, so that phase's tables are dead).
template <int T, int NQR, bool FROM_B, class MID>
__device__ __forceinline__ void exchange(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                         uint2* lds, MID mid) {
    constexpr int QL = Geo<T>::Q / NQR;
    if (RS16_ABLATE == 4) return mid();
#pragma unroll
    for (int r = 0; r < NQR; r++) {
        if (my_round<NQR>(c, r)) put_rows<T, QL, FROM_B>(L, H, c, lds);
        __syncthreads();
        if (r == 0) mid();
        if (my_round<NQR>(c, r)) get_rows<T, QL, !FROM_B>(L, H, c, lds);
        __syncthreads();
    }
}

// y = x + (in-tile formal derivative part) of the rows in registers, where
// the LDS image is filled from (SL, SH) -- the rows themselves for the
// (I + H) step of DEC_MID, z for DEC_LAST's y = u + L(z).  In rounds; with
// T <= 4 every row bit is a register bit and no LDS is needed.
template <int T, int NQR, bool LB>
__device__ __forceinline__ void tile_fd(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR],
                                        const uint32_t (&SL)[Geo<T>::NR], const uint32_t (&SH)[Geo<T>::NR],
                                        const Thr& c, uint2* lds) {
    constexpr int QL = Geo<T>::Q / NQR;
    if (RS16_ABLATE == 4) return;
    if constexpr (T <= 4) {
        fd_rows<T, QL, LB>(L, H, SL, SH, c, lds);
    } else {
#pragma unroll
        for (int r = 0; r < NQR; r++) {
            if (my_round<NQR>(c, r)) put_rows<T, QL, LB>(SL, SH, c, lds);
            __syncthreads();
            if (my_round<NQR>(c, r)) fd_rows<T, QL, LB>(L, H, SL, SH, c, lds);
            __syncthreads();
        }
    }
}

template <int P, int T>
__global__ void __launch_bounds__(Geo<T>::THREADS, (P == DEC_SINGLE ? 1 : 4)) pass_kernel(PassArgs a) {
    using PT = ProgTraits<P>;
    using SM = Smem<P, T>;
    using G = Geo<T>;
    constexpr int NR = G::NR;
    constexpr int R = G::R;
    constexpr int NQR = Rnd<P, T>::NQR;
    constexpr int QL = Rnd<P, T>::QL;
    constexpr bool TWO = SM::TWO;
    constexpr bool ZERO_SKIP = P == DEC_MID && T > 4;  // DEC_MID runs with T >= 5 only
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint2* lds = (uint2*)smem;
    uint4* tab1 = (uint4*)(smem + SM::TAB1_OFF);
    uint4* tab2 = (uint4*)(smem + SM::TAB2_OFF);
    uint4* ert = (uint4*)(smem + SM::ERT_OFF);
    uint4* rvt = (uint4*)(smem + SM::RVT_OFF);
    uint32_t* lostf = (uint32_t*)(smem + SM::LOST_OFF);

    // Block -> (tile, slab), XCD-aware: blocks are dealt to the 8 XCDs
    // round-robin (XCD = b mod 8).  With a tile count that is a multiple of 8,
    // all slabs of a tile run on one XCD (they share their twiddle tables in
    // its L2) and consecutive tiles go to different XCDs, so tiles of uneven
    // work (DEC_FIRST zero tiles, pruned rows) spread evenly over the chip.
    const uint32_t b = blockIdx.x, ntiles = gridDim.x / a.nslab;
    uint32_t slab, tile;
    if ((ntiles & 7) == 0) {
        const uint32_t i = b >> 3;
        slab = i % a.nslab;
        tile = (i / a.nslab) * 8 + (b & 7);
    } else {
        slab = b % a.nslab;
        tile = b / a.nslab;
    }
    tile += a.tile_base;

    Thr c;
    c.lane = threadIdx.x & 63;
    c.w = uni(threadIdx.x >> 6);
    c.qt = c.lane % G::Q;
    c.s = c.w * G::HWS + c.lane / G::Q;
    c.ql = c.qt % QL;
    c.round = c.qt / QL;
    c.b_low = tile & ((1u << a.lo) - 1);
    c.b_high = tile >> a.lo;
    const uint32_t Qg = slab * G::Q + c.qt;
    c.active = Qg < a.qrow;
    c.offL = (Qg >> 3) * 64 + (Qg & 7) * 4;

    uint32_t L[NR], H[NR];
    // IFFT starts with the low k bits (layout A), FFT with the high ones (B).
    constexpr bool START_B = !PT::IFFT;
    // Final layout: after FFT -> A; after IFFT only -> B (T > 4); T <= 4: A == B.
    constexpr bool END_B = !PT::FFT && T > 4;

    // ---------------- zero rows of DEC_MID ----------------
    // Row r of this pass came from DEC_FIRST tile r >> lo = k + (b_high << T).
    // zrow bit m: this thread's (layout-A) row m is such a skipped, zero row;
    // zmask bit j: tile rows [16j, 16j+16) all are (uniform, scalar loads).
    uint32_t zrow = 0, zmask = 0;
    if constexpr (ZERO_SKIP) {
        if (a.zflags) {
            const uint8_t* zt = a.zflags + (c.b_high << T);
            const uint4 f = *(const uint4*)(zt + (c.s << R));
            const uint32_t fw[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
            for (int m = 0; m < NR; m++) zrow |= ((fw[m >> 2] >> (8 * (m & 3))) & 1u) << m;
            const cu32p zf = (cu32p)zt;
#pragma unroll
            for (int j = 0; j < G::SETS; j++)
                if ((zf[4 * j] & zf[4 * j + 1] & zf[4 * j + 2] & zf[4 * j + 3]) == 0x01010101u) zmask |= 1u << j;
        }
    }

    // ---------------- load ----------------
    constexpr int NZ = PT::LOAD == LD_DEC_LAST ? NR : 1;
    uint32_t zl[NZ], zh[NZ];
    bool rcv = false;    // DEC_FIRST: one of this thread's rows was received
    bool ztile = false;  // DEC_LAST: z of this tile is zero (DEC_FIRST skipped the tile)
    if constexpr (PT::LOAD == LD_PLAIN) {
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t r = row_rel<T>(c, a, kidx<T, START_B>(c, m));
            if ((zrow >> m) & 1u) L[m] = H[m] = 0;
            else ld_quad(a.in + (uint64_t)r * a.S, c, L[m], H[m]);
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
        // received rows (multiplied after the staging barrier), else zero
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t r = row_rel<T>(c, a, kidx<T, START_B>(c, m));
            L[m] = H[m] = 0;
            if (r < a.a_count) {
                if (!a.flags_a || a.flags_a[r]) {
                    rcv = true;
                    ld_quad(a.seg_a + (uint64_t)r * a.S, c, L[m], H[m]);
                }
            } else if (r >= a.chunk && r - a.chunk < a.b_count) {
                const uint32_t i = r - a.chunk;
                if (!a.flags_b || a.flags_b[i]) {
                    rcv = true;
                    ld_quad(a.seg_b + (uint64_t)i * a.S, c, L[m], H[m]);
                }
            }
        }
    } else {  // LD_DEC_LAST: u in registers, z for y = u + L(z)
        ztile = a.zflags && a.zflags[tile];
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t r = row_rel<T>(c, a, kidx<T, START_B>(c, m));
            if (ztile) zl[m] = zh[m] = 0;
            else ld_quad(a.in + (uint64_t)r * a.S, c, zl[m], zh[m]);
            ld_quad(a.in2 + (uint64_t)r * a.S, c, L[m], H[m]);
        }
    }
    if constexpr (P == DEC_FIRST) {
        if (blockIdx.x == 0 && a.zflags)  // tiles not launched: their segment was lost whole
            for (uint32_t t = threadIdx.x; t < a.ztiles; t += G::THREADS)
                if (t < a.zt_lo || t >= a.zt_hi) a.zflags[t] = 1;
        // A tile without received rows is zero after the erasure multiply
        // and through the IFFT: flag it for DEC_MID / DEC_LAST and stop
        // before staging anything.
        const int any = __syncthreads_or(rcv ? 1 : 0);
        if (a.zflags) {
            if (slab == 0 && threadIdx.x == 0) a.zflags[tile] = any ? 0 : 1;
            if (!any) return;
        }
    }
    // Erasure logs of this tile's rows: the last 256-point FWHT of eval_poly,
    // done here when the caller left it undone (ework); overlaps the tile loads.
    const uint32_t* el = nullptr;
    if constexpr (SM::ELOG_BYTES > 0) {
        if (a.ework) {
            uint32_t* elds = (uint32_t*)(smem + SM::ELOG_OFF);
            if (threadIdx.x < 256) elds[threadIdx.x] = a.ework[(tile << 8) + threadIdx.x];
            fwht256_tile(elds);
            el = elds;
        }
    }
    // Stage the first direction's tables (and, in two-direction programs,
    // the second direction's layout-B tables, and the decoder's per-row
    // multipliers); their loads overlap the tile's.
    {
        Stager<T, G::NTAB> s1;
        s1.issue(a, TwiddleEntry<T>{a, c, 0, PT::IFFT ? a.skew_ifft : a.skew_fft});
        if constexpr (TWO) {
            Stager<T, G::NTAB - G::TSPLIT> s2;
            s2.issue(a, TwiddleEntry<T>{a, c, G::TSPLIT, a.skew_fft});
            s2.commit(tab2);
        }
        if constexpr (PT::LOAD == LD_GATHER_DEC) {
            Stager<T, (1 << T)> se;
            se.issue(a, GatherEntry<T>{a, c, el});
            se.commit(ert);
        }
        if constexpr (PT::STORE == ST_RESTORE && !(PT::FFT && T > 4)) {
            Stager<T, (1 << T)> sr;
            sr.issue(a, RevealEntry<T>{a, c, el});
            const bool lf = threadIdx.x < (1u << T) && row_lost_original(a, row_rel<T>(c, a, threadIdx.x));
            sr.commit(rvt);
            if (threadIdx.x < (1u << T)) lostf[threadIdx.x] = lf;
        }
        s1.commit(tab1);
    }
    __syncthreads();  // staged tables visible
    if constexpr (PT::LOAD == LD_GATHER_DEC) {
#pragma unroll
        for (int m = 0; m < NR; m++) {
            uint32_t tt[20];
            load_table_lds(tt, ert + kidx<T, START_B>(c, m) * 5);
            const uint32_t yl = L[m], yh = H[m];
            L[m] = H[m] = 0;
            mul_xor(L[m], H[m], yl, yh, tt);
        }
    }
    if constexpr (PT::LOAD == LD_DEC_LAST) {
        if (!ztile) tile_fd<T, NQR, START_B>(L, H, zl, zh, c, lds);
    }

    // ---------------- IFFT ----------------
    bool in_b = START_B;
    if constexpr (PT::IFFT) {
        // DEC_MID: a wave whose rows all are zero skips its layout-A layers
        bool skip_a = false;
        if constexpr (ZERO_SKIP) skip_a = __all(zrow == (1u << NR) - 1);
        if (!skip_a) layers<T, false, 0, R, false, false>(L, H, c, a, tab1, tab2);
        if constexpr (T > 4) {
            // Two-direction programs: the second direction's layout-A tables
            // replace the first's, which are dead once every wave has passed
            // the exchange's first barrier.
            Stager<T, (TWO ? G::TSPLIT : 0)> s3;
            if constexpr (TWO) s3.issue(a, TwiddleEntry<T>{a, c, 0, a.skew_fft});
            // the gather multipliers share the image's LDS: every wave must be past them
            if constexpr (PT::LOAD == LD_GATHER_DEC) __syncthreads();
            exchange<T, NQR, false>(L, H, c, lds, [&]() {
                if constexpr (TWO) s3.commit(tab1);
            });
            layers<T, true, 4, (T > 4 ? T : 4), false, false, (ZERO_SKIP ? PR_ZERO : PR_NONE)>(L, H, c, a, tab1,
                                                                                                tab2, zmask);
            in_b = true;
        }
    }
    // ---------------- formal derivative (tile bits) ----------------
    if constexpr (PT::FD) {
        if (in_b) tile_fd<T, NQR, true>(L, H, L, H, c, lds);
        else tile_fd<T, NQR, false>(L, H, L, H, c, lds);
    }
    // ---------------- FFT ----------------
    if constexpr (PT::FFT) {
        if constexpr (T > 4) {
            // Reveal multipliers are staged late (T > 4), to keep their
            // registers out of the load phase.
            Stager<T, (PT::STORE == ST_RESTORE ? (1 << T) : 0)> sr;
            bool lf = false;
            if constexpr (PT::STORE == ST_RESTORE) {
                sr.issue(a, RevealEntry<T>{a, c, el});
                lf = threadIdx.x < (1u << T) && row_lost_original(a, row_rel<T>(c, a, threadIdx.x));
            }
            layers<T, true, 4, (T > 4 ? T : 4), true, TWO, (P == DEC_MID ? PR_OUT : PR_NONE)>(L, H, c, a, tab1,
                                                                                             tab2);
            exchange<T, NQR, true>(L, H, c, lds, [&]() {
                if constexpr (PT::STORE == ST_RESTORE) {
                    sr.commit(rvt);
                    if (threadIdx.x < (1u << T)) lostf[threadIdx.x] = lf;
                }
            });
            in_b = false;
        }
        // two-direction, T <= 4: the whole second direction is in tab2
        bool need = true;
        if constexpr (P == DEC_MID) need = (c.s << R) < a.need_hi && ((c.s + 1) << R) > a.need_lo;
        if (need) layers<T, false, 0, R, true, (TWO && T <= 4)>(L, H, c, a, tab1, tab2);
    }

    // ---------------- store ----------------
#pragma unroll
    for (int m = 0; m < NR; m++) {
        const uint32_t k = kidx<T, END_B>(c, m);
        const uint32_t r = row_rel<T>(c, a, k);
        if constexpr (PT::STORE == ST_PLAIN) {
            if (P != DEC_MID || (k >= a.need_lo && k < a.need_hi)) st_quad(a.out + (uint64_t)r * a.S, c, L[m], H[m]);
        } else if constexpr (PT::STORE == ST_RECOVERY) {
            if (r < a.out_rows) st_quad(a.out + (uint64_t)r * a.S, c, L[m], H[m]);
        } else {
            if (lostf[k]) {
                uint32_t tt[20];
                load_table_lds(tt, rvt + k * 5);
                uint32_t ol = 0, oh = 0;
                mul_xor(ol, oh, L[m], H[m], tt);
                const uint32_t i = r - (a.rest_seg_b ? a.chunk : 0);
                st_quad(a.rest + (uint64_t)i * a.S, c, ol, oh);
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

#define RS16_TH(P)                                                                                             \
    {Geo<0>::THREADS, Geo<1>::THREADS, Geo<2>::THREADS, Geo<3>::THREADS, Geo<4>::THREADS, Geo<5>::THREADS,       \
     Geo<6>::THREADS, Geo<7>::THREADS, Geo<8>::THREADS}
static const int kThreads[9] = RS16_TH(0);
static const int kQuads[9] = {Geo<0>::Q, Geo<1>::Q, Geo<2>::Q, Geo<3>::Q, Geo<4>::Q,
                              Geo<5>::Q, Geo<6>::Q, Geo<7>::Q, Geo<8>::Q};
#undef RS16_TH

hipError_t launch_pass(int prog, int T, const PassArgs& args, uint32_t num_tiles, hipStream_t s) {
    if (prog < 0 || prog >= NUM_PROGS || T < 0 || T > 8) return hipErrorInvalidValue;
    if (num_tiles == 0 || args.qrow == 0) return hipSuccess;
    PassArgs a = args;
    a.nslab = (a.qrow + kQuads[T] - 1) / kQuads[T];
    if (a.need_hi == 0) a.need_hi = 1u << T;  // no pruning
    const size_t lds = (size_t)kSmem[prog][T];
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)kPass[prog][T], hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
        if (e != hipSuccess) return e;
    }
    dim3 grid(num_tiles * a.nslab), block(kThreads[T]);
    hipLaunchKernelGGL(kPass[prog][T], grid, block, lds, s, a);
    return hipGetLastError();
}

}  // namespace rs16
