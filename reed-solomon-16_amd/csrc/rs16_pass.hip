// rs16_pass.hip -- the HBM-pass kernels of the MI355X GF(2^16) Reed-Solomon
// engine: the FFT/IFFT butterflies of the reference `Engine`
// (src/engine/engine_nosimd.rs:190-384, spec src/engine/engine_naive.rs:43-124)
// fused with the Rate-level steps around them (src/rate/rate_high.rs:44-83,
// 168-247; src/rate/rate_low.rs:168-247).
//
// Structure of one pass
// ---------------------
//   A transform of 2^L rows runs in ceil(L/8) HBM passes.  A pass works on
//   items: an item is a tile of 2^T rows (T <= 8) x Q quads (a quad = 4
//   elements = one lo dword + one hi dword, rs16_gf.hpp), loaded, run
//   through T layers and stored.  Tile t covers rows
//   b_low + (k << lo) + (b_high << (lo+T)), k in [0, 2^T): lo = 0 gives
//   contiguous tiles, lo > 0 strided ones; the slab of an item selects its Q
//   quads of the row.
//
//   One item per workgroup: the twiddle tables of the tile are requested
//   first and the tile's rows right behind them, then staged, computed and
//   stored (a software-pipelined persistent variant
//   measured slower at every T, CHANGELOG.md round 3).
//
//   Lane = quad.  Each thread keeps 16 rows ("a row set") of its quad in
//   VGPRs (8 at T = 5); a wave holds 64/Q row sets (Q = 32 quads per tile row
//   from T = 5 on: 2 row sets per wave).  The 4 layers whose row bits are in registers
//   are radix-16 butterfly networks with no data movement; an LDS transpose
//   switches between layout A (k bits 0-3 in registers) and layout B (k bits
//   T-4..T-1).
//
//   Twiddle tables: a tile needs 2^T - 1 distinct twiddles per transform
//   direction (one per (layer, group)).  Their 80-byte v_perm multiply tables
//   are staged into LDS (one level of loads from skew_tab) and read with ds_read_b128
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
//
//   Zero twiddles: the sentinel sits exactly at skew indices 2^i - 1, i.e. at
//   the first group of each layout-B layer of the two-direction passes; those
//   groups run the XOR half of the butterfly only (wave-uniform test).
//
//   Batched stripes (PassArgs::stripe_tiles): one launch covers independent
//   stripes of one geometry; a workgroup's tile index splits into (stripe,
//   tile within the stripe) and the stripe displaces its array pointers.
#include "rs16_internal.hpp"
#include "rs16_fwht.hpp"
#include "rs16_colops.hpp"
#include "rs16_diag.hpp"

namespace rs16 {

typedef const __attribute__((address_space(4))) uint32_t* cu32p;

// (timing A/B builds: -DRS16_NO_EARLY_B=1 keeps the IFFT-only passes' stores after the last block)
#ifndef RS16_NO_EARLY_B
#define RS16_NO_EARLY_B 0
#endif

enum LoadMode { LD_PLAIN = 0, LD_GATHER_ENC, LD_GATHER_DEC, LD_DEC_LAST };
enum StoreMode { ST_PLAIN = 0, ST_RECOVERY, ST_RESTORE };

// Store cache policy: non-temporal stores in the single-direction passes,
// plain stores in the two-direction passes (same-box A/B, CHANGELOG.md round 3:
// nt / sc1 / sc0 sc1 everywhere and nt loads all measured slower).
template <int P> struct ProgTraits;
#define RS16_PROG(P, LD, I, F, FF, ST)          \
    template <> struct ProgTraits<P> {         \
        static constexpr int LOAD = LD;        \
        static constexpr bool IFFT = I;        \
        static constexpr bool FD = F;          \
        static constexpr bool FFT = FF;        \
        static constexpr int STORE = ST;       \
        static constexpr bool ST_NT = !(I && FF);                                           \
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
RS16_PROG(DEC_HALF_LAST, LD_PLAIN, false, false, true, ST_RESTORE)
RS16_PROG(DEC_HALF_SINGLE, LD_GATHER_DEC, true, false, true, ST_RESTORE)
#undef RS16_PROG

// Quads per tile row of the T = 7 passes (the encoder's first / last
// passes and the identity decode's): 64 -- 8-wave workgroups, two per CU,
// 512 items for a 32768-row stripe, each twiddle table staged once per 64
// quad columns -- against 32 (4-wave workgroups, four per CU, 1024 items):
// same-box A/B x 8, 805-815 -> 797-838 GiB/s, mean +1.5 %, 6 of 8 pairs
// faster (profiles/r06_t7_q64_ab.txt).  (-DRS16_T7_Q=32: the old geometry.)
#ifndef RS16_T7_Q
#define RS16_T7_Q 64
#endif
// Row bits in registers: 4 (16 rows per thread) from T = 6 on; 3 at T = 5
// (the passes of the n <= 2048 codecs, which are latency-bound: 8 rows per
// thread and 16 quads per tile row give twice the waves, each with half the
// butterfly chain).  At T = 8 a tile row has 32 quads (8-wave workgroups,
// two per CU; 16 quads in 4-wave workgroups measured slower).
template <int T> struct Geo {
    static constexpr int R = T > 4 ? (T == 5 ? 3 : 4) : T;  // row bits held in registers
    static constexpr int NR = 1 << R;                     // rows per thread (a row set)
    static constexpr int SETS = 1 << (T - R);             // row sets per tile
    // quads per tile row: 32 (two 16-row sets per wave) from T = 6 on, 16
    // (four 8-row sets per wave) at T = 5, 64 (one row set) below
    static constexpr int Q = T > 4 ? (R == 3 ? 16 : (T == 7 ? RS16_T7_Q : 32)) : 64;
    static constexpr int HWS = 64 / Q;                    // row sets per wave
    static constexpr int W = SETS / HWS > 0 ? SETS / HWS : 1;  // waves per workgroup
    static constexpr int SHB = T - R;                     // layout B: k = s + (m << SHB)
    static constexpr int THREADS = 64 * W;
    static constexpr int NTAB = (1 << T) - 1;             // twiddle groups per direction
    // Tables of layers kb >= R (layout-B phase) come last: t >= TSPLIT.
    static constexpr int TSPLIT = T > 4 ? (1 << T) - (1 << (T - R)) : 0;
};

template <int P, int T, int QL> struct SmemL;
// The layout switch goes through an LDS image of 2^T rows x QL quads x 8
// bytes, in Q / QL rounds.  One round (4 barriers -> 2 per switch, every
// LDS instruction with all lanes) when the program's whole layout still lets
// two workgroups share a CU (<= 80 KiB: the T = 7 encode passes, 64-quad
// rows); else two rounds of Q / 2 quads (the T = 8 passes, the decoders' T =
// 7 passes with their multiplier tables).
#ifndef RS16_ONE_ROUND_MAX
#define RS16_ONE_ROUND_MAX (80 * 1024)
#endif
// The encoder's two-direction pass at T = 8 (ENC_MID, also the identity
// decode's middle pass): its one-round image (64 KiB) shares its LDS with
// the layout-A twiddle tables, which are dead during both layout switches
// (-DRS16_MID_SHARED=0: two rounds, tables beside the image).
#ifndef RS16_MID_SHARED
#define RS16_MID_SHARED 1
#endif
#ifndef RS16_DEC_MID_SHARED
#define RS16_DEC_MID_SHARED 1
#endif
template <int P, int T> struct Rnd {
    static constexpr int NQR = T >= 7 && SmemL<P, T, Geo<T>::Q>::BYTES > RS16_ONE_ROUND_MAX ? 2 : 1;
    static constexpr int QL = Geo<T>::Q / NQR;
};

// Dynamic LDS layout of program P at tile bits T (bytes):
//   [image: 2^T x QL x 8][ert: 2^T x 80 (gather multipliers)]
//   [tab1: NTAB x 80 (first direction)][tab2: NTAB x 80 (second direction)]
//   [rvt: 2^T x 80 (reveal multipliers)][lost: 2^T x u32 (row is a lost original)]
//   [elog: 256 x u32]
// Everything but the image is per tile key and stays resident across the
// items of that key.  At T = 8 the largest program (DEC_LAST) needs 75 KiB,
// so two workgroups share a CU.
template <int P, int T, int QL> struct SmemL {
    using PT = ProgTraits<P>;
    static constexpr bool TWO = PT::IFFT && PT::FFT;
    static constexpr int IMG_BYTES = T > 4 ? (1 << T) * QL * 8 : 0;
    // SHARED (ENC_MID at T = 8, one round): [image 64 KiB, holding the
    // layout-A tables of each direction outside the switches][IFFT layout-B
    // tables][FFT layout-B tables]
    static constexpr bool SHARED = RS16_MID_SHARED && (P == ENC_MID || (P == DEC_MID && RS16_DEC_MID_SHARED)) && T == 8 && QL == Geo<T>::Q;
    static constexpr int ERT_BYTES = PT::LOAD == LD_GATHER_DEC ? (1 << T) * 80 : 0;
    static constexpr int ERT_OFF = IMG_BYTES;
    static constexpr int TABB_OFF = IMG_BYTES;  // (SHARED: the IFFT's layout-B tables)
    static constexpr int TAB1_BYTES = SHARED ? 0 : Geo<T>::NTAB * 80;
    // Restage (one-item build, T > 4): tab2 holds only the second
    // direction's layout-B tables; its layout-A tables are written over the
    // first direction's in tab1 at the first layout switch.
    static constexpr bool RESTAGE = TWO && T > 4;
    static constexpr int TAB2_BYTES = TWO ? (RESTAGE ? Geo<T>::NTAB - Geo<T>::TSPLIT : Geo<T>::NTAB) * 80 : 0;
    static constexpr int RVT_BYTES = PT::STORE == ST_RESTORE ? (1 << T) * 80 : 0;
    static constexpr int LOST_BYTES = PT::STORE == ST_RESTORE ? (1 << T) * 4 : 0;
    static constexpr int TAB1_OFF = SHARED ? 0 : ERT_OFF + ERT_BYTES;
    static constexpr int TAB2_OFF = SHARED ? TABB_OFF + (Geo<T>::NTAB - Geo<T>::TSPLIT) * 80 : TAB1_OFF + TAB1_BYTES;
    static constexpr int RVT_OFF = TAB2_OFF + TAB2_BYTES;
    static constexpr int LOST_OFF = RVT_OFF + RVT_BYTES;
    // erasure logs of the tile's rows when the pass finishes eval_poly (ework)
    static constexpr int ELOG_BYTES = (PT::LOAD == LD_GATHER_DEC || PT::STORE == ST_RESTORE) ? 256 * 4 : 0;
    static constexpr int ELOG_OFF = LOST_OFF + LOST_BYTES;
    static constexpr int BYTES = ELOG_OFF + ELOG_BYTES;
};
template <int P, int T> struct Smem : SmemL<P, T, Rnd<P, T>::QL> {};

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
// row_rel(kidx(m)) split into a wave-uniform part (the row of the wave's
// first row set, in SGPRs) and the lane's row-set offset (a VGPR that does
// not depend on m): the HBM row addresses become one scalar multiply-add per
// row plus a per-lane byte offset computed once (PassArgs::voff32).
template <int T, bool LB> __device__ __forceinline__ uint32_t lane_rows(const Thr& c, const PassArgs& a) {
    const uint32_t hs = c.s - c.w * Geo<T>::HWS;  // row set within the wave
    return (LB ? hs : hs << Geo<T>::R) << a.lo;
}
// (the wave's row of row register 0, read into SGPRs once per item: a
// readfirstlane inside the per-row branches would be repeated per row)
template <int T, bool LB> struct WaveRows {
    uint32_t base, lo;
    __device__ __forceinline__ WaveRows(const Thr& c, const PassArgs& a) : lo(a.lo) {
        const uint32_t sw = uni(c.w) * Geo<T>::HWS;
        base = uni(c.b_low + (c.b_high << (a.lo + T)) + ((LB ? sw : sw << Geo<T>::R) << a.lo));
    }
    __device__ __forceinline__ uint32_t operator()(int m) const {
        return base + ((LB ? (uint32_t)m << Geo<T>::SHB : (uint32_t)m) << lo);
    }
};
// A wave-uniform row base address, pinned to SGPRs so that the compiler
// adds the lane offset in the load / store itself (SGPR base + VGPR offset)
// instead of folding the row product into a per-lane 64-bit multiply-add.
typedef __attribute__((address_space(1))) uint8_t gbyte;
typedef __attribute__((address_space(1))) uint32_t gu32;
__device__ __forceinline__ gbyte* sgpr_ptr(const uint8_t* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = uni((uint32_t)v), hi = uni((uint32_t)(v >> 32));
    return (gbyte*)(((uint64_t)hi << 32) | lo);
}
// r = ur + lr < lim for a uniform ur and a per-lane lr (one vector compare)
__device__ __forceinline__ bool row_below(uint32_t ur, uint32_t lr, uint32_t lim) {
    return ur < lim && lr < lim - ur;
}

// The last pass's lost-original tiles (2^T rows each) span at most tl_max
// tiles: tile_last_kernel is the last pass of the stripe (else DEC_LAST).
template <int T> __device__ __forceinline__ bool tl_covers(const PassArgs& a) {
    const uint32_t r0 = ((cu32p)a.lostrange)[0], r1 = ((cu32p)a.lostrange)[1];
    return r0 < r1 && ((r1 - 1) >> T) - (r0 >> T) < a.tl_max;
}

// The consumed U rows [nlo, nhi) of the general decode's middle pass, when
// at most MID_DIRECT_MAX (mid_direct_kernel: the direct product).
__device__ __forceinline__ bool mid_need(const PassArgs& a, uint32_t& nlo, uint32_t& nhi) {
    const uint32_t r0 = ((cu32p)a.lostrange)[0], r1 = ((cu32p)a.lostrange)[1];
    if (r0 >= r1) return false;
    nlo = max(a.need_lo, r0 >> a.lo);
    nhi = min(a.need_hi, ((r1 - 1) >> a.lo) + 1);
    return nhi > nlo && nhi - nlo <= MID_DIRECT_MAX;
}

// Priority schedule: a wave lowers its issue priority (s_setprio 3 -> 0) as
// its item progresses, so that waves that are behind win the arbitration.
// Hardware age order alone lets the oldest workgroup of a CU run ahead and
// leaves a low-occupancy one-workgroup tail (scripts/stamps.py: 10-16 us
// spread of workgroup end times).  Measured (bench, 2 runs each): this
// schedule 620 / 614 GiB/s; on the two-direction passes only 611 / 611; a
// later schedule 607; none 595 / 594.
// At point `at` of program P's item (0 staged, 1 first layout-A layers done,
// 2 first direction done, 3 layout-B FFT done, 4 last switch done, 5 stores).
// (A static pair schedule -- slots 0-1 at priority 3 for the whole item,
// slots 2-3 at 0 -- measured no better on the T = 7 passes and 3.5 us worse
// on the T = 8 ones, same-box A/B x 3, round 4.  Round 6, two workgroups per
// CU everywhere: without the schedule, or with a static bias for the younger
// workgroup, ENC_MID runs 2-3 us slower: profiles/r06_prio_schedules_rejected.txt.)
template <int P, int at, int T = 7> __device__ __forceinline__ void prio() {
    constexpr int v[6] = {3, 2, -1, 1, -1, 0};
    if constexpr (v[at] >= 0) __builtin_amdgcn_s_setprio(v[at]);
}


// s_waitcnt immediate (gfx9 encoding) that waits for vmcnt <= n only
// (expcnt and lgkmcnt at their maxima, i.e. not waited for).
__host__ __device__ constexpr int vmcnt_wait(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }

// Row loads / stores at an address that includes the lane's offset.
__device__ __forceinline__ void ld_ptr(const PassArgs& a, const gbyte* p, bool ok, uint32_t& L, uint32_t& H) {
    (void)a;
    L = H = 0;
    if (ok) {
        // (global address space from the SGPR base on: base + 32-bit lane
        // offset selects the SGPR-base form of global_load)
        const gu32* g = (const gu32*)p;
        L = g[0];
        H = g[8];
    }
}
template <bool NT>
__device__ __forceinline__ void st_ptr(const PassArgs& a, gbyte* p, bool ok, uint32_t L, uint32_t H) {
    (void)a;
    if (ok) {
        gu32* g = (gu32*)p;
        if constexpr (NT) {
            __builtin_nontemporal_store(L, g);
            __builtin_nontemporal_store(H, g + 8);
        } else {
            g[0] = L;
            g[8] = H;
        }
    }
}
// Branch-free: a row that is not read is read from the zero page instead
// (PassArgs::zero), so the item's loads are a fixed sequence and the
// compiler's vmcnt waits (for the staged tables and erasure logs, issued
// before the rows) count exactly instead of waiting for every row.
__device__ __forceinline__ void ld_sel(const PassArgs& a, const gbyte* p, bool ok, uint32_t offL, uint32_t& L,
                                       uint32_t& H) {
    // (offL & 0x7FFF: the zero page is RS16_ZERO_BYTES = 64 KiB, rows can be wider)
    const gu32* g = (const gu32*)(ok ? p : (const gbyte*)a.zero + (offL & 0x7FFFu));
    L = g[0];
    H = g[8];
}
// Per-lane byte offset of the lane's quad in the row lane_rows below the
// wave's row: 32 bits (global_load/store with an SGPR base) when the launch
// allows it (PassArgs::voff32), else 64 bits.
template <bool V32> struct LaneOff {
    uint32_t v;
    __device__ __forceinline__ LaneOff(uint32_t lr, uint64_t S, uint32_t offL) : v(lr * (uint32_t)S + offL) {}
    template <class B> __device__ __forceinline__ B* at(B* base) const { return base + v; }
};
template <> struct LaneOff<false> {
    uint64_t v;
    __device__ __forceinline__ LaneOff(uint32_t lr, uint64_t S, uint32_t offL) : v((uint64_t)lr * S + offL) {}
    template <class B> __device__ __forceinline__ B* at(B* base) const { return base + v; }
};

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

    // table i = entry(i) of `tabs` (TAB_DWORDS dwords per entry)
    template <class F> __device__ __forceinline__ void issue(const uint32_t* tabs, F entry) {
        const u32x4* tab = (const u32x4*)tabs;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int idx = (int)threadIdx.x + i * Geo<T>::THREADS;
            if (idx < N * 5) v[i] = tab[(size_t)entry(idx / 5) * (TAB_DWORDS / 4) + idx % 5];
        }
    }
    __device__ __forceinline__ void commit(uint4* dst) const {
        u32x4* d = (u32x4*)dst;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int idx = (int)threadIdx.x + i * Geo<T>::THREADS;
            if (idx < N * 5) d[idx] = v[i];
        }
    }
};

// Twiddle of tile group t (t in [0, 2^T - 1)) as an index of skew_tab (the
// v_perm table of every skew entry, so staging is one load deep): layer kb with
// offset(kb) = 2^T - 2^(T-kb) <= t < offset(kb+1), group j = t - offset(kb)
// covering tile rows k with k >> (kb+1) == j.
template <int T> struct TwiddleEntry {
    const PassArgs& a;
    const Thr& c;
    int t_begin;
    uint32_t skew;
    __device__ __forceinline__ uint32_t operator()(int i) const {
        const int t = t_begin + i;
        // kb = T - 1 - floor(log2(2^T - 1 - t)) (closed form, so the staging
        // loads of a thread issue back to back)
        const int kb = T - 32 + __clz((uint32_t)((1 << T) - 1 - t));
        const uint32_t j = (uint32_t)(t - ((1 << T) - (1 << (T - kb))));
        const uint32_t d = 1u << (a.lo + kb);
        const uint32_t g = (c.b_high << (a.lo + T)) + (j << (kb + 1 + a.lo));
        return g + d + skew - 1;
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
// Decoder rows: pass row r is decode work row r + row_base_in (gather side)
// or r + row_base_out (reveal side) -- non-zero in the half-transform decode.
template <int T> struct GatherEntry {
    const PassArgs& a;
    const Thr& c;
    const uint32_t* el;
    __device__ __forceinline__ uint32_t operator()(int k) const {
        const uint32_t r = row_rel<T>(c, a, (uint32_t)k) + a.row_base_in;
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
        const uint32_t r = row_rel<T>(c, a, (uint32_t)k) + a.row_base_out;
        return row_lost_original(a, r) ? GF_MODULUS - (el ? el[k] : a.elog[r]) : ZERO_ENTRY;
    }
};

// The last 256-point FWHT of eval_poly (src/engine.rs:207-218; row bits 0-7,
// add/sub mod 65535 as NoSimd::fwht_private, src/engine/engine_nosimd.rs:153-183)
// over the 256-row block of a tile's rows in LDS; every thread of the
// workgroup (NT of them) calls it.
template <int NT> __device__ __forceinline__ void fwht256_tile(uint32_t* s) {
#pragma unroll
    for (uint32_t d = 1; d < 256; d <<= 1) {
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < 128; t += NT) {
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
// No per-group action (GroupLoop's default).
struct NoFin {
    template <class X> __device__ __forceinline__ void operator()(const X&, const X&, int) const {}
};

// Breadth-first (layer by layer), except the last FFT block in layout A of
// all 4 register bits: there the groups run depth-first in pre-order (a
// group, then its two halves), so rows m, m + 1 are final right after their
// layer-0 group and can be stored there (EarlyStore).
template <int T, bool LB, int KB0, int KB1, bool FFT> struct LayerSeq {
    static constexpr int SH = LB ? Geo<T>::SHB : 0;
    static constexpr int NR = Geo<T>::NR;
    static constexpr bool DF = FFT && !LB && KB0 == 0 && KB1 == Geo<T>::R && NR >= 8;
    // pre-order of the group tree (node (kb, gi), children (kb-1, 2gi) and
    // (kb-1, 2gi+1)), (kb, gi) packed as kb * 16 + gi; radix 16:
    // (3,0) (2,0) (1,0) (0,0) (0,1) (1,1) (0,2) (0,3) (2,1) (1,2) ...
    static constexpr int df_at(int g) {
        int skb[16] = {}, sgi[16] = {};
        int sp = 0, n = 0;
        skb[sp] = KB1 - 1, sgi[sp] = 0, sp++;
        while (sp > 0) {
            sp--;
            const int kb = skb[sp], gi = sgi[sp];
            if (n++ == g) return kb * 16 + gi;
            if (kb > 0) {
                skb[sp] = kb - 1, sgi[sp] = 2 * gi + 1, sp++;
                skb[sp] = kb - 1, sgi[sp] = 2 * gi, sp++;
            }
        }
        return 0;
    }
    static constexpr int kb_of(int s) { return FFT ? KB1 - 1 - s : KB0 + s; }
    static constexpr int groups_of(int s) { return NR >> (kb_of(s) - SH + 1); }
    static constexpr int total() {
        int n = 0;
        for (int s = 0; s < KB1 - KB0; s++) n += groups_of(s);
        return n;
    }
    static constexpr int step_of(int g) {
        if (DF) return KB1 - 1 - df_at(g) / 16;
        int s = 0;
        while (g >= groups_of(s)) g -= groups_of(s), s++;
        return s;
    }
    static constexpr int index_of(int g) {
        if (DF) return df_at(g) % 16;
        int s = 0;
        while (g >= groups_of(s)) g -= groups_of(s), s++;
        return g;
    }
};

// Where group G's table lives: tile group id t = offset(kb) + j, with
// j = k >> (kb+1) of the group's rows (per row set in layout A, uniform in
// layout B); in two-direction kernels the second direction's tables are in
// tab2.
template <int T, bool LB, int KB0, int KB1, bool FFT, int G, bool IN_TAB2>
__device__ __forceinline__ const uint4* group_table(const Thr& c, const uint4* tab1, const uint4* tab2) {
    using S = LayerSeq<T, LB, KB0, KB1, FFT>;
    constexpr int s = S::step_of(G), gi = S::index_of(G);
    constexpr int kb = S::kb_of(s);
    constexpr int off = (1 << T) - (1 << (T - kb));
    // layout A: k = (s << R) + m  ->  j = (s << (R-1-kb)) + gi ; layout B: j = gi
    const uint32_t j = LB ? (uint32_t)gi : (c.s << (Geo<T>::R - 1 - kb)) + gi;
    const uint32_t t = off + j;
    // tab2 starts at the first layout-B table when the layout-A ones are
    // restaged into tab1 (Smem::RESTAGE); T <= 4 has no layout B (TSPLIT = 0)
    constexpr uint32_t base2 = T > 4 ? Geo<T>::TSPLIT : 0;
    return IN_TAB2 ? tab2 + (t - base2) * 5 : tab1 + t * 5;
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
template <int P, int T, bool LB, int KB0, int KB1, bool FFT, bool IN_TAB2, int PRUNE, int G, class FIN = NoFin>
struct GroupLoop {
    static __device__ __forceinline__ void run(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                               const PassArgs& a, const uint4* tab1, const uint4* tab2,
                                               const uint32_t (&cur)[20], uint32_t zmask, const FIN& fin = FIN()) {
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
        // Zero twiddle (the reference's GF_MODULUS sentinel: XOR only, no
        // multiply, engine_naive.rs:64,116).  The sentinel skew entries are
        // exactly the indices 2^i - 1 (rs16_tables.cpp checks this when it
        // builds the tables), which only the first group of a layer-B layer
        // can hit (index = b_high 2^(lo+T) + (2 gi + 1) 2^(lo+kb) + skew - 1):
        // ENC_MID's FFT half and the half decode's IFFT half (skew 0, b_high
        // 0) skip 15 of their 128 multiplies per row set this way.  Layout-B
        // twiddles are uniform, so this is a uniform branch.
        bool mul = true;
        if constexpr (LB && gi == 0 && ProgTraits<P>::IFFT && ProgTraits<P>::FFT) {
            const uint32_t idx = (c.b_high << (a.lo + T)) + (1u << (a.lo + kb)) + (FFT ? a.skew_fft : a.skew_ifft) - 1;
            mul = (idx & (idx + 1)) != 0;
        }
        if (need && mul) {
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
        } else if (need) {
#pragma unroll
            for (int j = 0; j < (1 << rb); j++) {
                const int m = (gi << (rb + 1)) + j, m2 = m + (1 << rb);
                L[m2] ^= L[m];
                H[m2] ^= H[m];
            }
        }
        // (only the group's own rows: a row of a later group may still be
        // in flight from HBM, and pinning it here would make the compiler
        // wait for every row load before the second group of the first layer)
#pragma unroll
        for (int j = 0; j < (1 << rb); j++) {
            const int m = (gi << (rb + 1)) + j, m2 = m + (1 << rb);
            asm volatile("" : "+v"(L[m]), "+v"(H[m]), "+v"(L[m2]), "+v"(H[m2]));
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (S::DF && kb == 0) fin(L, H, gi << 1);  // rows 2 gi, 2 gi + 1 are final
        if constexpr (more)
            GroupLoop<P, T, LB, KB0, KB1, FFT, IN_TAB2, PRUNE, G + 1, FIN>::run(L, H, c, a, tab1, tab2, nxt, zmask, fin);
    }
};

// A uniform LDS address held in one VGPR.  Layout-B table addresses are
// compile-time constants; left to the compiler, each ds_read gets its own
// s_add + v_mov to build the address (150 VALU moves per ENC_MID item).
// Through one opaque VGPR base the constant part folds into the ds_read
// offset field instead.
__device__ __forceinline__ const uint4* lds_vgpr(const uint4* p) {
#ifndef RS16_NO_LDS_VBASE
    uint32_t v = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint4*)p;
    asm volatile("" : "+v"(v));
    return (const uint4*)(const __attribute__((address_space(3))) uint4*)(uintptr_t)v;
#else
    return p;
#endif
}

// Apply the layers for k-bits [KB0, KB1) held in registers of layout LB.
template <int P, int T, bool LB, int KB0, int KB1, bool FFT, bool IN_TAB2, int PRUNE = PR_NONE, class FIN = NoFin>
__device__ __forceinline__ void layers(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                       const PassArgs& a, const uint4* tab1, const uint4* tab2,
                                       uint32_t zmask = 0, const FIN& fin = FIN()) {
    if constexpr (KB1 > KB0) {
        if constexpr (LB) {
            if constexpr (IN_TAB2) tab2 = lds_vgpr(tab2);
            else tab1 = lds_vgpr(tab1);
        }
        uint32_t t0[20];
        load_table_lds(t0, group_table<T, LB, KB0, KB1, FFT, 0, IN_TAB2>(c, tab1, tab2));
        GroupLoop<P, T, LB, KB0, KB1, FFT, IN_TAB2, PRUNE, 0, FIN>::run(L, H, c, a, tab1, tab2, t0, zmask, fin);
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

// Layout switch through LDS, in rounds.  `mid` runs after the first barrier.
struct NoMid {
    __device__ __forceinline__ void operator()() const {}
};
// `post` runs in the thread's own round after its rows are read (the image
// of that round is still in place).
template <int T, int NQR, bool FROM_B, class MID = NoMid, class POST = NoMid>
__device__ __forceinline__ void exchange(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                         uint2* lds, MID mid = MID(), POST post = POST()) {
    constexpr int QL = Geo<T>::Q / NQR;
#pragma unroll
    for (int r = 0; r < NQR; r++) {
        if (my_round<NQR>(c, r)) put_rows<T, QL, FROM_B>(L, H, c, lds);
        __syncthreads();
        if (r == 0) mid();
        if (my_round<NQR>(c, r)) {
            get_rows<T, QL, !FROM_B>(L, H, c, lds);
            post();
        }
        __syncthreads();
    }
}

// DEC_MID's second layout switch when its consumed rows lie in the
// layout-B register rows [m0, m0 + ND) (fd_few): only those rows go through
// LDS -- every thread writes ND rows, the threads whose layout-A rows they
// are read them -- in one round with one barrier, instead of all 2^T rows
// in two rounds.  The other threads' rows are not consumed (the layout-A
// FFT layers skip them, the store masks them).
template <int T, int ND>
__device__ __forceinline__ void few_switch(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const Thr& c,
                                           uint2* lds, uint32_t m0) {
    constexpr int Q = Geo<T>::Q, SHB = Geo<T>::SHB, R = Geo<T>::R, NR = Geo<T>::NR;
    constexpr uint32_t ROWS = (uint32_t)ND << SHB, PLANE = ROWS * Q;
    uint32_t* img = (uint32_t*)lds;
    const uint32_t base = m0 << SHB;
#pragma unroll
    for (int m = 0; m < NR; m++) {
        const uint32_t i = (uint32_t)m - m0;  // (uniform)
        if (i < (uint32_t)ND) {
            const uint32_t r = c.s + (i << SHB);  // layout B: k = s + (m << SHB)
            img[r * Q + c.qt] = L[m];
            img[PLANE + r * Q + c.qt] = H[m];
        }
    }
    __syncthreads();
    const uint32_t k0 = c.s << R;  // layout A: k = (s << R) + m
    if (k0 >= base && k0 < base + ROWS) {
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t r = k0 - base + (uint32_t)m;
            L[m] = img[r * Q + c.qt];
            H[m] = img[PLANE + r * Q + c.qt];
        }
    }
}

// DEC_MID's formal derivative split by row bits (the two-direction pass's
// layers: IFFT bits [0, R) in layout A, bits [R, T) in layout B, then the
// FFT back).  With w = the rows after the layout-A IFFT layers, z = M_B(w)
// after the layout-B ones, and F_B the layout-B FFT layers (F_B M_B = I:
// same twiddles, inverse butterflies), a term P_b (row k|2^b into row k,
// k_b = 0) of a bit b < R commutes with the butterflies of bits above b, so
//   F_B((I + sum_b P_b) z) = F_B((I + sum_{b >= R} P_b) z) + sum_{b < R} P_b w:
// the terms of the layout-B bits come from registers after the layout-B
// IFFT layers (fd_regs), those of the layout-A bits from the image of w that
// the first layout switch writes anyway (fd_image, read in the switch), and
// they are added to the FFT's rows after its layout-B layers.  No LDS round
// of its own, no barrier.  (DEC_LAST's y = u + L(z) is the same identity one
// pass up: tile_last_kernel.)
template <int T>
__device__ __forceinline__ void fd_regs(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR]) {
    constexpr int R = Geo<T>::R, SHB = Geo<T>::SHB;
#pragma unroll
    for (int m = 0; m < Geo<T>::NR; m++) {
#pragma unroll
        for (int b = R; b < T; b++) {
            const int mb = b - SHB;  // layout B: k = s + (m << SHB)
            if (!((m >> mb) & 1)) {  // the source row m | 2^mb is updated later
                L[m] ^= L[m | (1 << mb)];
                H[m] ^= H[m | (1 << mb)];
            }
        }
    }
}
// XOR_{b < R, k_b = 0} w[k | 2^b] from the image of w (any layout: the image
// is indexed by tile row)
template <int T, int QL>
__device__ __forceinline__ void fd_image(uint32_t& dl, uint32_t& dh, const Thr& c, const uint2* lds, uint32_t k) {
    dl = dh = 0;
#pragma unroll
    for (int b = 0; b < Geo<T>::R; b++) {
        const uint32_t* p = Img<T, QL>::at((uint2*)lds, c, k | (1u << b));
        const uint32_t vl = p[0], vh = p[Img<T, QL>::PLANE];
        const bool take = !((k >> b) & 1);
        dl ^= take ? vl : 0u;
        dh ^= take ? vh : 0u;
    }
}

// Two-direction programs of the one-item build (Smem::RESTAGE): the second
// direction's layout-A tables are requested before the first layout switch
// and written over the first direction's layout-A tables (dead by then) in
// tab1 between its barriers.
template <int P, int T> struct LateS2 {
    static constexpr bool value = Smem<P, T>::RESTAGE;
};

// y = x + (in-tile formal derivative part) of the rows in registers, where
// the LDS image is filled from (SL, SH) -- the rows themselves for the
// (I + H) step of DEC_MID, z for DEC_LAST's y = u + L(z).  In rounds; with
// T <= 4 every row bit is a register bit and no LDS is needed.
template <int T, int NQR, bool LB>
__device__ __forceinline__ void tile_fd(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR],
                                        const uint32_t (&SL)[Geo<T>::NR], const uint32_t (&SH)[Geo<T>::NR],
                                        const Thr& c, uint2* lds) {
    constexpr int QL = Geo<T>::Q / NQR;
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

// One item's rows in registers plus what the item's load learned.
template <int P, int T> struct ItemRegs {
    static constexpr int NR = Geo<T>::NR;
    static constexpr int NZ = ProgTraits<P>::LOAD == LD_DEC_LAST ? NR : 1;
    uint32_t L[NR], H[NR];
    uint32_t zl[NZ], zh[NZ];  // DEC_LAST: z rows for y = u + L(z)
    uint32_t zrow, zmask;     // DEC_MID zero rows (see below)
    bool ztile;               // DEC_LAST: z of this tile is zero (DEC_FIRST skipped it)
};

// Per-item coordinates of this thread: item -> (tile, slab).
__device__ __forceinline__ void set_item(Thr& c, const PassArgs& a, uint32_t item, uint32_t Q, uint32_t& tile,
                                         uint32_t& slab) {
    // One item per workgroup, XCD-aware: workgroups are dealt to the 8 XCDs
    // round-robin (XCD = block mod 8, speed only), so with a tile count that
    // is a multiple of 8 all slabs of a tile run on one XCD (they share the
    // tile's twiddle tables in its L2) and consecutive tiles go to different
    // XCDs (tiles of uneven work spread evenly).
    if ((a.ntiles & 7) == 0) {
        const uint32_t i = item >> 3;
        slab = i % a.nslab;
        tile = (i / a.nslab) * 8 + (item & 7);
    } else {
        tile = item / a.nslab;
        slab = item - tile * a.nslab;
    }
    const uint32_t Qg = slab * Q + c.qt;
    c.active = Qg < a.qrow;
    c.offL = (Qg >> 3) * 64 + (Qg & 7) * 4;
}

// The one-item build's row loads of an item: row address = SGPR base of the
// wave's row (one scalar multiply-add per row) + the lane's offset.
template <int P, int T, bool V32>
__device__ __forceinline__ void load_rows(const PassArgs& a, const Thr& c, uint32_t tile, ItemRegs<P, T>& d) {
    using PT = ProgTraits<P>;
    using G = Geo<T>;
    constexpr int NR = G::NR, R = G::R;
    constexpr bool START_B = !PT::IFFT;
    const uint32_t lr = lane_rows<T, START_B>(c, a);
    const WaveRows<T, START_B> wr(c, a);
    if constexpr (PT::LOAD == LD_PLAIN) {
        const LaneOff<V32> lo(lr, a.S_in, c.offL);
#pragma unroll
        for (int m = 0; m < NR; m++) {
            // (in_rows_mask: every chunk of the launch reads the one chunk at in)
            const uint32_t ur = a.in_rows_mask ? (wr(m) & a.in_rows_mask) : wr(m);
            ld_sel(a, lo.at(sgpr_ptr(a.in + (uint64_t)ur * a.S_in)), c.active & !((d.zrow >> m) & 1u), c.offL, d.L[m], d.H[m]);
        }
    } else if constexpr (PT::LOAD == LD_GATHER_ENC) {
        // HighRateEncoder::encode: work[0..k) = originals, rest zero (rate_high.rs:50-54)
        const LaneOff<V32> lo(lr, a.S_seg, c.offL);
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t ur = wr(m);
            ld_sel(a, lo.at(sgpr_ptr(a.seg_a + (uint64_t)ur * a.S_seg)), c.active & row_below(ur, lr, a.a_count),
                   c.offL, d.L[m], d.H[m]);
        }
    } else if constexpr (PT::LOAD == LD_GATHER_DEC) {
        // received rows (multiplied by their erasure logs in process_item), else
        // zero.  Received bits of the wave's rows: rows [row0, row0 + 16 HWS)
        // of the bitmap (row0 a multiple of 16, of 32 when HWS > 1), scalar loads.
        static_assert(START_B == false && T <= 8, "gather runs in layout A");
        const uint32_t row0 = row_rel<T>(c, a, (c.w * G::HWS) << R) + a.row_base_in;
        const cu32p rb = (cu32p)a.rbits + (row0 >> 5);
        const uint32_t sub = c.s - c.w * G::HWS;
        uint32_t bits;
        // (uni(): each word stays a scalar load; a select of two loads would
        // be folded into one per-lane vector load)
        if constexpr (NR == 8) bits = uni(rb[0]) >> ((row0 & 31) + sub * 8);  // (HWS * 8 <= 32 rows)
        else if constexpr (G::HWS == 4) bits = ((sub >> 1) ? uni(rb[1]) : uni(rb[0])) >> ((sub & 1) * 16);
        else if constexpr (G::HWS == 2) bits = uni(rb[0]) >> (sub * 16);
        else bits = uni(rb[0]) >> (row0 & 31);
        bits &= (1u << NR) - 1;
        const LaneOff<V32> lo(lr, a.S_seg, c.offL);
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t ur = wr(m) + a.row_base_in;
            const gbyte* p;
            if constexpr (V32) {
                // (voff32: the wave's rows never straddle the segment boundary)
                p = lo.at(sgpr_ptr(ur >= a.chunk ? a.seg_b + (int64_t)((int64_t)ur - a.chunk) * (int64_t)a.S_seg
                                                 : a.seg_a + (uint64_t)ur * a.S_seg));
            } else {
                const uint32_t r = ur + lr;
                p = (const gbyte*)((r >= a.chunk ? a.seg_b + (uint64_t)(r - a.chunk) * a.S_seg
                                                 : a.seg_a + (uint64_t)r * a.S_seg) +
                                   c.offL);
            }
            ld_sel(a, p, c.active & ((bits >> m) & 1u), c.offL, d.L[m], d.H[m]);
        }
    } else {  // LD_DEC_LAST: u in registers, z for y = u + L(z)
        d.ztile = a.zflags && ((((cu32p)a.zflags)[tile >> 2] >> (8 * (tile & 3))) & 1u);
        const LaneOff<V32> lo(lr, a.S_in, c.offL);
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const uint32_t ur = wr(m);
            ld_sel(a, lo.at(sgpr_ptr(a.in + (uint64_t)ur * a.S_in)), c.active & !d.ztile, c.offL, d.zl[m], d.zh[m]);
            ld_sel(a, lo.at(sgpr_ptr(a.in2 + (uint64_t)ur * a.S_in)), c.active, c.offL, d.L[m], d.H[m]);
        }
    }
}

// Issue the HBM loads of one item (and read its decode flags).
template <int P, int T>
__device__ __forceinline__ void load_item(const PassArgs& a, const Thr& c, uint32_t tile, ItemRegs<P, T>& d) {
    using PT = ProgTraits<P>;
    using G = Geo<T>;
    constexpr int NR = G::NR, R = G::R;
    [[maybe_unused]] constexpr bool START_B = !PT::IFFT;
    d.zrow = d.zmask = 0;
    d.ztile = false;
    // ---------------- zero rows of DEC_MID ----------------
    // Row r of this pass came from DEC_FIRST tile r >> lo = k + (b_high << T).
    // zrow bit m: this thread's (layout-A) row m is such a skipped, zero row;
    // zmask bit j: tile rows [16j, 16j+16) all are (uniform, scalar loads).
    if constexpr (P == DEC_MID && T > 4 && R != 4) {
        // (8-row sets: one flag byte per row, per lane; no zmask pruning)
        if (a.zflags) {
            const uint8_t* zt = a.zflags + (c.b_high << T) + (c.s << R);
#pragma unroll
            for (int m = 0; m < NR; m++) d.zrow |= (uint32_t)(zt[m] & 1u) << m;
        }
    } else if constexpr (P == DEC_MID && T > 4) {
        if (a.zflags) {
            const uint8_t* zt = a.zflags + (c.b_high << T);
            // the wave's HWS row sets are 16 * HWS consecutive flag bytes:
            // scalar loads, then each lane picks its row set's 16
            const cu32p zw = (cu32p)(zt + ((c.w * G::HWS) << R));
            const uint32_t sub = c.s - c.w * G::HWS;
            uint32_t fw[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                uint32_t v = uni(zw[j]);
#pragma unroll
                for (int x = 1; x < G::HWS; x++) v = sub == (uint32_t)x ? uni(zw[4 * x + j]) : v;
                fw[j] = v;
            }
#pragma unroll
            for (int m = 0; m < NR; m++) d.zrow |= ((fw[m >> 2] >> (8 * (m & 3))) & 1u) << m;
            const cu32p zf = (cu32p)zt;
#pragma unroll
            for (int j = 0; j < G::SETS; j++)
                if ((zf[4 * j] & zf[4 * j + 1] & zf[4 * j + 2] & zf[4 * j + 3]) == 0x01010101u) d.zmask |= 1u << j;
        }
    }
    if (a.voff32) load_rows<P, T, true>(a, c, tile, d);
    else load_rows<P, T, false>(a, c, tile, d);
}

// Stage everything that depends on the tile key of the thread's current
// item: twiddle tables of both directions, and for the decoder's first /
// last pass the per-row erasure and reveal multipliers (and the last 256-point
// FWHT of eval_poly when the caller left it undone, ework).  In two steps:
// issue() sends the twiddle-table loads (one level deep, from skew_tab), so
// the caller can issue the tile's data loads behind them; finish() stages the
// per-row multipliers, writes everything to LDS and ends with a barrier.  The
// caller must have a barrier between the previous key's last use of these
// LDS regions and finish().
// Reveal multipliers (65535 - e of the lost originals) and lost-row flags of
// the tile; programs with a last layout switch stage them there
// (LateReveal), off the load phase -- they are read only by the stores.
template <int P, int T> struct LateReveal {
    static constexpr bool value = ProgTraits<P>::STORE == ST_RESTORE && ProgTraits<P>::FFT && T > 4;
};
template <int P, int T> struct RevealStage {
    using SM = Smem<P, T>;
    using G = Geo<T>;
    Stager<T, (1 << T)> sr;
    uint32_t lost[((1 << T) + G::THREADS - 1) / G::THREADS];
    __device__ __forceinline__ void issue(const PassArgs& a, const Thr& c, const uint32_t* el) {
        sr.issue(a.mul_tab, RevealEntry<T>{a, c, el});
#pragma unroll
        for (int i = 0; i < (int)(sizeof lost / sizeof lost[0]); i++) {
            const uint32_t k = threadIdx.x + i * G::THREADS;
            lost[i] = k < (1u << T) && row_lost_original(a, row_rel<T>(c, a, k) + a.row_base_out);
        }
    }
    __device__ __forceinline__ void commit(const PassArgs& a, const Thr& c, uint8_t* smem) const {
        (void)a;
        (void)c;
        uint32_t* lostf = (uint32_t*)(smem + SM::LOST_OFF);
#pragma unroll
        for (int i = 0; i < (int)(sizeof lost / sizeof lost[0]); i++) {
            const uint32_t k = threadIdx.x + i * G::THREADS;
            if (k < (1u << T)) lostf[k] = lost[i];
        }
        sr.commit((uint4*)(smem + SM::RVT_OFF));
    }
};

template <int P, int T> struct TileStage {
    using PT = ProgTraits<P>;
    using SM = Smem<P, T>;
    using G = Geo<T>;
    // second direction at the start: all of it, or only its layout-B tables
    static constexpr int N2 = !SM::TWO ? 0 : (LateS2<P, T>::value ? G::NTAB - G::TSPLIT : G::NTAB);
    static constexpr bool S2 = N2 > 0;
    // (SHARED: the first direction's layout-A tables into the image region,
    // its layout-B tables beside it)
    static constexpr int N1 = SM::SHARED ? G::TSPLIT : G::NTAB;
    static constexpr int N1B = SM::SHARED ? G::NTAB - G::TSPLIT : 0;
    Stager<T, N1> s1;
    Stager<T, N1B> s1b;
    Stager<T, N2> s2;

    uint32_t ev[4];  // wave 0: the tile's 256-row block of eval_poly's work (ework)
    // decoder gather: the received-bitmap words of this thread's erasure-table
    // rows, loaded before the tile's rows so that the table loads that depend
    // on them issue back to back (a per-row flag load after the rows would
    // wait for all of them, once per table)
    static constexpr int PER_E = ((1 << T) * 5 + G::THREADS - 1) / G::THREADS;
    uint32_t rw[PT::LOAD == LD_GATHER_DEC ? PER_E : 1];

    // the 256-row block holding the tile's decode rows (contiguous tiles of
    // 2^T <= 256 rows at a multiple of 2^T lie in one block)
    __device__ __forceinline__ uint32_t elog_row0(const PassArgs& a, const Thr& c) const {
        const uint32_t base = PT::LOAD == LD_GATHER_DEC ? a.row_base_in : a.row_base_out;
        return row_rel<T>(c, a, 0) + base;
    }
    __device__ __forceinline__ void issue(const PassArgs& a, const Thr& c) {
        if constexpr (SM::ELOG_BYTES > 0) {
            // requested first: the erasure logs head the staging chain
            if (a.ework && c.w == 0) {
                const uint32_t* src = a.ework + (elog_row0(a, c) & ~255u) + c.lane;
#pragma unroll
                for (int j = 0; j < 4; j++) ev[j] = src[64 * j];
            }
        }
        if constexpr (PT::LOAD == LD_GATHER_DEC) {
#pragma unroll
            for (int i = 0; i < PER_E; i++) {
                const uint32_t idx = threadIdx.x + (uint32_t)i * G::THREADS;
                const uint32_t k = min(idx / 5, (1u << T) - 1);
                rw[i] = a.rbits[(row_rel<T>(c, a, k) + a.row_base_in) >> 5];
            }
        }
        s1.issue(a.skew_tab, TwiddleEntry<T>{a, c, 0, PT::IFFT ? a.skew_ifft : a.skew_fft});
        if constexpr (N1B > 0) s1b.issue(a.skew_tab, TwiddleEntry<T>{a, c, G::TSPLIT, a.skew_ifft});
        if constexpr (S2) s2.issue(a.skew_tab, TwiddleEntry<T>{a, c, G::NTAB - N2, a.skew_fft});
    }
    // Decoder gather staging, run before the tile's row loads: the erasure
    // logs' last FWHT into LDS, then the "MULTIPLY SHARDS" table loads into
    // se (committed by finish()).
    Stager<T, (PT::LOAD == LD_GATHER_DEC ? (1 << T) : 0)> se;
    const uint32_t* el = nullptr;
    __device__ __forceinline__ void gather(const PassArgs& a, const Thr& c, uint8_t* smem) {
        if constexpr (SM::ELOG_BYTES > 0) {
            if (a.ework) {
                // the last 256-point FWHT of eval_poly, by wave 0 in registers
                uint32_t* elds = (uint32_t*)(smem + SM::ELOG_OFF);
                if (c.w == 0) {
                    fwht256_wave(ev);
#pragma unroll
                    for (int j = 0; j < 4; j++) elds[c.lane + 64 * j] = ev[j];
                }
                __syncthreads();
                el = elds + (elog_row0(a, c) & 255u);
            }
        }
        if constexpr (PT::LOAD == LD_GATHER_DEC) {
            // "MULTIPLY SHARDS" tables (GatherEntry, with the received bit from rw)
            static_assert(PER_E == Stager<T, (1 << T)>::PER, "one table chunk per (thread, i)");
            const u32x4* tab = (const u32x4*)a.mul_tab;
            // (two uniform paths: with the logs in LDS every table load issues
            // back to back; only the HBM-logs path waits per row)
            auto gather_rows = [&](auto log_of) {
#pragma unroll
                for (int i = 0; i < PER_E; i++) {
                    const uint32_t idx = threadIdx.x + (uint32_t)i * G::THREADS;
                    const uint32_t k = min(idx / 5, (1u << T) - 1);
                    const uint32_t r = row_rel<T>(c, a, k) + a.row_base_in;
                    const bool rcv = (rw[i] >> (r & 31)) & 1u;
                    const uint32_t e = rcv ? log_of(k, r) : ZERO_ENTRY;
                    if (idx < (1u << T) * 5)
                        se.v[i] = tab[(size_t)e * (TAB_DWORDS / 4) + idx % 5];
                }
            };
            if (el) gather_rows([&](uint32_t k, uint32_t) { return el[k]; });
            else gather_rows([&](uint32_t, uint32_t r) { return a.elog[r]; });
        }
    }
    template <bool GATHERED = false>
    __device__ __forceinline__ void finish(const PassArgs& a, const Thr& c, uint8_t* smem) {
        if constexpr (!GATHERED) gather(a, c, smem);
        if constexpr (PT::LOAD == LD_GATHER_DEC) se.commit((uint4*)(smem + SM::ERT_OFF));
        if constexpr (PT::STORE == ST_RESTORE && !LateReveal<P, T>::value) {
            RevealStage<P, T> rs;
            rs.issue(a, c, el);
            rs.commit(a, c, smem);
        }
        if constexpr (S2) s2.commit((uint4*)(smem + SM::TAB2_OFF));
        s1.commit((uint4*)(smem + SM::TAB1_OFF));
        if constexpr (N1B > 0) s1b.commit((uint4*)(smem + SM::TABB_OFF));
        __syncthreads();  // staged tables visible
    }
};

// Received counts of a decode with identity multipliers (PassArgs::rcount,
// ENC_FIRST / ENC_LAST launched by decode_passes): wave j of the first
// slab's workgroup counts chunk j of its tile (a tile below 64 rows: the
// chunk's first tile counts it).  Behind uniform branches: the flag bytes
// are the workgroup's first loads (so the compiler's waits for the later
// loads do not change), the ballots run after the staging barrier (the bytes
// are older than the tables it waited for) and the counts, in SGPRs, are
// stored after the item.
template <int P, int T> struct RcvCount {
    static constexpr bool ON = P == ENC_FIRST || P == ENC_LAST;
    static constexpr uint32_t NCH = (1u << T) >= 64 ? (1u << T) / 64 : 1;
    bool go;
    uint32_t r0, f, cnt;
    __device__ __forceinline__ void issue(const PassArgs& a, const Thr& c, bool first) {
        go = false;
        if constexpr (ON) {
            r0 = uni(row_rel<T>(c, a, 0) + 64u * c.w);
            go = first && a.rcount && c.w < NCH && (r0 & 63u) == 0;
            if (go) f = !a.cnt_flags || a.cnt_flags[r0 + c.lane];
        }
    }
    __device__ __forceinline__ void count() {
        if constexpr (ON)
            if (go) cnt = uni((uint32_t)__popcll(__ballot(f != 0)));
    }
    __device__ __forceinline__ void store(const PassArgs& a, const Thr& c) const {
        if constexpr (ON) {
            if (go && c.lane == 0) {
                const uint32_t ch = (r0 + a.cnt_base) >> 6;
                a.rcount[2 * ch + a.cnt_seg] = cnt;
                a.rcount[2 * ch + 1 - a.cnt_seg] = 0;
            }
        }
    }
};

// Compute and store one item whose rows are in d (every thread of the
// workgroup calls it for the same item).
// The one-item build's store of row register m of an item (the counterpart
// of load_rows): recovery / work rows as they are, lost originals revealed
// (x (65535 - e), rate_high.rs:236-242) into the caller's original array.
template <int P, int T, bool V32>
__device__ __forceinline__ void store_row(const PassArgs& a, const Thr& cs, uint32_t L, uint32_t H, int m,
                                          const uint4* rvt, const uint32_t* lostf) {
    using PT = ProgTraits<P>;
    constexpr bool END_B = !PT::FFT && T > 4;
    constexpr bool NT = PT::ST_NT;
    const uint32_t lr = lane_rows<T, END_B>(cs, a);
    const WaveRows<T, END_B> wr(cs, a);
    const uint32_t ur = wr(m);
    if constexpr (PT::STORE == ST_PLAIN) {
        const LaneOff<V32> lo(lr, a.S_out, cs.offL);
        const uint32_t k = kidx<T, END_B>(cs, m);
        st_ptr<NT>(a, lo.at(sgpr_ptr(a.out + (uint64_t)ur * a.S_out)),
                   cs.active & (P != DEC_MID || (k >= a.need_lo && k < a.need_hi)), L, H);
    } else if constexpr (PT::STORE == ST_RECOVERY) {
        const LaneOff<V32> lo(lr, a.S_out, cs.offL);
        st_ptr<NT>(a, lo.at(sgpr_ptr(a.out + (uint64_t)ur * a.S_out)), cs.active & row_below(ur, lr, a.out_rows), L, H);
    } else {
        // lost original row r -> restored-originals row r + row_base_out - (segment start)
        const LaneOff<V32> lo(lr, a.S_rest, cs.offL);
        const int64_t shift = (int64_t)a.row_base_out - (a.rest_seg_b ? (int64_t)a.chunk : 0);
        const uint32_t k = kidx<T, END_B>(cs, m);
        // (a row that is not a lost original is neither multiplied nor
        // stored: the branch is per row set, so a wave whose rows were all
        // received skips the reveal -- most rows of a decode with few losses)
        if (cs.active & (lostf[k] != 0)) {
            uint32_t tt[20];
            load_table_lds(tt, rvt + k * 5);
            uint32_t ol = 0, oh = 0;
            mul_xor(ol, oh, L, H, tt);
            st_ptr<NT>(a, lo.at(sgpr_ptr(a.rest + ((int64_t)ur + shift) * (int64_t)a.S_rest)), true, ol, oh);
        }
    }
}
template <int P, int T, bool V32>
__device__ __forceinline__ void store_rows(const PassArgs& a, const Thr& cs, const uint32_t (&L)[Geo<T>::NR],
                                           const uint32_t (&H)[Geo<T>::NR], const uint4* rvt, const uint32_t* lostf) {
#pragma unroll
    for (int m = 0; m < Geo<T>::NR; m++) store_row<P, T, V32>(a, cs, L[m], H[m], m, rvt, lostf);
}
// Early stores: the last FFT block in layout A runs depth-first (LayerSeq),
// so rows m, m + 1 are final as soon as their layer-0 group is done; this
// functor stores them there, spreading the item's stores over the block
// instead of a burst after it.
template <int P, int T> struct EarlyStore {
    const PassArgs& a;
    const Thr& cs;
    const uint4* rvt;
    const uint32_t* lostf;
    __device__ __forceinline__ void operator()(const uint32_t (&L)[Geo<T>::NR], const uint32_t (&H)[Geo<T>::NR],
                                               int m) const {
        if (a.voff32) {
            store_row<P, T, true>(a, cs, L[m], H[m], m, rvt, lostf);
            store_row<P, T, true>(a, cs, L[m + 1], H[m + 1], m + 1, rvt, lostf);
        } else {
            store_row<P, T, false>(a, cs, L[m], H[m], m, rvt, lostf);
            store_row<P, T, false>(a, cs, L[m + 1], H[m + 1], m + 1, rvt, lostf);
        }
    }
};

// The same for a pass that ends with its IFFT in layout B (ENC_FIRST, the
// decoders' first pass, GEN_IFFT): the rows with register bit 0 clear and
// those with it set go through the block's layers separately -- the layer of
// register bit 0 (layout-B bit SHB, the first one at T = 8) all in the first
// half, every higher layer's butterfly pairs m, m + 2^rb with m of the half's
// parity -- so the even rows are final after the first half and are stored
// there (fin), and the odd rows' butterflies run while those stores drain.
// Same groups, tables and butterflies as layers<.., LB = true, .., IFFT>,
// in another order; every group's table is read (LDS) one group ahead.
template <int T> struct HalfSeq {
    static constexpr int SH = Geo<T>::SHB, NR = Geo<T>::NR;
    // step g -> half * 256 + kb * 16 + gi
    static constexpr int at(int g) {
        int n = 0;
        for (int half = 0; half < 2; half++)
            for (int kb = Geo<T>::R; kb < T; kb++) {
                const int rb = kb - SH;
                if (rb == 0 && half == 1) continue;  // (bit 0's layer: all in the first half)
                for (int gi = 0; gi < (NR >> (rb + 1)); gi++)
                    if (n++ == g) return half * 256 + kb * 16 + gi;
            }
        return -1;
    }
    static constexpr int total() {
        int g = 0;
        while (at(g) >= 0) g++;
        return g;
    }
};
template <int T, int G, class FIN> struct HalfLoop {
    static __device__ __forceinline__ void run(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR],
                                               const uint4* tab1, const uint32_t (&cur)[20], const FIN& fin) {
        using S = HalfSeq<T>;
        constexpr int e = S::at(G), half = e >> 8, kb = (e >> 4) & 15, gi = e & 15, rb = kb - S::SH;
        constexpr bool more = G + 1 < S::total();
        uint32_t nxt[20];
        if constexpr (more) {
            constexpr int kb2 = (S::at(G + 1) >> 4) & 15, gi2 = S::at(G + 1) & 15;
            load_table_lds(nxt, tab1 + ((1 << T) - (1 << (T - kb2)) + gi2) * 5);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < (1 << rb); j++) {
            if (rb > 0 && (j & 1) != half) continue;
            const int m = (gi << (rb + 1)) + j, m2 = m + (1 << rb);
            L[m2] ^= L[m];
            H[m2] ^= H[m];
            mul_xor(L[m], H[m], L[m2], H[m2], cur);
            asm volatile("" : "+v"(L[m]), "+v"(H[m]), "+v"(L[m2]), "+v"(H[m2]));
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (more) {
            if constexpr (half == 0 && (S::at(G + 1) >> 8) == 1) fin(L, H);  // the even rows are final
            HalfLoop<T, G + 1, FIN>::run(L, H, tab1, nxt, fin);
        }
    }
};
template <int T, class FIN>
__device__ __forceinline__ void ifft_b_halves(uint32_t (&L)[Geo<T>::NR], uint32_t (&H)[Geo<T>::NR], const uint4* tab1,
                                              const FIN& fin) {
    constexpr int e = HalfSeq<T>::at(0), kb = (e >> 4) & 15, gi = e & 15;
    tab1 = lds_vgpr(tab1);
    uint32_t t0[20];
    load_table_lds(t0, tab1 + ((1 << T) - (1 << (T - kb)) + gi) * 5);
    HalfLoop<T, 0, FIN>::run(L, H, tab1, t0, fin);
}
// fin of ifft_b_halves: the even rows
template <int P, int T> struct EvenStore {
    const PassArgs& a;
    const Thr& cs;
    __device__ __forceinline__ void operator()(const uint32_t (&L)[Geo<T>::NR], const uint32_t (&H)[Geo<T>::NR]) const {
#pragma unroll
        for (int m = 0; m < Geo<T>::NR; m += 2) {
            if (a.voff32) store_row<P, T, true>(a, cs, L[m], H[m], m, nullptr, nullptr);
            else store_row<P, T, false>(a, cs, L[m], H[m], m, nullptr, nullptr);
        }
    }
};

template <int P, int T>
__device__ __forceinline__ void process_item(const PassArgs& a, const Thr& c, uint32_t tile, uint32_t slab,
                                             ItemRegs<P, T>& d, uint8_t* smem) {
    using PT = ProgTraits<P>;
    using SM = Smem<P, T>;
    using G = Geo<T>;
    constexpr int NR = G::NR;
    constexpr int R = G::R;
    constexpr int NQR = Rnd<P, T>::NQR;
    constexpr bool TWO = SM::TWO;
    // (DEC_MID runs with T >= 5 only; the 16-row-block pruning needs R = 4)
    constexpr bool ZERO_SKIP = P == DEC_MID && T > 4 && G::R == 4;
    // stores inside the last FFT block (one-item build, 16 rows per lane, not
    // the output-pruned DEC_MID; the reveal stores measured slower inside it)
    constexpr bool EARLY = LayerSeq<T, false, 0, R, true>::DF && P != DEC_MID && PT::STORE != ST_RESTORE && PT::FFT &&
                           T > 4;
    // the IFFT-only passes: early stores of the even rows (ifft_b_halves)
    constexpr bool EARLY_B = PT::IFFT && !PT::FFT && PT::STORE == ST_PLAIN && T > 4 && G::R == 4 && !RS16_NO_EARLY_B;
    uint2* lds = (uint2*)smem;
    const uint4* tab1 = (const uint4*)(smem + SM::TAB1_OFF);
    const uint4* tab2 = (const uint4*)(smem + SM::TAB2_OFF);
    const uint4* ert = (const uint4*)(smem + SM::ERT_OFF);
    const uint4* rvt = (const uint4*)(smem + SM::RVT_OFF);
    const uint32_t* lostf = (const uint32_t*)(smem + SM::LOST_OFF);
    uint32_t(&L)[NR] = d.L;
    uint32_t(&H)[NR] = d.H;
    constexpr bool START_B = !PT::IFFT;
    // Final layout: after FFT -> A; after IFFT only -> B (T > 4); T <= 4: A == B.
    [[maybe_unused]] constexpr bool END_B = !PT::FFT && T > 4;
    // DEC_MID whose consumed tile rows (the last pass's tiles with a lost
    // original, [need_lo, need_hi)) lie in few layout-B register rows: the
    // formal derivative split by row bits (fd_regs / fd_image), otherwise
    // through the LDS image (tile_fd).  The layout-A FFT layers make every
    // row of a consumed row's 2^R-row block an input of it: the block's
    // layout-B register rows [fd_m0, fd_m0 + FD_ND) take the fd_image terms.
    constexpr bool SPLIT_FD = P == DEC_MID && T > 4;
    constexpr int FD_PB = 1 << (R - G::SHB);            // register rows per 2^R-row block
    constexpr int FD_ND = FD_PB > 2 ? FD_PB : 2;        // register rows carried
    [[maybe_unused]] bool fd_few = false;
    [[maybe_unused]] uint32_t fd_m0 = 0;
    [[maybe_unused]] uint32_t dl[FD_ND], dh[FD_ND];
    if constexpr (SPLIT_FD) {
        const uint32_t lo = uni(a.need_lo), hi = uni(min(a.need_hi, 1u << T));
        const uint32_t m0 = (lo >> R) * FD_PB, m1 = hi <= lo ? m0 : (((hi - 1) >> R) + 1) * FD_PB;
        fd_few = !a.fd_lds && m1 - m0 <= (uint32_t)FD_ND;
        fd_m0 = hi <= lo ? 0u : min(m0, (uint32_t)(NR - FD_ND));
    }

    if constexpr (P == DEC_FIRST) {
        // A tile without received rows is zero after the erasure multiply
        // and through the IFFT: DEC_MID / DEC_LAST read it as zero, skip it.
        if (a.zflags && ((((cu32p)a.zflags)[tile >> 2] >> (8 * (tile & 3))) & 1u)) {
            __builtin_amdgcn_s_waitcnt(vmcnt_wait(0));  // (see the end of this function)
            return;
        }
    }
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
        if (!d.ztile) tile_fd<T, NQR, START_B>(L, H, d.zl, d.zh, c, lds);
    }

    // SHARED: the second direction's layout-A tables are requested after the
    // first layout switch and written over the image after the second
    [[maybe_unused]] Stager<T, (SM::SHARED ? G::TSPLIT : 0)> s3s;
    // ---------------- IFFT ----------------
    bool in_b = START_B;
    if constexpr (PT::IFFT) {
        // DEC_MID: a wave whose rows all are zero skips its layout-A layers
        bool skip_a = false;
        if constexpr (ZERO_SKIP) skip_a = __all(d.zrow == (1u << NR) - 1);
        if (!skip_a) layers<P, T, false, 0, R, false, false>(L, H, c, a, tab1, tab2);
        RS16_STAMP(a, 3);
        prio<P, 1, T>();
        if constexpr (T > 4) {
            constexpr bool LS2 = LateS2<P, T>::value && !SM::SHARED;
            Stager<T, (LS2 ? G::TSPLIT : 0)> s3;
            if constexpr (LS2) s3.issue(a.skew_tab, TwiddleEntry<T>{a, c, 0, a.skew_fft});
            // (SHARED: the image overwrites the layout-A tables -- every wave
            // must be done with them first)
            if constexpr (SM::SHARED) __syncthreads();
            exchange<T, NQR, false>(
                L, H, c, lds,
                [&]() {
                    if constexpr (LS2) s3.commit((uint4*)(smem + SM::TAB1_OFF));
                },
                [&]() {
                    if constexpr (SPLIT_FD) {
                        if (fd_few) {
                            constexpr int QL = G::Q / NQR;
#pragma unroll
                            for (int i = 0; i < FD_ND; i++)
                                fd_image<T, QL>(dl[i], dh[i], c, lds, kidx<T, true>(c, fd_m0 + i));
                        }
                    }
                });
            RS16_STAMP(a, 4);
            if constexpr (SM::SHARED) s3s.issue(a.skew_tab, TwiddleEntry<T>{a, c, 0, a.skew_fft});
            if constexpr (EARLY_B) {
                Thr cs = c;
                asm volatile("" : "+v"(cs.offL));
                ifft_b_halves<T>(L, H, tab1, EvenStore<P, T>{a, cs});
            } else {
                // (SHARED: the layout-B tables t >= TSPLIT sit beside the image)
                const uint4* tab1b = SM::SHARED ? (const uint4*)(smem + SM::TABB_OFF) - G::TSPLIT * 5 : tab1;
                layers<P, T, true, R, (T > 4 ? T : R), false, false, (ZERO_SKIP ? PR_ZERO : PR_NONE)>(L, H, c, a, tab1b,
                                                                                                    tab2, d.zmask);
            }
            in_b = true;
        }
        RS16_STAMP(a, 5);
        prio<P, 2, T>();
    }
    // ---------------- formal derivative (tile bits) ----------------
    if constexpr (PT::FD) {
        if constexpr (SPLIT_FD) {
            if (fd_few) fd_regs<T>(L, H);
            else tile_fd<T, NQR, true>(L, H, L, H, c, lds);
        } else {
            if (in_b) tile_fd<T, NQR, true>(L, H, L, H, c, lds);
            else tile_fd<T, NQR, false>(L, H, L, H, c, lds);
        }
        RS16_STAMP(a, 6);
    }
    // ---------------- FFT ----------------
    if constexpr (PT::FFT) {
        if constexpr (T > 4) {
            layers<P, T, true, R, (T > 4 ? T : R), true, TWO, (P == DEC_MID ? PR_OUT : PR_NONE)>(L, H, c, a, tab1,
                                                                                             tab2);
            if constexpr (SPLIT_FD) {
                // the layout-A bits' derivative terms (fd_image) join the
                // register rows that feed consumed rows
                if (fd_few) {
#pragma unroll
                    for (int m = 0; m < NR; m++) {
#pragma unroll
                        for (int i = 0; i < FD_ND; i++)
                            if ((uint32_t)m == fd_m0 + i) L[m] ^= dl[i], H[m] ^= dh[i];
                    }
                }
            }
            RS16_STAMP(a, 7);
            prio<P, 3, T>();
            // reveal multipliers: requested before the last layout switch,
            // written to LDS between its barriers (read after the layers)
            RevealStage<P, (LateReveal<P, T>::value ? T : 0)> rs;
            if constexpr (LateReveal<P, T>::value) {
                const uint32_t* el = nullptr;
                if (a.ework) {
                    const uint32_t base = a.row_base_out;
                    el = (const uint32_t*)(smem + SM::ELOG_OFF) + ((row_rel<T>(c, a, 0) + base) & 255u);
                }
                rs.issue(a, c, el);
            }
            if constexpr (SPLIT_FD) {
                if (fd_few) few_switch<T, FD_ND>(L, H, c, lds, fd_m0);
                else exchange<T, NQR, true>(L, H, c, lds);
            } else {
                exchange<T, NQR, true>(L, H, c, lds, [&]() {
                    if constexpr (LateReveal<P, T>::value) rs.commit(a, c, smem);
                });
            }
            if constexpr (SM::SHARED) {
                // (the image is dead once every wave's rows are back in
                // registers: exchange() ends with a barrier, few_switch()
                // does not)
                if constexpr (SPLIT_FD) {
                    if (fd_few) __syncthreads();
                }
                s3s.commit((uint4*)(smem + SM::TAB1_OFF));
                __syncthreads();
            }
            RS16_STAMP(a, 8);
            prio<P, 4, T>();
            in_b = false;
        }
        bool need = true;
        if constexpr (P == DEC_MID) need = (c.s << R) < a.need_hi && ((c.s + 1) << R) > a.need_lo;
#ifndef RS16_NO_RESTORE_SKIP
        if constexpr (PT::STORE == ST_RESTORE && T > 4) {
            // a row set without a lost original stores nothing: its
            // layout-A FFT layers are skipped (a wave whose two row sets
            // both have none skips them -- most waves of a decode that lost
            // few, scattered originals)
            uint32_t any = 0;
#pragma unroll
            for (int m = 0; m < NR; m++) any |= lostf[kidx<T, false>(c, m)];
            need = any != 0;
        }
#endif
        // second direction's layout-A tables: restaged into tab1 (T > 4), else in tab2
        if constexpr (EARLY) {
            Thr cs = c;
            asm volatile("" : "+v"(cs.offL));
            layers<P, T, false, 0, R, true, (TWO && !(SM::RESTAGE))>(L, H, c, a, tab1, tab2, 0,
                                                                   EarlyStore<P, T>{a, cs, rvt, lostf});
        } else if (need) {
            layers<P, T, false, 0, R, true, (TWO && !(SM::RESTAGE))>(L, H, c, a, tab1, tab2);
        }
        RS16_STAMP(a, 9);
    }
    if constexpr (EARLY) {
        RS16_STAMP(a, 10);
        RS16_STAMP_END(a);
        return;
    }

    prio<P, 5, T>();
    // ---------------- store ----------------
    // The next item's loads were issued before this item's butterflies and
    // have landed by now: retire them before the stores, so that the stores
    // stay in flight across the loop latch (with 2 NR loads + 2 NR stores
    // outstanding there, the compiler's own wait would be vmcnt(0)).
    __builtin_amdgcn_s_waitcnt(vmcnt_wait(0));
    // Row addresses are recomputed here from opaque copies of the item
    // coordinates: otherwise the compiler keeps the load-time addresses of
    // the same rows live through all the butterflies (32 VGPRs).
    Thr cs = c;
    cs.b_low = uni(cs.b_low);
    cs.b_high = uni(cs.b_high);
    asm volatile("" : "+s"(cs.b_low), "+s"(cs.b_high));
    asm volatile("" : "+v"(cs.offL));
    if constexpr (EARLY_B) {
        // (the even rows went out inside the last block)
#pragma unroll
        for (int m = 1; m < NR; m += 2) {
            if (a.voff32) store_row<P, T, true>(a, cs, L[m], H[m], m, rvt, lostf);
            else store_row<P, T, false>(a, cs, L[m], H[m], m, rvt, lostf);
        }
    } else {
        if (a.voff32) store_rows<P, T, true>(a, cs, L, H, rvt, lostf);
        else store_rows<P, T, false>(a, cs, L, H, rvt, lostf);
    }
    RS16_STAMP(a, 10);
    RS16_STAMP_END(a);
}

// The pass: workgroup b processes item b of the launch (4 waves per SIMD,
// except the one-pass decoders, whose larger register sets take 1).
template <int P, int T>
__global__ void __launch_bounds__(Geo<T>::THREADS, ((P == DEC_SINGLE || P == DEC_HALF_SINGLE) ? 1 : 4))
    pass_kernel(PassArgs a) {
    using G = Geo<T>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t item = blockIdx.x;  // (launch_pass: one workgroup per item)

    Thr c;
    c.lane = threadIdx.x & 63;
    c.w = uni(threadIdx.x >> 6);
    c.qt = c.lane % G::Q;
    c.s = c.w * G::HWS + c.lane / G::Q;
    c.ql = c.qt % Rnd<P, T>::QL;
    c.round = c.qt / Rnd<P, T>::QL;

    uint32_t tile, slab;
    set_item(c, a, item, G::Q, tile, slab);

    bool first_stripe = true;
    if (a.stripe_tiles) {
        // batched stripes: the stripe's arrays, the tile within the stripe
        const uint32_t st = uni(tile / a.stripe_tiles);
        first_stripe = st == 0;
        tile -= st * a.stripe_tiles;
        a.in += st * a.bs_in;
        a.in2 += st * a.bs_in2;
        a.out += st * a.bs_out;
        a.seg_a += st * a.bs_seg;
        a.seg_b += st * a.bs_seg_b;
        a.rest += st * a.bs_rest;
        // stripes with losses of their own: their flags and decode metadata
        // (all strides 0 when the stripes share one erasure pattern)
        if (a.flags_a) a.flags_a += st * a.bs_fa;
        if (a.flags_b) a.flags_b += st * a.bs_fb;
        if (a.elog) a.elog += st * a.bs_elog;
        if (a.ework) a.ework += st * a.bs_elog;
        if (a.rbits) a.rbits += st * a.bs_rbits;
        if (a.zflags) a.zflags += st * a.bs_zflags;
        if (a.lostrange) a.lostrange += st * a.bs_lost;
    }
    tile += a.tile_base;
    c.b_low = tile & ((1u << a.lo) - 1);
    c.b_high = tile >> a.lo;
    RcvCount<P, T> rcn;
    rcn.issue(a, c, slab == 0 && first_stripe);
    if constexpr (P == DEC_FIRST) {
        // a tile without received rows is skipped (process_item): return
        // before its table staging and row loads, so its slot frees at once
        if (a.zflags && ((((cu32p)a.zflags)[tile >> 2] >> (8 * (tile & 3))) & 1u)) return;
    }
    if constexpr (P == DEC_MID) {
        // mid_direct_kernel computed this stripe's consumed rows already
        uint32_t nlo, nhi;
        if (a.mid_direct && a.lostrange && mid_need(a, nlo, nhi)) return;
    }
    if constexpr (P == DEC_LAST) {
        // A tile without a lost original stores nothing: return before any
        // load (the decode's lost rows are [lostrange[0], lostrange[1])).
        if (a.lostrange) {
            const uint32_t r0 = ((cu32p)a.lostrange)[0], r1 = ((cu32p)a.lostrange)[1];
            if (!((tile << T) < r1 && ((tile + 1) << T) > r0)) return;
            // (tile_last_kernel took this stripe's few tiles)
            if (a.tl_max && tl_covers<T>(a)) return;
        }
    }
    // one item per workgroup (launch_pass sets per_wg = 1): straight-line code
    // (a loop lets the compiler hoist per-row address terms out of it, which
    // costs more VGPRs than the 128 of four waves per SIMD).  The twiddle
    // tables are requested first, the tile's rows right behind them, so the
    // staging latency hides under the row loads.
    RS16_STAMP(a, 0);
    // Load-issue order: the workgroup in slot 0 of its CU (HW_ID.tg_id) issues
    // its rows first, slot 1 next, ...  Same-box A/B: kernel times equal,
    // step time -2 % (643-645 -> 654-659 GiB/s, 3 pairs).  The progress-based
    // schedule (prio<P, at>) takes over once the tables are staged.
    if constexpr (T >= 7) {
        const uint32_t slot = (__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 16) & 15u;
        if (slot == 0) __builtin_amdgcn_s_setprio(3);
        else if (slot == 1) __builtin_amdgcn_s_setprio(2);
        else if (slot == 2) __builtin_amdgcn_s_setprio(1);
        // (a second-slot sleep before the loads, 2 or 4 us, measured neutral
        // to slower on the T = 7 passes: profiles/r06_t7_slot_sleep_rejected.txt)
    }
    TileStage<P, T> st;
    st.issue(a, c);  // twiddle tables first: they do not queue behind the tile
    // Decoder gather: the erasure tables are requested ahead of the rows (their
    // logs: the tile's eval_poly block + one FWHT, issued with the twiddles),
    // so they do not queue behind the tile in the memory pipeline (same-box
    // A/B: DEC_HALF_FIRST -0.9 us, 3 pairs)
    constexpr bool EARLY = ProgTraits<P>::LOAD == LD_GATHER_DEC;
    if constexpr (EARLY) st.gather(a, c, smem);
    ItemRegs<P, T> cur;
    load_item<P, T>(a, c, tile, cur);
    if constexpr (P == DEC_MID) {
        // Only the last pass's tiles that hold a lost original are consumed:
        // tile row k = rows [k << lo, (k + 1) << lo) (read with the rows in flight)
        if (a.lostrange) {
            const uint32_t r0 = ((cu32p)a.lostrange)[0], r1 = ((cu32p)a.lostrange)[1];
            const bool any = r0 < r1;
            a.need_lo = max(a.need_lo, any ? r0 >> a.lo : 0u);
            a.need_hi = min(a.need_hi, any ? ((r1 - 1) >> a.lo) + 1 : 0u);
        }
    }
    RS16_STAMP(a, 1);
    prio<P, 0, T>();
    st.template finish<EARLY>(a, c, smem);
    rcn.count();
    RS16_STAMP(a, 2);
    process_item<P, T>(a, c, tile, slab, cur, smem);
    rcn.store(a, c);
}

// ---------------------------------------------------------------------------
// The general decode's last pass (DEC_LAST: y = u + L(z) -> FFT of the tile's
// 8 low row bits -> reveal x (65535 - e) -> store the lost originals,
// rate_high.rs:232-242 / rate_low.rs:232-242) as one wave per quad column of
// a 256-row tile instead of one 8-wave workgroup per (tile, 32-quad slab):
// lane l holds 4 rows of its quad column, the FFT runs in 4 radix-4 blocks
// in registers with in-wave row-bit exchanges (colops, as the column codec
// at 256 rows), the in-tile formal-derivative terms come from registers and
// lane shuffles (no LDS image, no barrier).  Four quad columns per
// workgroup share the tile's 255 twiddle tables (staged by LDS-DMA once) and
// the tile's erasure logs.  A decode that lost few originals needs this pass
// for a handful of tiles only (lost-range pruning): there the 8-wave item's
// latency (two waves per SIMD through 8 layers of 16 rows) was the whole
// pass, 25 us for the reference bench's 1 % loss; here each wave carries a
// quarter of the rows.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) tile_last_kernel(PassArgs a) {
    using namespace colops;
    constexpr int T = 8;
    constexpr uint32_t NTAB = (1u << T) - 1;
    __shared__ __attribute__((aligned(16))) uint8_t tabs[NTAB * 80];
    __shared__ uint32_t elds[256];
    const uint32_t t = threadIdx.x, lane = t & 63, w = uni(t >> 6);
    const uint32_t nq4 = (a.qrow + 3) / 4;
    uint32_t tile = blockIdx.x / nq4;
    const uint32_t qg = blockIdx.x - tile * nq4;
    if (a.stripe_tiles) {
        const uint32_t st = uni(tile / a.stripe_tiles);
        tile -= st * a.stripe_tiles;
        a.in += st * a.bs_in;
        a.in2 += st * a.bs_in2;
        a.rest += st * a.bs_rest;
        if (a.flags_a) a.flags_a += st * a.bs_fa;
        if (a.flags_b) a.flags_b += st * a.bs_fb;
        if (a.elog) a.elog += st * a.bs_elog;
        if (a.ework) a.ework += st * a.bs_elog;
        if (a.zflags) a.zflags += st * a.bs_zflags;
        if (a.lostrange) a.lostrange += st * a.bs_lost;
    }
    if (a.lostrange) {
        // The grid covers min(tiles, tl_max) tiles per stripe, counted from
        // the first one with a lost original; lost originals over more than
        // tl_max tiles are DEC_LAST's (its 8-wave items win there:
        // scripts/probe_general.py, break-even 16-32 tiles), and a tile past
        // the last lost original stores nothing.
        const uint32_t r0 = ((cu32p)a.lostrange)[0], r1 = ((cu32p)a.lostrange)[1];
        if (!tl_covers<T>(a)) return;
        tile += r0 >> T;
        if (tile > ((r1 - 1) >> T)) return;
    } else {
        tile += a.tile_base;
    }
    RS16_STAMP(a, 0);
    const uint32_t q = qg * 4 + w;
    const bool active = q < a.qrow;
    const uint32_t offL = (q >> 3) * 64 + (q & 7) * 4;
    const bool ztile = a.zflags && ((((cu32p)a.zflags)[tile >> 2] >> (8 * (tile & 3))) & 1u);
    // ---- requests: z and u of the lane's rows in the first FFT block's
    // layout (row bits 6, 7 in registers: row k = lane + 64 m), the tile's
    // erasure-log block (wave 0, when eval_poly left its last H_lo to this
    // pass), then the twiddle tables by LDS-DMA
    uint32_t ZL[4], ZH[4], YL[4], YH[4];
    const uint8_t* zpage = a.zero + (offL & 0x7FFFu);
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const uint64_t r = ((uint64_t)tile << T) + lane + 64u * m;
        const uint32_t* pz = (const uint32_t*)(active && !ztile ? a.in + r * a.S_in + offL : zpage);
        const uint32_t* pu = (const uint32_t*)(active ? a.in2 + r * a.S_in + offL : zpage);
        ZL[m] = pz[0];
        ZH[m] = pz[8];
        YL[m] = pu[0];
        YH[m] = pu[8];
    }
    const uint32_t row0 = (tile << T) + a.row_base_out;  // the tile's first decode work row
    uint32_t ev[4] = {0, 0, 0, 0};
    if (a.ework && w == 0) {
#pragma unroll
        for (int j = 0; j < 4; j++) ev[j] = a.ework[(row0 & ~255u) + lane + 64u * j];
    }
#pragma unroll
    for (uint32_t i = 0; i * 256 < NTAB * 5; i++) {
        const uint32_t c = i * 256 + t;
        if (c < NTAB * 5) {
            // chunk c = part c % 5 of table tb = c / 5 (tile-group order: layer
            // kb at groups [2^T - 2^(T-kb), ...), group j = row >> (kb + 1))
            const uint32_t tb = c / 5, part = c - tb * 5;
            const uint32_t kb = (uint32_t)(T - 32 + __clz(NTAB - tb));
            const uint32_t j = tb - ((1u << T) - (1u << (T - kb)));
            const uint32_t idx = (tile << T) + (j << (kb + 1)) + (1u << kb) + a.skew_fft - 1;
            __builtin_amdgcn_global_load_lds((colops::glb_vp)(a.skew_tab + (size_t)idx * TAB_DWORDS + part * 4),
                                             (colops::lds_vp)(tabs + (i * 256 + 64 * w) * 16), 16, 0, 0);
        }
    }
    RS16_STAMP(a, 1);
    __builtin_amdgcn_s_waitcnt(0);
    if (a.ework && w == 0) {
        fwht256_wave(ev);  // the last 256-point FWHT of eval_poly (src/engine.rs:207-218)
#pragma unroll
        for (int j = 0; j < 4; j++) elds[lane + 64 * j] = ev[j];
    }
    __syncthreads();  // tables and logs in LDS
    RS16_STAMP(a, 2);
    // ---- reveal multipliers of the lane's output rows (the last block's
    // layout: row k = 4 lane + m), requested now, used after the FFT
    uint32_t rt[4][20];
    bool lost[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const uint32_t r = row0 + 4 * lane + m;
        lost[m] = active && row_lost_original(a, r);
        const uint32_t e = a.ework ? elds[(4 * lane + m + row0) & 255u] : (lost[m] ? a.elog[r] : 0u);
        glb_table(rt[m], a.mul_tab, lost[m] ? GF_MODULUS - e : ZERO_ENTRY);
    }
    // ---- y = u + L(z): the formal derivative's terms of the tile's row bits
    // (src/engine.rs:233-238 in closed form): y[k] ^= z[k | 2^b] for every
    // bit b < 8 that is 0 in k -- bits 6, 7 are register bits, 0-5 lane bits
    if (!ztile) {
#pragma unroll
        for (int m = 0; m < 4; m++) {
            if (!(m & 1)) YL[m] ^= ZL[m | 1], YH[m] ^= ZH[m | 1];
            if (!(m & 2)) YL[m] ^= ZL[m | 2], YH[m] ^= ZH[m | 2];
        }
#define RS16_FDL(B)                                                                   \
        {                                                                             \
            const bool take = !(lane & (1u << (B)));                                  \
            _Pragma("unroll") for (int m = 0; m < 4; m++) {                           \
                const uint32_t pl = (uint32_t)xshfl<(1 << (B))>((int)ZL[m]);          \
                const uint32_t ph = (uint32_t)xshfl<(1 << (B))>((int)ZH[m]);          \
                YL[m] ^= take ? pl : 0u;                                              \
                YH[m] ^= take ? ph : 0u;                                              \
            }                                                                         \
        }
        RS16_FDL(0) RS16_FDL(1) RS16_FDL(2) RS16_FDL(3) RS16_FDL(4) RS16_FDL(5)
#undef RS16_FDL
    }
    // ---- FFT of the tile's 8 row bits, high layers first: blocks (6, 7),
    // (4, 5), (2, 3), (0, 1)
    auto tabs_of = [&](BlockTabs& bt, auto b0c, auto b1c) {
        constexpr int B0 = decltype(b0c)::value, B1 = decltype(b1c)::value;
        const uint32_t r0 = brow<B0, B1>(lane, 0), r2 = brow<B0, B1>(lane, 2);
        auto off = [](int kb, uint32_t r) { return (((1u << T) - (1u << (T - kb))) + (r >> (kb + 1))) * 80u; };
        lds_table(bt.w0, tabs, off(B0, r0));
        lds_table(bt.w2, tabs, off(B0, r2));
        lds_table(bt.w1, tabs, off(B1, r0));
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    using I5 = std::integral_constant<int, 5>;
    using I6 = std::integral_constant<int, 6>;
    using I7 = std::integral_constant<int, 7>;
    RS16_STAMP(a, 3);
    BlockTabs ta, tb;
    tabs_of(ta, I6(), I7());
    tabs_of(tb, I4(), I5());
    compute<true, true, true>(YL, YH, ta);
    wave_exchange<4, 5>(YL, YH);
    tabs_of(ta, I2(), I3());
    compute<true, true, true>(YL, YH, tb);
    wave_exchange<2, 3>(YL, YH);
    tabs_of(tb, I0(), I1());
    compute<true, true, true>(YL, YH, ta);
    wave_exchange<0, 1>(YL, YH);
    compute<true, true, true>(YL, YH, tb);
    RS16_STAMP(a, 9);
    // ---- reveal (x (65535 - e)) and store the lost originals in place
    // (restored-originals row = work row - the originals' segment start)
    const int64_t shift = (int64_t)a.row_base_out - (a.rest_seg_b ? (int64_t)a.chunk : 0);
#pragma unroll
    for (int m = 0; m < 4; m++) {
        if (!lost[m]) continue;
        uint32_t ol = 0, oh = 0;
        mul_xor(ol, oh, YL[m], YH[m], rt[m]);
        const int64_t rr = (int64_t)(tile << T) + 4 * lane + m + shift;
        uint32_t* p = (uint32_t*)(a.rest + rr * (int64_t)a.S_rest + offL);
        // (plain stores: 32768:32768 1 %-loss decode 103.1 -> 101.5 us against
        // non-temporal ones, same-box A/B x 3)
        p[0] = ol;
        p[8] = oh;
    }
    RS16_STAMP(a, 10);
    RS16_STAMP_END(a);
}

hipError_t launch_tile_last(const PassArgs& a, uint32_t num_tiles, hipStream_t s) {
    if (num_tiles == 0 || a.qrow == 0) return hipSuccess;
    const uint32_t nwg = num_tiles * ((a.qrow + 3) / 4);
    hipLaunchKernelGGL(tile_last_kernel, dim3(nwg), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The general decode's middle pass as a direct product.  DEC_MID is the same
// linear map u = FFT_hi (I + H) IFFT_hi z on every tile column j (rows
// t << lo | j; its twiddles do not involve j), a 2^hi x 2^hi matrix M over
// GF(2^16) (mid_matrix_entries, rs16_tables.cpp).  When the lost originals
// lie in few last-pass tiles, DEC_LAST consumes only the U rows t in
// [nlo, nhi) -- nhi - nlo <= MID_DIRECT_MAX -- and each is a sum over the
// live z rows (DEC_FIRST tiles with a received row, zflags):
//   u[o << lo | j] = sum over live t of M[o][t] z[t << lo | j]
// -- (nhi - nlo) x (live rows) multiplies per column instead of DEC_MID's
// 2^hi-point IFFT, derivative and output-pruned FFT (at the reference
// bench's 1 % loss: 2 x 129 against ~1300 butterflies, and one dispatch
// round instead of two).  Workgroup = (column j, 64-quad slab, stripe);
// its 8 waves take the rows t = w mod 8 (the zero tiles cluster, so
// interleaved), all of a wave's rows requested at once, and multiply them by
// the tables of rows [nlo, nhi) of M in LDS (one LDS-DMA copy of the
// contiguous v_perm tables), then XOR their partial sums through LDS; wave o
// stores row nlo + o.  A stripe whose consumed rows exceed
// MID_DIRECT_MAX returns here and DEC_MID computes it (PassArgs::mid_direct).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(512) mid_direct_kernel(PassArgs a, const uint32_t* mtab, uint32_t hi) {
    constexpr uint32_t W = 8, RPW = 256 / W;  // waves; rows per wave at 2^hi = 256
    extern __shared__ __attribute__((aligned(16))) uint8_t mlds[];
    // blockIdx.x = column j x slabs + 64-quad slab (one index: the stamps' workgroup id)
    const uint32_t nslab = (a.qrow + 63) / 64;
    const uint32_t j = blockIdx.x / nslab, slab = blockIdx.x - j * nslab;
    const uint32_t t0 = threadIdx.x, lane = t0 & 63, w = uni(t0 >> 6);
    if (blockIdx.z) {  // stripe z (PassArgs::stripe_tiles convention: displacements per stripe)
        const uint32_t st = blockIdx.z;
        a.in += st * a.bs_in;
        a.out += st * a.bs_out;
        if (a.zflags) a.zflags += st * a.bs_zflags;
        a.lostrange += st * a.bs_lost;
    }
    uint32_t nlo, nhi;
    if (!mid_need(a, nlo, nhi)) return;
    const uint32_t N = 1u << hi, nout = nhi - nlo, rpw = N / W;
    RS16_STAMP(a, 0);
    const uint32_t Qg = slab * 64 + lane;
    const bool active = Qg < a.qrow;
    const uint32_t offL = (Qg >> 3) * 64 + (Qg & 7) * 4;
    const uint8_t* zpage = a.zero + (offL & 0x7FFFu);
    // The wave's rows t = w + 8 u (a dead row -- DEC_FIRST tile without a
    // received row -- reads the zero page) and the tables of rows [nlo, nhi)
    // of M (LDS-DMA, L2-resident after the first workgroups).
    // (lane u reads row u's zero-tile flag: one load and a ballot)
    const bool lv_lane = lane < rpw && !(a.zflags && a.zflags[w + W * lane]);
    const uint64_t live = __ballot(lv_lane);
    const uint8_t* rbase = a.in + ((uint64_t)w << a.lo | j) * a.S_in;
    const uint64_t rstride = ((uint64_t)W << a.lo) * a.S_in;
    // Rows in batches of RPB: batch b + 1 is requested once batch b has
    // landed, before batch b's multiplies.  (All rows requested at once land
    // together at the end of the chip-wide load phase and the VALU idles
    // through it: 14.8 us per workgroup, half of it loads,
    // `profiles/r05_mid_direct.txt`.)
    constexpr uint32_t RPB = 8, NB = RPW / RPB;
    uint32_t zl[2][RPB], zh[2][RPB];
    auto fetch = [&](uint32_t b, uint32_t (&l)[RPB], uint32_t (&h)[RPB]) {
#pragma unroll
        for (uint32_t v = 0; v < RPB; v++) {
            const uint32_t u = b * RPB + v;
            const uint32_t* p = (const uint32_t*)(active && ((live >> u) & 1u) ? rbase + u * rstride + offL : zpage);
            l[v] = p[0];
            h[v] = p[8];
        }
    };
    fetch(0, zl[0], zh[0]);
    uint4* tabs = (uint4*)mlds;
    colops::dma_copy_rt<W * 64>((const uint8_t*)(mtab + (size_t)nlo * N * 20), mlds, nout * N * 80);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();  // tables in LDS
    RS16_STAMP(a, 1);
    uint32_t acc[MID_DIRECT_MAX][2] = {};
    auto multiply = [&](uint32_t b, const uint32_t (&l)[RPB], const uint32_t (&h)[RPB]) {
#pragma unroll
        for (uint32_t v = 0; v < RPB; v++) {
            const uint32_t u = b * RPB + v;
            if (!((live >> u) & 1u)) continue;  // (uniform)
            const uint32_t t = w + W * u;
#pragma unroll
            for (uint32_t o = 0; o < MID_DIRECT_MAX; o++) {
                if (o >= nout) break;
                uint32_t tt[20];
                load_table_lds(tt, tabs + (o * N + t) * 5);
                mul_xor(acc[o][0], acc[o][1], l[v], h[v], tt);
            }
        }
    };
#pragma unroll
    for (uint32_t b = 0; b < NB; b++) {
        if (b * RPB >= rpw) break;  // (uniform: 2^hi < 256)
        if (b + 1 < NB && (b + 1) * RPB < rpw) fetch(b + 1, zl[(b + 1) & 1], zh[(b + 1) & 1]);
        multiply(b, zl[b & 1], zh[b & 1]);
        __builtin_amdgcn_s_waitcnt(vmcnt_wait(0));
    }
    RS16_STAMP(a, 2);
    // XOR the waves' partial sums: row o by wave o
    __syncthreads();  // (the tables are no longer read: the partials reuse their LDS)
    uint2* part = (uint2*)mlds;
#pragma unroll
    for (uint32_t o = 0; o < MID_DIRECT_MAX; o++)
        if (o < nout) part[(w * MID_DIRECT_MAX + o) * 64 + lane] = make_uint2(acc[o][0], acc[o][1]);
    __syncthreads();
    if (w < nout) {
        uint32_t xl = 0, xh = 0;
#pragma unroll
        for (uint32_t v = 0; v < W; v++) {
            const uint2 q = part[(v * MID_DIRECT_MAX + w) * 64 + lane];
            xl ^= q.x;
            xh ^= q.y;
        }
        if (active) {
            uint32_t* p = (uint32_t*)(a.out + ((uint64_t)(nlo + w) << a.lo | j) * a.S_out + offL);
            p[0] = xl;
            p[8] = xh;
        }
    }
    RS16_STAMP_END(a);
}

hipError_t launch_mid_direct(const PassArgs& a, const uint32_t* mtab, uint32_t hi, uint32_t ns, hipStream_t s) {
    if (a.qrow == 0 || ns == 0) return hipSuccess;
    const uint32_t N = 1u << hi;
    // tables of up to MID_DIRECT_MAX rows (bounded by the host's consumed range)
    const uint32_t rows = std::min(MID_DIRECT_MAX, a.need_hi > a.need_lo ? a.need_hi - a.need_lo : 0u);
    if (rows == 0 || hi > 8 || hi < 3) return rows == 0 ? hipSuccess : hipErrorInvalidValue;
    const size_t lds = std::max((size_t)rows * N * 80, (size_t)8 * MID_DIRECT_MAX * 64 * 8);
    if (lds > 65536) {  // (as launch_pass: set on every call, i.e. on the current device)
        hipError_t e = hipFuncSetAttribute((const void*)mid_direct_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(mid_direct_kernel, dim3((1u << a.lo) * ((a.qrow + 63) / 64), 1, ns), dim3(512), lds, s, a, mtab,
                       hi);
    return hipGetLastError();
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
    RS16_ROW(DEC_HALF_LAST), RS16_ROW(DEC_HALF_SINGLE),
};
#undef RS16_ROW

#define RS16_SM(P)                                                                                             \
    {Smem<P, 0>::BYTES, Smem<P, 1>::BYTES, Smem<P, 2>::BYTES, Smem<P, 3>::BYTES, Smem<P, 4>::BYTES,             \
     Smem<P, 5>::BYTES, Smem<P, 6>::BYTES, Smem<P, 7>::BYTES, Smem<P, 8>::BYTES}
static const int kSmem[NUM_PROGS][9] = {
    RS16_SM(GEN_FFT),    RS16_SM(GEN_IFFT),  RS16_SM(ENC_FIRST), RS16_SM(ENC_MID),  RS16_SM(ENC_LAST),
    RS16_SM(ENC_SINGLE), RS16_SM(DEC_FIRST), RS16_SM(DEC_MID),   RS16_SM(DEC_LAST), RS16_SM(DEC_SINGLE),
    RS16_SM(DEC_HALF_LAST), RS16_SM(DEC_HALF_SINGLE),
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
    a.ntiles = num_tiles;
    const uint32_t nwg = num_tiles * a.nslab;  // one workgroup per (tile, slab) item
    if (a.need_hi == 0) a.need_hi = 1u << T;  // no pruning
    {
        const uint64_t hws = kQuads[T] >= 64 ? 1 : 64 / kQuads[T];
        const uint64_t smax = std::max(std::max(a.S_in, a.S_out), std::max(a.S_seg, a.S_rest));
        const uint64_t span = (uint64_t)1 << (T + a.lo);  // rows of one tile's aligned block
        const bool fits = (hws - 1) * ((uint64_t)16 << a.lo) * smax + 1024 < ((uint64_t)1 << 32);
        const bool aligned = a.chunk % span == 0 && a.row_base_in % span == 0;
        // (RS16_DIAG_FORCE_VOFF64: always the 64-bit lane offsets)
        a.voff32 = fits && aligned && !(a.diag & DIAG_FORCE_VOFF64) ? 1u : 0u;
        a.fd_lds = (a.diag & DIAG_FD_LDS) ? 1u : 0u;
    }
    const size_t lds = (size_t)kSmem[prog][T];
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)kPass[prog][T], hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
        if (e != hipSuccess) return e;
    }
    dim3 grid(nwg), block(kThreads[T]);
    hipLaunchKernelGGL(kPass[prog][T], grid, block, lds, s, a);
    return hipGetLastError();
}

}  // namespace rs16
