// rs16_col.hip -- one-launch codec for transforms of 512 / 1024 rows (the
// n <= 2048 configurations of BASELINE configs[1] / [2], 1000:1000 shards).
//
// What it computes: a whole single-chunk encode (HighRateEncoder::encode,
// src/rate/rate_high.rs:44-83, and LowRateEncoder::encode with one recovery
// chunk, src/rate/rate_low.rs:44-83) or a whole half-transform decode
// (every original lost; rate_high.rs:168-247) in ONE kernel:
//
//   ENC: x = rows [0, in_rows) of `in` (rows above zero)
//        out[0, out_rows) = FFT_skew_fft(IFFT_skew_ifft(x))
//   DEC: x[r] = received(r) ? in[r] * e[base_in + r] : 0           (gather)
//        out[r] = FFT_skew_fft(IFFT_skew_ifft(x))[r] * (65535 - e[base_out + r])
//
// with the reference's butterflies (engine_naive.rs:43-124): FFT layer of
// distance d = 2^kb: a ^= b * skew[g + d + delta - 1]; b ^= a (g = group
// start), IFFT: b ^= a; a ^= b * skew[...], the GF_MODULUS sentinel mapped to
// the all-zero v_perm table (skew_tab, rs16_tables.cpp).
//
// Why one launch: at 1000:1000 x 1 KiB the three-pass codec is a chain of
// latency-bound kernels of 128-256 one-wave workgroups (CHANGELOG.md round 3).  Here
// every quad column (8 bytes of each row: 4 elements, an independent set of
// codewords, src/algorithm.md:18-32) is one workgroup that keeps the whole
// column -- 2^L rows x 8 bytes, 8 KiB at L = 10 -- resident for all 2L layers:
//
//   * 2^L / 4 threads (4 waves at L = 10, one per SIMD), 4 rows per thread.
//     Layers go in radix-4 blocks over two row bits (b0, b1): the thread's
//     4 rows are its index with b0 / b1 inserted, so both layers of a block
//     are in registers.  Between blocks the row bits of registers and lanes
//     trade places inside the wave -- DPP lane swaps for lane bits 0-3,
//     v_permlane16/32_swap for bits 4-5, no LDS and no barrier -- except
//     around the block whose row bits are the wave index (two exchanges
//     through an 8 KiB LDS image, XOR-swizzled so that the b64 accesses are
//     bank-conflict free).
//   * The 2 (2^L - 1) twiddle tables of the codec (80-byte v_perm tables,
//     rs16_gf.hpp) come from contiguous images the engine builds on first use
//     (HostTables::col_img): those of layers 0 and 1 (3/4 of them, each used
//     by one thread in one block) straight into the thread's registers, those
//     of layers >= 2 into LDS by LDS-DMA loads (global_load_lds_dwordx4, no
//     VGPRs, no address arithmetic; 40 KiB at L = 10) issued behind the row
//     loads (the decoder: behind its polynomial, ColEval) so that the
//     compiler's vmcnt waits on the rows do not drain the DMA.
//   * The IFFT's last block and the FFT's first share their row bits: no
//     exchange between the two directions.
//   * Rows are loaded straight into the first block's layout and stored from
//     the last one's (rows 4t .. 4t + 3); a workgroup reads all of its rows
//     before it writes any, so in / out may alias (the work-buffer API).
//   * Workgroups are dealt to XCDs so that the 16 quad columns of a 128-byte
//     line run on one XCD (one HBM fetch per line and XCD).
#include "rs16_internal.hpp"
#include "rs16_fwht.hpp"
#include "rs16_colops.hpp"
#include "rs16_diag.hpp"

// (timing A/B builds: 0 = the radix-2 decoder's eval with 16-term wave layers)
#ifndef RS16_COL_EVAL_XP
#define RS16_COL_EVAL_XP 1
#endif

namespace rs16 {

namespace {
using namespace colops;

// LDS layout (bytes).  The tables of layers 0 and 1 (3/4 of each
// direction's 2^L - 1) are each used by one thread in one block (the first
// IFFT block, the last FFT block): every thread loads its own straight from
// the image into registers at the start (load_tabs01_img), so LDS holds
// layers 2 .. L-1 of both directions only, staged by LDS-DMA (2 (N/4 - 1)
// x 80 bytes, 40 KiB at L = 10), the row image and the erasure logs:
//   IMG the row image of the LDS exchanges (N x 8 bytes)
//   A   the IFFT's tables of groups >= G2 (layer kb at group N - 2^(L-kb),
//       group j = row >> (kb+1); G2 = 3N/4 = the first group of layer 2)
//   B   the FFT's, likewise
//   ELOG the decoder's erasure logs / polynomial scratch (2N x 4 bytes)
// (an encode launches ELOG bytes, the IFFT-only encode B: more workgroups
// per CU)
template <int L> struct ColSmem {
    static constexpr int N = 1 << L;
    static constexpr int G0 = N - N / 4;  // first group of layer 2
    static constexpr int IMG = 0;
    static constexpr int A = IMG + N * 8;
    static constexpr int B = A + (N - 1 - G0) * 80;
    static constexpr int ELOG = B + (N - 1 - G0) * 80;
    static constexpr int BYTES = ELOG + 2 * N * 4;
    static_assert(L >= (int)COL_LMIN && L <= (int)COL_LMAX, "the column codec covers 2^6 .. 2^10 rows");
};

// The general decoder's 2^11-row transform (COL_DEC_GEN only): the same
// layout (its logs: N x 4 bytes).
template <> struct ColSmem<11> {
    static constexpr int N = 2048;
    static constexpr int G0 = N - N / 4;  // first group of layer 2
    static constexpr int IMG = 0;
    static constexpr int A = IMG + N * 8;
    static constexpr int B = A + (N - 1 - G0) * 80;
    static constexpr int ELOG = B + (N - 1 - G0) * 80;
    static constexpr int BYTES = ELOG + N * 4;
};

// LDS byte offset of the table of layer kb for row r, direction FFT or not.
template <int L, bool FFT> __device__ __forceinline__ uint32_t tab_off(int kb, uint32_t r) {
    constexpr int N = 1 << L;
    const uint32_t t = (uint32_t)(N - (N >> kb)) + (r >> (kb + 1));
    // (layers >= 2 only: layers 0 and 1 come from registers, load_tabs01_img)
    return (FFT ? ColSmem<L>::B : ColSmem<L>::A) + (t - ColSmem<L>::G0) * 80u;
}

template <int L, bool FFT, int B0, int B1, bool D0, bool D1>
__device__ __forceinline__ void load_tabs(BlockTabs& w, uint32_t t, const uint8_t* smem) {
    const uint32_t r0 = brow<B0, B1>(t, 0), r2 = brow<B0, B1>(t, 2);
    if (D0) {
        lds_table(w.w0, smem, tab_off<L, FFT>(B0, r0));
        lds_table(w.w2, smem, tab_off<L, FFT>(B0, r2));
    }
    if (D1) lds_table(w.w1, smem, tab_off<L, FFT>(B1, r0));
}
template <int L> __device__ __forceinline__ void load_tabs01_img(BlockTabs& w, uint32_t t, const uint8_t* img) {
    constexpr uint32_t N = 1u << L;
    const uint32_t r0 = brow<0, 1>(t, 0), r2 = brow<0, 1>(t, 2);
    img_table(w.w0, img, r0 >> 1);
    img_table(w.w2, img, r2 >> 1);
    img_table(w.w1, img, N / 2 + (r0 >> 2));
}

// Rows of block (B0, B1) -> LDS image; barrier; rows of block (C0, C1) <- image.
// (Each thread writes back exactly the rows it read at the previous
// exchange, so no barrier is needed between an exchange's read and the next
// exchange's write.)
struct NoMid {
    __device__ __forceinline__ void operator()() const {}
};
template <int B0, int B1, int C0, int C1, class MID = NoMid>
__device__ __forceinline__ void exchange(uint32_t (&XL)[4], uint32_t (&XH)[4], uint32_t t, uint8_t* smem,
                                         MID mid = MID()) {
    uint2* img = (uint2*)smem;
#pragma unroll
    for (int m = 0; m < 4; m++) img[swz(brow<B0, B1>(t, m))] = make_uint2(XL[m], XH[m]);
    __syncthreads();
    mid();
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const uint2 v = img[swz(brow<C0, C1>(t, m))];
        XL[m] = v.x;
        XH[m] = v.y;
    }
}


// ---------------------------------------------------------------------------
// eval_poly inside the decoder (COL_DEC_EVAL, high rate, n = 2N <= 2048 work
// rows).  The reference evaluates H(LogWalsh . H(e)) over 65536 points
// (src/engine.rs:207-218; erasure vector from rate_high.rs:183-197).  With e
// zero outside [0, n) and only outputs in [0, n) needed, that is the XOR
// convolution out[i] = sum_j e[j] W[i ^ j], W = H(LogWalsh), i.e.
// H_n(H_n(e) . V) with the constant V = n^-1 H_n(W[0, n)) (HostTables::col_v):
// two n-point transforms per workgroup instead of a separate kernel.  Exact
// integers (|H_n(e)| <= n, |H_n(Y)| <= n 65535), reduced mod 65535 (65535 and
// 0 are the same log to every consumer, exp[65535] == exp[0]).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t fold65535(uint32_t u) {
    u = (u & 0xFFFFu) + (u >> 16);
    return (u & 0xFFFFu) + (u >> 16);
}
__device__ __forceinline__ uint32_t mod65535(int v) { return fold65535((uint32_t)(v + 65535 * 4096)); }

// In-place n-point integer FWHT of the workgroup's points p = t + NT j
// (x[j] in thread t): register layers (bits of j), lane layers (shuffles),
// wave layers through the LDS scratch `sx` (n ints).  Ends with a barrier
// (sx free again).
template <int NT, int PTS> __device__ __forceinline__ void fwht_points(int (&x)[PTS], int* sx) {
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
    for (int d = 1; d < PTS; d <<= 1)
#pragma unroll
        for (int j = 0; j < PTS; j++)
            if (!(j & d)) {
                const int u = x[j], v = x[j + d];
                x[j] = u + v;
                x[j + d] = u - v;
            }
#define RS16_LANE(D)                                              \
    if constexpr ((D) < NT) {                                     \
        _Pragma("unroll") for (int j = 0; j < PTS; j++) {         \
            const int p = xshfl<(D)>(x[j]);                       \
            x[j] = (lane & (D)) ? p - x[j] : x[j] + p;            \
        }                                                         \
    }
    RS16_LANE(1) RS16_LANE(2) RS16_LANE(4) RS16_LANE(8)
#undef RS16_LANE
    // lane bits 4 and 5: trade places with register bit 0 (v_permlane16_swap /
    // v_permlane32_swap, no LDS), butterfly the register pairs, trade back
#pragma unroll
    for (int lb = 4; lb <= 5 && (1 << lb) < NT; lb++)
#pragma unroll
        for (int j = 0; j < PTS; j += 2) {
            auto sw = [&]() {
                const auto r = lb == 4 ? __builtin_amdgcn_permlane16_swap((uint32_t)x[j], (uint32_t)x[j + 1], false, false)
                                       : __builtin_amdgcn_permlane32_swap((uint32_t)x[j], (uint32_t)x[j + 1], false, false);
                x[j] = (int)r[0];
                x[j + 1] = (int)r[1];
            };
            sw();
            const int u = x[j], v = x[j + 1];
            x[j] = u + v;
            x[j + 1] = u - v;
            sw();
        }
    constexpr int NW = NT / 64;
    if constexpr (NW > 1) {
#pragma unroll
        for (int j = 0; j < PTS; j++) sx[t + NT * j] = x[j];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PTS; j++) {
            int acc = 0;
#pragma unroll
            for (int v = 0; v < NW; v++) {
                const int y = sx[lane + 64 * v + NT * j];
                acc += (__builtin_popcount(w & (uint32_t)v) & 1) ? -y : y;
            }
            x[j] = acc;
        }
        __syncthreads();
    }
}

// The same transform with its wave layers as lane layers (XP forms of
// ColEval, the radix-2 kernel): the points go once through LDS to layout X,
// where the wave bits of the thread index and its lane bits 0 .. WB-1 trade
// places, and back.  The wave layers of the 16-wave workgroups read 16
// values per point (fwht_points); here a point is read once per transpose.
// LDS addresses XOR-swizzled (bank = p ^ (p >> 6)): conflict-free both ways.
template <int NT> struct XLay {
    static constexpr int WB = NT >= 1024 ? 4 : NT >= 512 ? 3 : NT >= 256 ? 2 : NT >= 128 ? 1 : 0;
    static constexpr uint32_t LM = (1u << WB) - 1;
    // the point of thread t's register j in layout X (layout O: t + NT j)
    static __device__ __forceinline__ uint32_t px(uint32_t t, int j) {
        const uint32_t lane = t & 63, w = t >> 6;
        return w | (lane & 63u & ~LM) | ((lane & LM) << 6) | (uint32_t)j * NT;
    }
    static __device__ __forceinline__ uint32_t sw(uint32_t p) { return p ^ ((p >> 6) & 63u); }
};
// register layers, then lane layers of lane bits [B0, B1)
template <int PTS, int B0, int B1, bool REG> __device__ __forceinline__ void fwht_lanes(int (&x)[PTS]) {
    const uint32_t lane = threadIdx.x & 63;
    if constexpr (REG) {
#pragma unroll
        for (int d = 1; d < PTS; d <<= 1)
#pragma unroll
            for (int j = 0; j < PTS; j++)
                if (!(j & d)) {
                    const int u = x[j], v = x[j + d];
                    x[j] = u + v;
                    x[j + d] = u - v;
                }
    }
#define RS16_LANE(B)                                              \
    if constexpr ((B) >= B0 && (B) < B1) {                        \
        _Pragma("unroll") for (int j = 0; j < PTS; j++) {         \
            const int p = xshfl<(1 << (B))>(x[j]);                \
            x[j] = (lane & (1u << (B))) ? p - x[j] : x[j] + p;    \
        }                                                         \
    }
    RS16_LANE(0) RS16_LANE(1) RS16_LANE(2) RS16_LANE(3)
#undef RS16_LANE
#pragma unroll
    for (int lb = 4; lb <= 5; lb++) {
        if (lb < B0 || lb >= B1) continue;
#pragma unroll
        for (int j = 0; j < PTS; j += 2) {
            auto swp = [&]() {
                const auto r = lb == 4 ? __builtin_amdgcn_permlane16_swap((uint32_t)x[j], (uint32_t)x[j + 1], false, false)
                                       : __builtin_amdgcn_permlane32_swap((uint32_t)x[j], (uint32_t)x[j + 1], false, false);
                x[j] = (int)r[0];
                x[j + 1] = (int)r[1];
            };
            swp();
            const int u = x[j], v = x[j + 1];
            x[j] = u + v;
            x[j + 1] = u - v;
            swp();
        }
    }
}
// layout O -> X (TO_X) or X -> O through sx; barrier after the writes
template <int NT, int PTS, bool TO_X> __device__ __forceinline__ void fwht_xpose(int (&x)[PTS], int* sx) {
    using X = XLay<NT>;
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < PTS; j++) sx[X::sw(TO_X ? t + NT * j : X::px(t, j))] = x[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PTS; j++) x[j] = sx[X::sw(TO_X ? X::px(t, j) : t + NT * j)];
}

// The erasure logs of work rows [0, NT PTS) into elds, and the received
// counts per 64-row chunk (rcount, workgroup 0) for rs16_decode_check.
// Segment A = recovery rows [0, in_rows) (flags), [in_rows, chunk) padding
// (erased), segment B = originals [chunk, chunk + o_rows) (flags_o), zero
// above (rate_high.rs:183-197).  PTS = 8: the half decode's 2N work rows;
// PTS = 4: the general decode's N.
// In two steps: load() issues every load (the flag bytes and V of the
// thread's points) -- the kernel calls it before its row loads and table
// DMA, so that waiting for them does not wait for the DMA (vmcnt counts in
// issue order) -- and run() computes.
template <int L, int PTS, int NT_ = (1 << L) / 4, bool XP = false> struct ColEval {
    static constexpr int N = 1 << L, NT = NT_;
    uint8_t f[PTS];
    uint32_t vt[PTS];
    __device__ __forceinline__ void load(const ColArgs& a) {
        const uint32_t t = threadIdx.x;
#pragma unroll
        for (int j = 0; j < PTS; j++) {
            const uint32_t p = t + NT * j;
            const bool in_a = p < a.in_rows, in_b = p >= a.chunk && p - a.chunk < a.o_rows;
            const uint8_t* fp = in_a && a.flags ? a.flags + p : (in_b && a.flags_o ? a.flags_o + (p - a.chunk) : a.zero);
            f[j] = *(const __attribute__((address_space(1))) uint8_t*)fp;
            vt[j] = a.vtab[XP ? XLay<NT>::px(t, j) : p];  // (XP: the product is taken in layout X)
        }
    }
    // the erasure vector of the thread's points (and the received counts):
    // the first use of the loaded bytes
    int x[PTS];
    __device__ __forceinline__ void prep(const ColArgs& a) {
        const uint32_t t = threadIdx.x, lane = t & 63;
        uint32_t ca = 0, cb = 0;
#pragma unroll
        for (int j = 0; j < PTS; j++) {
            const uint32_t p = t + NT * j;
            const bool in_a = p < a.in_rows, in_b = p >= a.chunk && p - a.chunk < a.o_rows;
            const bool rcv = in_a ? (!a.flags || f[j]) : (in_b && (!a.flags_o || f[j]));
            x[j] = (in_a || in_b) ? !rcv : (int)(p < a.chunk ? a.e_pad : a.e_tail);
            if (blockIdx.x == 0 && a.rcount) {
                // (below 64 threads a 64-row chunk spans 64 / NT values of j)
                constexpr int PER = NT >= 64 ? 1 : 64 / NT;
                ca += (uint32_t)__popcll(__ballot(rcv && in_a));
                cb += (uint32_t)__popcll(__ballot(rcv && in_b));
                if ((j + 1) % PER == 0) {
                    if (lane == 0) {
                        a.rcount[2 * (p >> 6)] = ca;
                        a.rcount[2 * (p >> 6) + 1] = cb;
                    }
                    ca = cb = 0;
                }
            }
        }
    }
    __device__ __forceinline__ void run(const ColArgs& a, uint32_t* elds) {
        const uint32_t t = threadIdx.x;
        int* sx = (int*)elds;
        if constexpr (XP) {
            constexpr int WB = XLay<NT>::WB;
            // H(e): every bit but the wave bits in layout O, those in X
            fwht_lanes<PTS, 0, 6, true>(x);
            fwht_xpose<NT, PTS, true>(x, sx);
            fwht_lanes<PTS, 0, WB, false>(x);
#pragma unroll
            for (int j = 0; j < PTS; j++) x[j] = (int)fold65535(mod65535(x[j]) * vt[j]);
            // H(.): every bit but point bits [0, WB) in X, those in O
            fwht_lanes<PTS, 0, 6, true>(x);
            __syncthreads();  // (every thread has read its X points)
            fwht_xpose<NT, PTS, false>(x, sx);
            __syncthreads();  // (elds overwrites sx)
            fwht_lanes<PTS, 0, WB, false>(x);
#pragma unroll
            for (int j = 0; j < PTS; j++) elds[t + NT * j] = mod65535(x[j] + (int)a.e_k);
            return;
        }
        fwht_points<NT, PTS>(x, sx);
        RS16_STAMP(a, 2);
#pragma unroll
        for (int j = 0; j < PTS; j++) x[j] = (int)fold65535(mod65535(x[j]) * vt[j]);
        fwht_points<NT, PTS>(x, sx);
        RS16_STAMP(a, 3);
#pragma unroll
        for (int j = 0; j < PTS; j++) elds[t + NT * j] = mod65535(x[j] + (int)a.e_k);
    }
};

// The formal derivative (Engine::formal_derivative, src/engine.rs:233-238) of
// the whole column, in the closed form out[j] = d[j] ^ XOR{ d[j | 2^b] : bit b
// of j is 0 }, between the general decoder's IFFT and FFT:
// register bits from registers, every other bit from an LDS image of d.
template <int L, int B0, int B1>
__device__ __forceinline__ void col_fd(uint32_t (&XL)[4], uint32_t (&XH)[4], uint32_t t, uint8_t* smem) {
    uint2* img = (uint2*)(smem + ColSmem<L>::IMG);
    __syncthreads();  // (every wave is past its IFFT tables and earlier image reads)
#pragma unroll
    for (int m = 0; m < 4; m++) img[swz(brow<B0, B1>(t, m))] = make_uint2(XL[m], XH[m]);
    __syncthreads();
    uint32_t AL[4], AH[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const uint32_t j = brow<B0, B1>(t, m);
        uint32_t al = XL[m], ah = XH[m];
        if (!(m & 1)) al ^= XL[m | 1], ah ^= XH[m | 1];
        if (!(m & 2)) al ^= XL[m | 2], ah ^= XH[m | 2];
#pragma unroll
        for (int b = 0; b < L; b++) {
            if (b == B0 || b == B1) continue;
            const uint2 v = img[swz(j | (1u << b))];
            const bool take = !((j >> b) & 1u);
            al ^= take ? v.x : 0u;
            ah ^= take ? v.y : 0u;
        }
        AL[m] = al;
        AH[m] = ah;
    }
#pragma unroll
    for (int m = 0; m < 4; m++) XL[m] = AL[m], XH[m] = AH[m];
    __syncthreads();  // (the image is free again)
}

template <int L, int MODE>
__global__ __launch_bounds__((1 << L) / 4) void col_kernel(ColArgs a) {
    constexpr bool DEC = MODE != COL_ENC, GEN = MODE == COL_DEC_GEN;
    constexpr bool EVAL = MODE == COL_DEC_EVAL || GEN;  // the polynomial in the kernel
    constexpr int N = 1 << L, NT = N / 4;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t t = threadIdx.x;
    RS16_STAMP(a, 0);

    // workgroup -> (stripe, quad column), XCD-aware: consecutive columns on
    // one XCD (workgroups are dealt to the 8 XCDs round-robin)
    const uint32_t total = a.qrow * a.nstripes;
    uint32_t g = blockIdx.x;
    if ((total & 7u) == 0) g = (g & 7u) * (total >> 3) + (g >> 3);
    const uint32_t st = g / a.qrow, q = g - st * a.qrow;
    const uint32_t offL = (q >> 3) * 64u + (q & 7u) * 4u;
    const uint8_t* in = a.in + st * a.bs_in + offL;
    uint8_t* out = a.out + st * a.bs_out + offL;
    // stripes with losses of their own (all strides 0 when shared)
    if (a.flags) a.flags += st * a.bs_flags;
    if (a.flags_o) a.flags_o += st * a.bs_flags_o;
    if (a.elog) a.elog += st * a.bs_elog;

    // ---- requests: the rows, the tables (LDS-DMA), the decoder's erasure data
    // (the compiler drains every LDS-DMA load at the first use of an ordinary
    // load while one is in flight: the decoder's polynomial starts once the
    // tables are in)
    auto dma_tables = [&]() {
        constexpr int G0 = ColSmem<L>::G0;
        dma_copy<NT>(a.img_ifft + G0 * 80, smem + ColSmem<L>::A, (N - 1 - G0) * 80);
        dma_copy<NT>(a.img_fft + G0 * 80, smem + ColSmem<L>::B, (N - 1 - G0) * 80);
    };
    // ---- the decoder's erasure data first: the gather rows' received flags,
    // the polynomial's inputs (EVAL) or eval_poly's output (EWORK), issued
    // ahead of the row loads and the table DMA so that the polynomial can
    // start as soon as they land (a wait for them would otherwise include
    // every DMA issued before them; vmcnt counts in issue order)
    [[maybe_unused]] uint8_t fr[4] = {0, 0, 0, 0};
    [[maybe_unused]] ColEval<L, (DEC && EVAL) ? (GEN ? 4 : 8) : 1> ce;
    [[maybe_unused]] uint32_t zv[2][4];
    if constexpr (DEC) {
#pragma unroll
        for (int m = 0; m < 4; m++) {
            // (branch-free: rows outside both segments read a zero byte)
            const uint32_t r = 4 * t + m;
            const bool in_a = r < a.in_rows, in_b = GEN && r >= a.chunk && r - a.chunk < a.o_rows;
            const uint8_t* fp = in_a && a.flags ? a.flags + r : (in_b && a.flags_o ? a.flags_o + (r - a.chunk) : a.zero);
            fr[m] = *(const __attribute__((address_space(1))) uint8_t*)fp;
        }
        if constexpr (EVAL) {
            ce.load(a);
        } else if constexpr (L >= 9) {
            const uint32_t w = t >> 6, lane = t & 63;
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int j = 0; j < 4; j++) zv[b][j] = a.elog[(2 * w + b) * 256 + lane + 64 * j];
        }
    }
    // the tables of the first IFFT block and the last FFT block (layers 0
    // and 1, one thread each) straight into registers (L = 11: at their blocks)
    BlockTabs ta, tb, t01f;
    if constexpr (L <= 10) {
        load_tabs01_img<L>(ta, t, a.img_ifft);
        load_tabs01_img<L>(t01f, t, a.img_fft);
    }
    uint32_t XL[4], XH[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const uint32_t r = 4 * t + m;
        // (a row that is not read comes from the zero page, RS16_ZERO_BYTES;
        // the decoder zeroes rows that were not received with its multiply)
        const uint8_t* src = a.zero + (offL & 0x7FFFu);
        if (r < a.in_rows) src = in + (size_t)r * a.S_in;
        // (the general decoder also gathers the received originals, rows [chunk, chunk + o_rows))
        if (GEN && r >= a.chunk && r - a.chunk < a.o_rows) src = a.in_b + st * a.bs_in_b + offL + (size_t)(r - a.chunk) * a.S_in;
        const uint32_t* p = (const uint32_t*)src;
        XL[m] = p[0];
        XH[m] = p[8];
    }
    // (the encoder stages its tables now; the decoder after its polynomial:
    // with an LDS-DMA load in flight, the compiler makes a use of any
    // ordinary load -- and a workgroup barrier -- wait for every load, DMA
    // included, and the polynomial needs both)
    if constexpr (!DEC) dma_tables();
    uint32_t gt[DEC ? 4 : 1][20];
    uint32_t ev[4] = {0, 0, 0, 0};
    bool lost[4] = {false, false, false, false};  // (GEN: the row is a lost original)
    if constexpr (DEC) {
        bool rcv[4];
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint32_t r = 4 * t + m;
            rcv[m] = r < a.in_rows && (!a.flags || fr[m] != 0);
            if (GEN && a.rev_a && r < a.in_rows) lost[m] = !rcv[m];  // (low rate: originals = segment A)
            if (GEN && r >= a.chunk && r - a.chunk < a.o_rows) {
                rcv[m] = !a.flags_o || fr[m] != 0;
                if (!a.rev_a) lost[m] = !rcv[m];
            }
        }
        uint32_t* elds = (uint32_t*)(smem + ColSmem<L>::ELOG);
        if constexpr (EVAL) {
            ce.prep(a);
            ce.run(a, elds);
            __syncthreads();
        } else if constexpr (L >= 9) {
            // eval_poly's output before its last 256-point FWHT (a.elog = the
            // engine's ework, loaded above): wave w finishes the blocks of rows
            // [512 w, 512 w + 512) (src/engine.rs:207-218) into LDS, for the
            // work rows this codec reads
            const uint32_t w = t >> 6, lane = t & 63;
#pragma unroll
            for (int b = 0; b < 2; b++) {
                fwht256_wave(zv[b]);
#pragma unroll
                for (int j = 0; j < 4; j++) elds[(2 * w + b) * 256 + lane + 64 * j] = zv[b][j];
            }
            __syncthreads();
        }
        // gather multipliers: the v_perm table of each received row's log
        // (MULTIPLY SHARDS, rate_high.rs:203-228: other rows times zero)
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint32_t r = 4 * t + m;
            glb_table(gt[m], a.mul_tab, rcv[m] ? elds[a.base_in + r] : ZERO_ENTRY);
            ev[m] = elds[a.base_out + r];
        }
        // the tables stream in behind the gather multipliers' loads (the
        // multiply below waits for both)
        dma_tables();
    }
    RS16_STAMP(a, 1);
    if constexpr (DEC) {
#pragma unroll
        for (int m = 0; m < 4; m++) {
            uint32_t zl = 0, zh = 0;
            mul_xor(zl, zh, XL[m], XH[m], gt[m]);
            XL[m] = zl;
            XH[m] = zh;
        }
    }
    if constexpr (L == 11) {
        __builtin_amdgcn_s_waitcnt(0);  // (the LDS-DMA loads have landed)
        __syncthreads();
    }
    RS16_STAMP(a, 2);

    // ---- IFFT (layers 0 .. L-1) then FFT (L-1 .. 0) in radix-4 blocks; the
    // next block's tables are read before each exchange.  Row bits 0-5 are
    // lane bits of some block (in-wave exchanges); from L = 9 on the top ones
    // are wave bits (two LDS exchanges); L = 7 ends with a one-layer block on
    // bits (4, 6).
  if constexpr (L == 11) {
    // the general decoder over 2^11 work rows (8 waves; row bits 6-10 of
    // some blocks are wave bits: four LDS exchanges, the last IFFT / first
    // FFT layer as a one-layer block on bits (8, 10))
    static_assert(GEN, "2^11 rows: the general decoder only");
    load_tabs01_img<L>(ta, t, a.img_ifft);
    compute<false, true, true>(XL, XH, ta);
    RS16_STAMP(a, 3);
    load_tabs<L, false, 2, 3, true, true>(tb, t, smem);
    wave_exchange<0, 1>(XL, XH);
    compute<false, true, true>(XL, XH, tb);
    load_tabs<L, false, 4, 5, true, true>(ta, t, smem);
    wave_exchange<2, 3>(XL, XH);
    compute<false, true, true>(XL, XH, ta);
    RS16_STAMP(a, 4);
    load_tabs<L, false, 6, 7, true, true>(tb, t, smem);
    wave_exchange<4, 5>(XL, XH);
    compute<false, true, true>(XL, XH, tb);
    load_tabs<L, false, 8, 9, true, true>(ta, t, smem);
    exchange<6, 7, 8, 9>(XL, XH, t, smem);
    compute<false, true, true>(XL, XH, ta);
    load_tabs<L, false, 8, 10, false, true>(tb, t, smem);
    __syncthreads();  // (every wave has read its rows of the image)
    exchange<8, 9, 8, 10>(XL, XH, t, smem);
    compute<false, false, true>(XL, XH, tb);
    RS16_STAMP(a, 5);
    col_fd<L, 8, 10>(XL, XH, t, smem);
    load_tabs<L, true, 8, 10, false, true>(tb, t, smem);
    compute<true, false, true>(XL, XH, tb);
    load_tabs<L, true, 8, 9, true, true>(ta, t, smem);
    __syncthreads();
    exchange<8, 10, 8, 9>(XL, XH, t, smem);
    compute<true, true, true>(XL, XH, ta);
    RS16_STAMP(a, 6);
    load_tabs<L, true, 6, 7, true, true>(tb, t, smem);
    __syncthreads();
    exchange<8, 9, 6, 7>(XL, XH, t, smem);
    compute<true, true, true>(XL, XH, tb);
    load_tabs<L, true, 4, 5, true, true>(ta, t, smem);
    wave_exchange<4, 5>(XL, XH);
    compute<true, true, true>(XL, XH, ta);
    RS16_STAMP(a, 7);
    load_tabs<L, true, 2, 3, true, true>(tb, t, smem);
    wave_exchange<2, 3>(XL, XH);
    compute<true, true, true>(XL, XH, tb);
    load_tabs01_img<L>(tb, t, a.img_fft);
    wave_exchange<0, 1>(XL, XH);
    RS16_STAMP(a, 8);
  } else {
    compute<false, true, true>(XL, XH, ta);  // (layers 0, 1: tables from registers)
    __builtin_amdgcn_s_waitcnt(0);  // (the LDS-DMA loads of layers >= 2 have landed)
    __syncthreads();
    RS16_STAMP(a, 3);
    load_tabs<L, false, 2, 3, true, true>(tb, t, smem);
    wave_exchange<0, 1>(XL, XH);
    compute<false, true, true>(XL, XH, tb);
    load_tabs<L, false, 4, 5, true, true>(ta, t, smem);
    wave_exchange<2, 3>(XL, XH);
    compute<false, true, true>(XL, XH, ta);
    RS16_STAMP(a, 4);
    if constexpr (L == 6) {
        // the FFT's first block keeps the row bits (4, 5)
        RS16_STAMP(a, 5);
        if constexpr (GEN) col_fd<L, 4, 5>(XL, XH, t, smem);
        load_tabs<L, true, 4, 5, true, true>(ta, t, smem);
        RS16_STAMP(a, 6);
    } else if constexpr (L == 7) {
        load_tabs<L, false, 4, 6, false, true>(tb, t, smem);
        swap_bit<1, 4>(XL);  // register bit 1: row bit 5 -> 6
        swap_bit<1, 4>(XH);
        compute<false, false, true>(XL, XH, tb);
        RS16_STAMP(a, 5);
        if constexpr (GEN) col_fd<L, 4, 6>(XL, XH, t, smem);
        load_tabs<L, true, 4, 6, false, true>(tb, t, smem);
        compute<true, false, true>(XL, XH, tb);
        load_tabs<L, true, 4, 5, true, true>(ta, t, smem);
        swap_bit<1, 4>(XL);
        swap_bit<1, 4>(XH);
        RS16_STAMP(a, 6);
    } else {
        load_tabs<L, false, 6, 7, true, true>(tb, t, smem);
        wave_exchange<4, 5>(XL, XH);
        compute<false, true, true>(XL, XH, tb);
        if constexpr (L == 8) {
            RS16_STAMP(a, 5);
            if constexpr (GEN) col_fd<L, 6, 7>(XL, XH, t, smem);
            load_tabs<L, true, 6, 7, true, true>(ta, t, smem);
        } else if constexpr (L == 10) {
            load_tabs<L, false, 8, 9, true, true>(ta, t, smem);
            exchange<6, 7, 8, 9>(XL, XH, t, smem);
            compute<false, true, true>(XL, XH, ta);
            RS16_STAMP(a, 5);
            if constexpr (GEN) col_fd<L, 8, 9>(XL, XH, t, smem);
            // the FFT's first block keeps the row bits: no exchange
            load_tabs<L, true, 8, 9, true, true>(tb, t, smem);
            compute<true, true, true>(XL, XH, tb);
            load_tabs<L, true, 6, 7, true, true>(ta, t, smem);
            __syncthreads();  // (every wave has read its rows of the image)
            exchange<8, 9, 6, 7>(XL, XH, t, smem);
        } else {
            load_tabs<L, false, 7, 8, false, true>(ta, t, smem);
            exchange<6, 7, 7, 8>(XL, XH, t, smem);
            compute<false, false, true>(XL, XH, ta);
            RS16_STAMP(a, 5);
            if constexpr (GEN) col_fd<L, 7, 8>(XL, XH, t, smem);
            load_tabs<L, true, 7, 8, false, true>(tb, t, smem);
            compute<true, false, true>(XL, XH, tb);
            load_tabs<L, true, 6, 7, true, true>(ta, t, smem);
            __syncthreads();  // (every wave has read its rows of the image)
            exchange<7, 8, 6, 7>(XL, XH, t, smem);
        }
        RS16_STAMP(a, 6);
        compute<true, true, true>(XL, XH, ta);
        load_tabs<L, true, 4, 5, true, true>(ta, t, smem);
        wave_exchange<4, 5>(XL, XH);
    }
    compute<true, true, true>(XL, XH, ta);
    RS16_STAMP(a, 7);
    load_tabs<L, true, 2, 3, true, true>(tb, t, smem);
    wave_exchange<2, 3>(XL, XH);
    compute<true, true, true>(XL, XH, tb);
    tb = t01f;  // (layers 1, 0: tables from registers)
    wave_exchange<0, 1>(XL, XH);
    RS16_STAMP(a, 8);
  }
    uint32_t rt[DEC ? 4 : 1][20];
    if constexpr (DEC) {
        // reveal multipliers (requested here so the tables are in flight
        // under the last block)
#pragma unroll
        for (int m = 0; m < 4; m++) glb_table(rt[m], a.mul_tab, GF_MODULUS - ev[m]);
    }
    compute<true, true, true>(XL, XH, tb);
    RS16_STAMP(a, 9);

    // ---- store rows 4t + m < out_rows (DEC: revealed, rate_high.rs:236-242)
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const uint32_t r = 4 * t + m;
        uint32_t vl = XL[m], vh = XH[m];
        if constexpr (DEC) {
            uint32_t zl = 0, zh = 0;
            mul_xor(zl, zh, vl, vh, rt[m]);
            vl = zl;
            vh = zh;
        }
        const bool st_ok = GEN ? lost[m] : r < a.out_rows;
        if (st_ok) {
            uint32_t* p = (uint32_t*)(out + (size_t)(GEN && !a.rev_a ? r - a.chunk : r) * a.S_out);
            __builtin_nontemporal_store(vl, p);
            __builtin_nontemporal_store(vh, p + 8);
        }
    }
    RS16_STAMP(a, 10);
    RS16_STAMP_END(a);
}


// ---------------------------------------------------------------------------
// Radix-2 form of the encode and the half decode for 2^8 .. 2^10 rows
// (col2_kernel): 2 rows per thread, 2^(L-1) threads -- 8 waves at L = 10, two
// per SIMD -- instead of 4 rows in 2^(L-2) threads.  The codec's time at
// 1000:1000 x 1 KiB is the dependency chain of one wave (one per SIMD, 128
// workgroups on 256 CUs, CHANGELOG.md round 4): halving a lane's rows halves the
// chain, and the second wave of each SIMD issues into the first one's
// stalls, at the price of one in-wave row-bit swap per layer instead of per
// two.  A layer's butterfly pairs the thread's two rows (register bit RB);
// lane bits trade places with RB by DPP / v_permlane swaps (swap2), wave
// bits by two LDS exchanges around the top layers.  Row-bit maps (RMap<RB,
// P...>: P_i = the row bit held by thread-index bit i):
//   S(k)  the IFFT's layer k <= 6: RB = k, lanes b0 .. b6 without b_k,
//         waves b7 .. (rows 2t, 2t + 1 at S(0): loads and stores contiguous)
//   M     layers 7 .. L-1: RB = b7, lanes (b0, b1, b2, b3, b8, b9 / b4),
//         waves the rest (16 consecutive lanes, consecutive rows: the b64
//         image accesses are conflict-free without a swizzle)
// ---------------------------------------------------------------------------
template <int RB, int... P> struct RMap {
    static constexpr int BITS = sizeof...(P);
    static __device__ __forceinline__ uint32_t row(uint32_t t, uint32_t m) {
        uint32_t r = m << RB;
        int i = 0;
        ((r |= ((t >> i++) & 1u) << P), ...);
        return r;
    }
};
// S(k) and M of a 2^L-row column (L = 8 .. 10)
template <int L, int K> struct SMap;
#define RS16_S(K, ...)                                                       \
    template <> struct SMap<11, K> { using M = RMap<K, __VA_ARGS__, 7, 8, 9, 10>; }; \
    template <> struct SMap<7, K> { using M = RMap<K, __VA_ARGS__>; };          \
    template <> struct SMap<8, K> { using M = RMap<K, __VA_ARGS__, 7>; };       \
    template <> struct SMap<9, K> { using M = RMap<K, __VA_ARGS__, 7, 8>; };    \
    template <> struct SMap<10, K> { using M = RMap<K, __VA_ARGS__, 7, 8, 9>; };
RS16_S(0, 1, 2, 3, 4, 5, 6)
RS16_S(1, 0, 2, 3, 4, 5, 6)
RS16_S(2, 0, 1, 3, 4, 5, 6)
RS16_S(3, 0, 1, 2, 4, 5, 6)
RS16_S(4, 0, 1, 2, 3, 5, 6)
RS16_S(5, 0, 1, 2, 3, 4, 6)
RS16_S(6, 0, 1, 2, 3, 4, 5)
#undef RS16_S
template <int L> struct MMap;
template <> struct MMap<8> { using M = RMap<7, 0, 1, 2, 3, 4, 5, 6>; };
template <> struct MMap<9> { using M = RMap<7, 0, 1, 2, 3, 8, 4, 5, 6>; };
template <> struct MMap<10> { using M = RMap<7, 0, 1, 2, 3, 8, 9, 4, 5, 6>; };
// L = 11: lanes (b0, b1, b2, b8, b9, b10), waves (b3, b4, b5, b6); lane bits
// 3 / 4 / 5 then hold b8 / b9 / b10 for the in-wave swaps of the middle
template <> struct MMap<11> { using M = RMap<7, 0, 1, 2, 8, 9, 10, 3, 4, 5, 6>; };
template <> struct SMap<11, 8> { using M = RMap<8, 0, 1, 2, 7, 9, 10, 3, 4, 5, 6>; };
template <> struct SMap<11, 9> { using M = RMap<9, 0, 1, 2, 7, 8, 10, 3, 4, 5, 6>; };
template <> struct SMap<11, 10> { using M = RMap<10, 0, 1, 2, 7, 8, 9, 3, 4, 5, 6>; };
// after the swap of lane bit 4 (L >= 9) / 5 (L = 10) in M: the register holds b8 / b9
template <> struct SMap<9, 8> { using M = RMap<8, 0, 1, 2, 3, 7, 4, 5, 6>; };
template <> struct SMap<10, 8> { using M = RMap<8, 0, 1, 2, 3, 7, 9, 4, 5, 6>; };
template <> struct SMap<10, 9> { using M = RMap<9, 0, 1, 2, 3, 7, 8, 4, 5, 6>; };
template <> struct SMap<8, 7> { using M = RMap<7, 0, 1, 2, 3, 4, 5, 6>; };
template <> struct SMap<9, 7> { using M = RMap<7, 0, 1, 2, 3, 8, 4, 5, 6>; };
template <> struct SMap<10, 7> { using M = RMap<7, 0, 1, 2, 3, 8, 9, 4, 5, 6>; };

// Trade the register bit with lane bit LB (rows m = 0, 1; see swap_bit).
template <int LB> __device__ __forceinline__ void swap2(uint32_t (&X)[2]) {
    if constexpr (LB == 4 || LB == 5) {
        const auto r = LB == 4 ? __builtin_amdgcn_permlane16_swap(X[0], X[1], false, false)
                               : __builtin_amdgcn_permlane32_swap(X[0], X[1], false, false);
        X[0] = r[0];
        X[1] = r[1];
    } else {
        const bool hi = (threadIdx.x >> LB) & 1u;
        const uint32_t u = (uint32_t)xshfl<(1 << LB)>((int)X[0]);
        const uint32_t v = (uint32_t)xshfl<(1 << LB)>((int)X[1]);
        X[1] = hi ? X[1] : u;
        X[0] = hi ? v : X[0];
    }
}
template <int LB> __device__ __forceinline__ void swap2(uint32_t (&XL)[2], uint32_t (&XH)[2]) {
    swap2<LB>(XL);
    swap2<LB>(XH);
}
template <bool FFT> __device__ __forceinline__ void bfly2(uint32_t (&XL)[2], uint32_t (&XH)[2], const uint32_t (&w)[20]) {
    if (FFT) {
        mul_xor(XL[0], XH[0], XL[1], XH[1], w);
        XL[1] ^= XL[0], XH[1] ^= XH[0];
    } else {
        XL[1] ^= XL[0], XH[1] ^= XH[0];
        mul_xor(XL[0], XH[0], XL[1], XH[1], w);
    }
}
// table of layer KB (>= 2: LDS) for the thread's pair under map MP
template <int L, bool FFT, int KB, class MP>
__device__ __forceinline__ void tab2(uint32_t (&w)[20], uint32_t t, const uint8_t* smem) {
    lds_table(w, smem, tab_off<L, FFT>(KB, MP::row(t, 0)));
}
// layers 0 and 1 straight from the table image (group index of the image:
// layer kb at N - 2^(L-kb), row >> (kb + 1))
template <int L, int KB, class MP>
__device__ __forceinline__ void tab2_img(uint32_t (&w)[20], uint32_t t, const uint8_t* img) {
    constexpr uint32_t N = 1u << L;
    img_table(w, img, (N - (N >> KB)) + (MP::row(t, 0) >> (KB + 1)));
}
// rows of map A -> LDS image; barrier; rows of map B <- image
template <class A, class B>
__device__ __forceinline__ void exchange2(uint32_t (&XL)[2], uint32_t (&XH)[2], uint32_t t, uint8_t* img8) {
    uint2* img = (uint2*)img8;
#pragma unroll
    for (int m = 0; m < 2; m++) img[A::row(t, m)] = make_uint2(XL[m], XH[m]);
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 2; m++) {
        const uint2 v = img[B::row(t, m)];
        XL[m] = v.x;
        XH[m] = v.y;
    }
}

// The formal derivative (closed form, col_fd) of the radix-2 kernel's rows
// at the middle, where the register holds row bit RB: that term from the
// register pair, every other bit's from an LDS image of the column.
template <class MP, int L, int RB>
__device__ __forceinline__ void col2_fd(uint32_t (&XL)[2], uint32_t (&XH)[2], uint32_t t, uint8_t* img8) {
    uint2* img = (uint2*)img8;
    __syncthreads();  // (every wave is past its earlier image reads)
#pragma unroll
    for (int m = 0; m < 2; m++) img[MP::row(t, m)] = make_uint2(XL[m], XH[m]);
    __syncthreads();
    uint32_t AL[2], AH[2];
#pragma unroll
    for (int m = 0; m < 2; m++) {
        const uint32_t j = MP::row(t, m);
        uint32_t al = XL[m], ah = XH[m];
        if (m == 0) al ^= XL[1], ah ^= XH[1];
#pragma unroll
        for (int b = 0; b < L; b++) {
            if (b == RB) continue;
            const uint2 v = img[j | (1u << b)];
            const bool take = !((j >> b) & 1u);
            al ^= take ? v.x : 0u;
            ah ^= take ? v.y : 0u;
        }
        AL[m] = al;
        AH[m] = ah;
    }
#pragma unroll
    for (int m = 0; m < 2; m++) XL[m] = AL[m], XH[m] = AH[m];
}

template <int L, int MODE>
__global__ __launch_bounds__((1 << L) / 2) void col2_kernel(ColArgs a) {
    static_assert(L >= 8 && L <= 11 && (L <= 10 || MODE == COL_DEC_GEN) && MODE != COL_DEC_EWORK,
                  "radix-2 column codec");
    constexpr bool DEC = MODE == COL_DEC_EVAL || MODE == COL_DEC_GEN, GEN = MODE == COL_DEC_GEN;
    // the high rate's multi-chunk encode in two launches: IFO = the IFFT of
    // chunk blockIdx.y of originals, stored whole; FFX = the FFT of the XOR
    // of a.nch such chunks (launch_col, rs16_engine::encode_high_multi)
    constexpr bool IFO = MODE == COL_ENC_IFFT, FFX = MODE == COL_ENC_FFTX;
    constexpr int N = 1 << L, NT = N / 2;
    using S0 = typename SMap<L, 0>::M;
    using S6 = typename SMap<L, 6>::M;
    using MM = typename MMap<L>::M;
    using FM = typename SMap<L, L - 1>::M;  // the rows' map between the IFFT's last layer and the FFT's first
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t t = threadIdx.x;
    RS16_STAMP(a, 0);

    const uint32_t total = a.qrow * a.nstripes;
    uint32_t g = blockIdx.x;
    if ((total & 7u) == 0) g = (g & 7u) * (total >> 3) + (g >> 3);
    const uint32_t st = g / a.qrow, q = g - st * a.qrow;
    const uint32_t offL = (q >> 3) * 64u + (q & 7u) * 4u;
    const uint8_t* in = a.in + st * a.bs_in + offL;
    uint8_t* out = a.out + st * a.bs_out + offL;
    if (a.flags) a.flags += st * a.bs_flags;
    if (a.flags_o) a.flags_o += st * a.bs_flags_o;
    // Multi-chunk encodes (grid row ch = blockIdx.y; images of consecutive
    // skew deltas are consecutive, HostTables::col_img): ENC = the low rate's
    // recovery chunk ch (FFT skew (ch + 1) 2^L, rows ch 2^L ..), IFO = the
    // high rate's chunk ch of originals (IFFT skew (ch + 1) 2^L)
    const uint32_t ch = blockIdx.y;
    uint32_t in_rows = a.in_rows, out_rows = a.out_rows;
    const uint8_t* img_ifft = a.img_ifft;
    const uint8_t* img_fft = a.img_fft;
    if constexpr (MODE == COL_ENC) {
        out += (size_t)ch * N * a.S_out;
        out_rows -= ch * N;
        img_fft += (size_t)ch * (N - 1) * 80;
    }
    if constexpr (IFO) {
        in += (size_t)ch * N * a.S_in;
        in_rows -= ch * N;
        out += (size_t)ch * N * a.S_out;
        img_ifft += (size_t)ch * (N - 1) * 80;
    }

    auto dma_tables = [&]() {
        constexpr int G0 = ColSmem<L>::G0;
        if constexpr (!FFX) dma_copy<NT>(img_ifft + G0 * 80, smem + ColSmem<L>::A, (N - 1 - G0) * 80);
        if constexpr (!IFO) dma_copy<NT>(img_fft + G0 * 80, smem + ColSmem<L>::B, (N - 1 - G0) * 80);
    };
    // segments of a row (GEN: A = rows [0, in_rows), B = [chunk, chunk + o_rows))
    auto in_a = [&](uint32_t r) { return r < in_rows; };
    auto in_b = [&](uint32_t r) { return GEN && r >= a.chunk && r - a.chunk < a.o_rows; };
    // ---- requests, as col_kernel: the decoder's flags and polynomial
    // inputs first, then the layer-0/1 tables into registers, the rows, the DMA
    [[maybe_unused]] uint8_t fr[2] = {0, 0};
    [[maybe_unused]] ColEval<L, (DEC ? (GEN ? N : 2 * N) / NT : 1), NT, RS16_COL_EVAL_XP> ce;
    if constexpr (DEC) {
#pragma unroll
        for (int m = 0; m < 2; m++) {
            const uint32_t r = S0::row(t, m);
            const uint8_t* fp = in_a(r) && a.flags ? a.flags + r
                                                   : (in_b(r) && a.flags_o ? a.flags_o + (r - a.chunk) : a.zero);
            fr[m] = *(const __attribute__((address_space(1))) uint8_t*)fp;
        }
        ce.load(a);
    }
    // (the FFT's layer-0/1 tables are requested after the prologue, under
    // the IFFT: the prologue is bound by the CU's L2 bandwidth, and a thread's
    // own tables for layers 0 and 1 are most of its bytes)
    uint32_t i0[20], i1[20], f0[20], f1[20];
    // GEN: requested with the per-row tables after the eval, by the waves
    // whose block is live (the eval's first barrier would wait for every
    // wave's table requests; 1 %-loss 1000:1000 decode 16.1 -> 15.4 us)
    constexpr bool LATE_I01 = GEN;
    if constexpr (FFX) {
        tab2_img<L, 0, S0>(f0, t, img_fft);
        tab2_img<L, 1, typename SMap<L, 1>::M>(f1, t, img_fft);
    } else if constexpr (!LATE_I01) {
        tab2_img<L, 0, S0>(i0, t, img_ifft);
        tab2_img<L, 1, typename SMap<L, 1>::M>(i1, t, img_ifft);
    }
    uint32_t XL[2], XH[2];
    if constexpr (FFX) {
        // the XOR of the nch chunks' rows (rate_high.rs:56-74), in map FM
#pragma unroll
        for (int m = 0; m < 2; m++) XL[m] = XH[m] = 0;
#pragma unroll 4
        for (uint32_t c = 0; c < a.nch; c++) {
#pragma unroll
            for (int m = 0; m < 2; m++) {
                const uint32_t* p = (const uint32_t*)(in + ((size_t)c * N + FM::row(t, m)) * a.S_in);
                XL[m] ^= p[0];
                XH[m] ^= p[8];
            }
        }
    } else {
#pragma unroll
        for (int m = 0; m < 2; m++) {
            const uint32_t r = S0::row(t, m);
            const uint8_t* src = a.zero + (offL & 0x7FFFu);
            if (in_a(r)) src = in + (size_t)r * a.S_in;
            if (in_b(r)) src = a.in_b + st * a.bs_in_b + offL + (size_t)(r - a.chunk) * a.S_in;
            const uint32_t* p = (const uint32_t*)src;
            XL[m] = p[0];
            XH[m] = p[8];
        }
    }
    // IFO: every row of the chunk, from the map after the IFFT's last layer
    auto store_mid = [&]() {
#pragma unroll
        for (int m = 0; m < 2; m++) {
            uint32_t* p = (uint32_t*)(out + (size_t)FM::row(t, m) * a.S_out);
            p[0] = XL[m];
            p[8] = XH[m];
        }
    };
    // (a decoder's DMA follows its per-row tables: the general decode with it
    // before the eval, whole or its IFFT half, measured 0.4 us slower)
    if constexpr (!DEC) dma_tables();
    [[maybe_unused]] uint32_t ev[2] = {0, 0};
    [[maybe_unused]] bool lost[2] = {false, false};  // (GEN: the row is a lost original)
    // GEN: a wave's rows in the maps S(k) are one 128-row block (wave index =
    // row bits 7 ..); a block with no received row is zero through the
    // IFFT's layers 0 .. 6 (ilive: they are skipped), a block with no lost
    // original feeds no stored row from the FFT's layer 6 on (flive: skipped
    // with the reveal).  Uniform branches.
    bool ilive = true, flive = true;
    if constexpr (DEC) {
        bool rcv[2];
#pragma unroll
        for (int m = 0; m < 2; m++) {
            const uint32_t r = S0::row(t, m);
            rcv[m] = in_a(r) && (!a.flags || fr[m] != 0);
            if (GEN && a.rev_a && in_a(r)) lost[m] = !rcv[m];  // (low rate: originals = segment A)
            if (in_b(r)) {
                rcv[m] = !a.flags_o || fr[m] != 0;
                if (!a.rev_a) lost[m] = !rcv[m];
            }
        }
        if constexpr (GEN) {
            ilive = __ballot(rcv[0] || rcv[1]) != 0;
            flive = __ballot(lost[0] || lost[1]) != 0;
        }
        uint32_t* elds = (uint32_t*)(smem + ColSmem<L>::ELOG);
        ce.prep(a);
        RS16_STAMP(a, 1);
        ce.run(a, elds);
        __syncthreads();
        RS16_STAMP(a, 4);
        uint32_t gt[2][20];
        if constexpr (LATE_I01) {
            if (ilive) {
                tab2_img<L, 0, S0>(i0, t, img_ifft);
                tab2_img<L, 1, typename SMap<L, 1>::M>(i1, t, img_ifft);
            }
        }
#pragma unroll
        for (int m = 0; m < 2; m++) {
            const uint32_t r = S0::row(t, m);
            // (a zero block's rows need no table: the ZERO_ENTRY product is 0)
            if (ilive) glb_table(gt[m], a.mul_tab, rcv[m] ? elds[a.base_in + r] : ZERO_ENTRY);
            ev[m] = elds[a.base_out + r];
        }
        dma_tables();
#pragma unroll
        for (int m = 0; m < 2; m++) {
            uint32_t zl = 0, zh = 0;
            if (ilive) mul_xor(zl, zh, XL[m], XH[m], gt[m]);
            XL[m] = zl;
            XH[m] = zh;
        }
    }
    RS16_STAMP(a, 5);
    // Each layer's LDS table is read one layer ahead (wa / wb), so its
    // latency hides under the previous layer's swap and butterfly.
    uint8_t* img = smem + ColSmem<L>::IMG;
    uint32_t wa[20], wb[20];
    using S2 = typename SMap<L, 2>::M;
    using S3 = typename SMap<L, 3>::M;
    using S4 = typename SMap<L, 4>::M;
    using S5 = typename SMap<L, 5>::M;
    if constexpr (FFX) {
        __builtin_amdgcn_s_waitcnt(0);  // (the LDS-DMA loads of layers >= 2 have landed)
        __syncthreads();
    } else {
    // ---- IFFT layers 0 .. 6 in registers and lanes
    if (ilive) bfly2<false>(XL, XH, i0);
    __builtin_amdgcn_s_waitcnt(0);  // (the LDS-DMA loads of layers >= 2 have landed)
    __syncthreads();
    RS16_STAMP(a, 6);
    if constexpr (L <= 10 && !IFO) {
        if (flive) {
            tab2_img<L, 0, S0>(f0, t, img_fft);
            tab2_img<L, 1, typename SMap<L, 1>::M>(f1, t, img_fft);
        }
    }
    if (ilive) {
        tab2<L, false, 2, S2>(wa, t, smem);
        swap2<0>(XL, XH);
        bfly2<false>(XL, XH, i1);
        tab2<L, false, 3, S3>(wb, t, smem);
        swap2<1>(XL, XH);
        bfly2<false>(XL, XH, wa);
        tab2<L, false, 4, S4>(wa, t, smem);
        swap2<2>(XL, XH);
        bfly2<false>(XL, XH, wb);
        tab2<L, false, 5, S5>(wb, t, smem);
        swap2<3>(XL, XH);
        bfly2<false>(XL, XH, wa);
        tab2<L, false, 6, S6>(wa, t, smem);
        swap2<4>(XL, XH);
        bfly2<false>(XL, XH, wb);
        tab2<L, false, 7, MM>(wb, t, smem);
        swap2<5>(XL, XH);
        bfly2<false>(XL, XH, wa);
    } else {
        // (a zero block stays zero in any row map)
        tab2<L, false, 7, MM>(wb, t, smem);
    }
    RS16_STAMP(a, 7);
    }
    // ---- layers 7 .. L-1 both ways around the middle, map M (GEN: the
    // formal derivative between the IFFT's last layer and the FFT's first)
    if constexpr (L == 11) {
        using S8 = typename SMap<L, 8>::M;
        using S9 = typename SMap<L, 9>::M;
        using S10 = typename SMap<L, 10>::M;
        tab2<L, false, 8, S8>(wa, t, smem);
        exchange2<S6, MM>(XL, XH, t, img);
        bfly2<false>(XL, XH, wb);  // IFFT 7
        tab2<L, false, 9, S9>(wb, t, smem);
        swap2<3>(XL, XH);
        bfly2<false>(XL, XH, wa);  // IFFT 8
        tab2<L, false, 10, S10>(wa, t, smem);
        swap2<4>(XL, XH);
        bfly2<false>(XL, XH, wb);  // IFFT 9
        tab2<L, true, 10, S10>(wb, t, smem);
        swap2<5>(XL, XH);
        bfly2<false>(XL, XH, wa);  // IFFT 10
        col2_fd<S10, L, 10>(XL, XH, t, img);
        tab2<L, true, 9, S9>(wa, t, smem);
        bfly2<true>(XL, XH, wb);   // FFT 10
        tab2<L, true, 8, S8>(wb, t, smem);
        swap2<5>(XL, XH);
        bfly2<true>(XL, XH, wa);   // FFT 9
        tab2<L, true, 7, MM>(wa, t, smem);
        swap2<4>(XL, XH);
        bfly2<true>(XL, XH, wb);   // FFT 8
        tab2<L, true, 6, S6>(wb, t, smem);
        swap2<3>(XL, XH);
        bfly2<true>(XL, XH, wa);   // FFT 7
        // (at 16 waves the FFT's layer-0/1 tables are requested here: 128 VGPRs)
        if (flive) {
            tab2_img<L, 0, S0>(f0, t, a.img_fft);
            tab2_img<L, 1, typename SMap<L, 1>::M>(f1, t, a.img_fft);
        }
        __syncthreads();  // (every wave has read its derivative terms from the image)
    } else if constexpr (L == 10) {
        using S8 = typename SMap<L, 8>::M;
        using S9 = typename SMap<L, 9>::M;
        if constexpr (!FFX) {
            tab2<L, false, 8, S8>(wa, t, smem);
            exchange2<S6, MM>(XL, XH, t, img);
            bfly2<false>(XL, XH, wb);  // IFFT 7
            tab2<L, false, 9, S9>(wb, t, smem);
            swap2<4>(XL, XH);
            bfly2<false>(XL, XH, wa);  // IFFT 8
            if constexpr (!IFO) tab2<L, true, 9, S9>(wa, t, smem);
            swap2<5>(XL, XH);
            bfly2<false>(XL, XH, wb);  // IFFT 9
            if constexpr (IFO) {
                store_mid();
                return;
            }
            if constexpr (GEN) col2_fd<S9, L, 9>(XL, XH, t, img);
        } else {
            tab2<L, true, 9, S9>(wa, t, smem);
        }
        tab2<L, true, 8, S8>(wb, t, smem);
        bfly2<true>(XL, XH, wa);   // FFT 9
        tab2<L, true, 7, MM>(wa, t, smem);
        swap2<5>(XL, XH);
        bfly2<true>(XL, XH, wb);   // FFT 8
        tab2<L, true, 6, S6>(wb, t, smem);
        swap2<4>(XL, XH);
        bfly2<true>(XL, XH, wa);   // FFT 7
        if constexpr (GEN) __syncthreads();
    } else if constexpr (L == 9) {
        using S8 = typename SMap<L, 8>::M;
        if constexpr (!FFX) {
            tab2<L, false, 8, S8>(wa, t, smem);
            exchange2<S6, MM>(XL, XH, t, img);
            bfly2<false>(XL, XH, wb);  // IFFT 7
            if constexpr (!IFO) tab2<L, true, 8, S8>(wb, t, smem);
            swap2<4>(XL, XH);
            bfly2<false>(XL, XH, wa);  // IFFT 8
            if constexpr (IFO) {
                store_mid();
                return;
            }
            if constexpr (GEN) col2_fd<S8, L, 8>(XL, XH, t, img);
        } else {
            tab2<L, true, 8, S8>(wb, t, smem);
        }
        tab2<L, true, 7, MM>(wa, t, smem);
        bfly2<true>(XL, XH, wb);   // FFT 8
        tab2<L, true, 6, S6>(wb, t, smem);
        swap2<4>(XL, XH);
        bfly2<true>(XL, XH, wa);   // FFT 7
        if constexpr (GEN) __syncthreads();
    } else {
        if constexpr (!FFX) {
            if constexpr (!IFO) tab2<L, true, 7, MM>(wa, t, smem);
            exchange2<S6, MM>(XL, XH, t, img);
            bfly2<false>(XL, XH, wb);  // IFFT 7
            if constexpr (IFO) {
                store_mid();
                return;
            }
            if constexpr (GEN) col2_fd<MM, L, 7>(XL, XH, t, img);
        } else {
            tab2<L, true, 7, MM>(wa, t, smem);
        }
        tab2<L, true, 6, S6>(wb, t, smem);
        bfly2<true>(XL, XH, wa);   // FFT 7
        if constexpr (GEN) __syncthreads();
    }
    RS16_STAMP(a, 8);
    tab2<L, true, 5, S5>(wa, t, smem);
    // (each thread writes the image rows it read in the first exchange: no
    // barrier; GEN: the derivative's image reads are behind a barrier above)
    exchange2<MM, S6>(XL, XH, t, img);
    [[maybe_unused]] uint32_t rt[DEC ? 2 : 1][20];
    if (flive) {
        bfly2<true>(XL, XH, wb);  // FFT 6
        tab2<L, true, 4, S4>(wb, t, smem);
        swap2<5>(XL, XH);
        bfly2<true>(XL, XH, wa);
        tab2<L, true, 3, S3>(wa, t, smem);
        swap2<4>(XL, XH);
        bfly2<true>(XL, XH, wb);
        tab2<L, true, 2, S2>(wb, t, smem);
        swap2<3>(XL, XH);
        bfly2<true>(XL, XH, wa);
        swap2<2>(XL, XH);
        bfly2<true>(XL, XH, wb);
        swap2<1>(XL, XH);
        bfly2<true>(XL, XH, f1);
        if constexpr (DEC) {
#pragma unroll
            for (int m = 0; m < 2; m++) glb_table(rt[m], a.mul_tab, GF_MODULUS - ev[m]);
        }
        swap2<0>(XL, XH);
        bfly2<true>(XL, XH, f0);
    }
    RS16_STAMP(a, 9);
    // ---- store rows < out_rows (DEC: revealed, rate_high.rs:236-242; GEN:
    // the lost originals only, restored in place)
#pragma unroll
    for (int m = 0; m < 2 && flive; m++) {
        const uint32_t r = S0::row(t, m);
        uint32_t vl = XL[m], vh = XH[m];
        if constexpr (DEC) {
            uint32_t zl = 0, zh = 0;
            mul_xor(zl, zh, vl, vh, rt[m]);
            vl = zl;
            vh = zh;
        }
        const bool st_ok = GEN ? lost[m] : r < out_rows;
        if (st_ok) {
            // (plain stores: same-box A/B against non-temporal ones, 3 pairs:
            // 1000:1000 decode 11.38 -> 11.18 us, 512:512 7.55 -> 7.40)
            uint32_t* p = (uint32_t*)(out + (size_t)(GEN && !a.rev_a ? r - a.chunk : r) * a.S_out);
            p[0] = vl;
            p[8] = vh;
        }
    }
    RS16_STAMP(a, 10);
    RS16_STAMP_END(a);
}

// ---------------------------------------------------------------------------
// Multi-chunk encodes of 128-row chunks in one launch (colm_kernel): the
// reference benchmark rows 100:1000 and 1000:100 (README.md:130-131), whose
// pass form is several launches.  One workgroup per quad column, ONE WAVE PER
// CHUNK, 2 rows per lane (the radix-2 maps of col2_kernel restricted to the
// 7 row bits of a chunk: register + 6 lane bits, no LDS exchange):
//   high rate (HighRateEncoder::encode, rate_high.rs:44-83): wave c takes
//     originals [128 c, 128 c + 128) (rows >= k zero), IFFT skew 128 (c + 1);
//     the chunks are XORed through LDS into wave 0, which runs the FFT (skew
//     0) and stores recovery rows < m;
//   low rate (LowRateEncoder::encode, rate_low.rs:44-83): every wave takes
//     the originals (rows >= k zero), IFFT skew 0, then its own recovery
//     chunk's FFT, skew 128 (c + 1), and stores rows 128 c + r < m.
// Each wave stages its own twiddles (layers 2-6, 31 tables x 80 B per
// direction, LDS-DMA from skew_tab) and loads those of layers 0 / 1 straight
// into registers, so no barrier precedes the transforms.
// ---------------------------------------------------------------------------
constexpr uint32_t CM_N = 128, CM_TABS = 31, CM_TAB_BYTES = CM_TABS * 80;
__device__ __forceinline__ uint32_t cm_idx(uint32_t kb, uint32_t r, uint32_t skew) {
    return (r & ~((2u << kb) - 1u)) + (1u << kb) + skew - 1u;  // group start + d + skew - 1
}
// the 31 tables of layers 2-6 at `skew` into dst (table tb: layer kb at
// 32 - 2^(7-kb) + group), by the calling wave
__device__ __forceinline__ void cm_stage(const uint32_t* skew_tab, uint8_t* dst, uint32_t skew, uint32_t lane) {
#pragma unroll
    for (uint32_t i = 0; i * 64 < CM_TABS * 5; i++) {
        const uint32_t c = i * 64 + lane;
        if (c < CM_TABS * 5) {
            const uint32_t tb = c / 5, part = c - tb * 5;
            const uint32_t kb = (uint32_t)__clz(31u - tb) - 25u;  // (tb < 16: 2, < 24: 3, < 28: 4, < 30: 5, 30: 6)
            const uint32_t j = tb - (32u - (1u << (7u - kb)));
            const uint32_t idx = cm_idx(kb, j << (kb + 1), skew);
            __builtin_amdgcn_global_load_lds((glb_vp)(skew_tab + (size_t)idx * TAB_DWORDS + part * 4),
                                             (lds_vp)(dst + i * 64 * 16), 16, 0, 0);
        }
    }
}
template <int KB, class MP>
__device__ __forceinline__ void cm_tab(uint32_t (&w)[20], uint32_t lane, const uint8_t* base) {
    const uint32_t r = MP::row(lane, 0);
    lds_table(w, base, (32u - (1u << (7 - KB)) + (r >> (KB + 1))) * 80u);
}

template <bool HI>
__global__ __launch_bounds__(1024) void colm_kernel(ColArgs a) {
    using S0 = typename SMap<7, 0>::M;
    using S1 = typename SMap<7, 1>::M;
    using S2 = typename SMap<7, 2>::M;
    using S3 = typename SMap<7, 3>::M;
    using S4 = typename SMap<7, 4>::M;
    using S5 = typename SMap<7, 5>::M;
    using S6 = typename SMap<7, 6>::M;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t t = threadIdx.x, lane = t & 63, c = __builtin_amdgcn_readfirstlane(t >> 6);
    const uint32_t total = a.qrow * a.nstripes;
    uint32_t g = blockIdx.x;
    if ((total & 7u) == 0) g = (g & 7u) * (total >> 3) + (g >> 3);
    const uint32_t st = g / a.qrow, q = g - st * a.qrow;
    const uint32_t offL = (q >> 3) * 64u + (q & 7u) * 4u;
    const uint8_t* in = a.in + st * a.bs_in + offL;
    uint8_t* out = a.out + st * a.bs_out + offL;
    const uint32_t sk_i = HI ? (c + 1) * CM_N : 0u, sk_f = HI ? 0u : (c + 1) * CM_N;
    const bool fft_wave = !HI || c == 0;
    uint8_t* tI = smem + c * 2 * CM_TAB_BYTES;
    uint8_t* tF = tI + CM_TAB_BYTES;
    // ---- requests: layer-0/1 tables, rows, then the LDS-DMA of layers 2-6
    uint32_t i0[20], i1[20], f0[20], f1[20];
    glb_table(i0, a.skew_tab, cm_idx(0, S0::row(lane, 0), sk_i));
    glb_table(i1, a.skew_tab, cm_idx(1, S1::row(lane, 0), sk_i));
    uint32_t XL[2], XH[2];
#pragma unroll
    for (int m = 0; m < 2; m++) {
        const uint32_t r = (HI ? c * CM_N : 0u) + S0::row(lane, m);
        const uint8_t* src = a.zero + (offL & 0x7FFFu);
        if (r < a.in_rows) src = in + (size_t)r * a.S_in;
        XL[m] = ((const uint32_t*)src)[0];
        XH[m] = ((const uint32_t*)src)[8];
    }
    cm_stage(a.skew_tab, tI, sk_i, lane);
    if (fft_wave) cm_stage(a.skew_tab, tF, sk_f, lane);
    __builtin_amdgcn_s_waitcnt(0);  // (the wave's own rows and tables: no barrier)
    if (fft_wave) {  // (needed at the end: requested under the IFFT)
        glb_table(f0, a.skew_tab, cm_idx(0, S0::row(lane, 0), sk_f));
        glb_table(f1, a.skew_tab, cm_idx(1, S1::row(lane, 0), sk_f));
    }
    // ---- IFFT layers 0 .. 6 (register + lane bits)
    uint32_t wa[20], wb[20];
    cm_tab<2, S2>(wa, lane, tI);
    bfly2<false>(XL, XH, i0);
    swap2<0>(XL, XH);
    bfly2<false>(XL, XH, i1);
    cm_tab<3, S3>(wb, lane, tI);
    swap2<1>(XL, XH);
    bfly2<false>(XL, XH, wa);
    cm_tab<4, S4>(wa, lane, tI);
    swap2<2>(XL, XH);
    bfly2<false>(XL, XH, wb);
    cm_tab<5, S5>(wb, lane, tI);
    swap2<3>(XL, XH);
    bfly2<false>(XL, XH, wa);
    cm_tab<6, S6>(wa, lane, tI);
    swap2<4>(XL, XH);
    bfly2<false>(XL, XH, wb);
    swap2<5>(XL, XH);
    bfly2<false>(XL, XH, wa);
    if constexpr (HI) {
        // ---- XOR of the chunks' IFFTs (rate_high.rs:55-75) into wave 0
        uint2* img = (uint2*)(smem + a.nch * 2 * CM_TAB_BYTES);
        if (c != 0) {
#pragma unroll
            for (int m = 0; m < 2; m++) img[c * CM_N + S6::row(lane, m)] = make_uint2(XL[m], XH[m]);
        }
        __syncthreads();
        if (c != 0) return;
        for (uint32_t cc = 1; cc < a.nch; cc++) {
#pragma unroll
            for (int m = 0; m < 2; m++) {
                const uint2 v = img[cc * CM_N + S6::row(lane, m)];
                XL[m] ^= v.x;
                XH[m] ^= v.y;
            }
        }
    } else {
        // every wave has consumed its loaded originals (the IFFT used them)
        // before wave 0 stores recovery rows [0, 128): the Rate API encodes
        // in place, recovery over the originals (rate_low.rs:44-83)
        __syncthreads();
    }
    // ---- FFT layers 6 .. 0
    cm_tab<6, S6>(wa, lane, tF);
    cm_tab<5, S5>(wb, lane, tF);
    bfly2<true>(XL, XH, wa);
    cm_tab<4, S4>(wa, lane, tF);
    swap2<5>(XL, XH);
    bfly2<true>(XL, XH, wb);
    cm_tab<3, S3>(wb, lane, tF);
    swap2<4>(XL, XH);
    bfly2<true>(XL, XH, wa);
    cm_tab<2, S2>(wa, lane, tF);
    swap2<3>(XL, XH);
    bfly2<true>(XL, XH, wb);
    swap2<2>(XL, XH);
    bfly2<true>(XL, XH, wa);
    swap2<1>(XL, XH);
    bfly2<true>(XL, XH, f1);
    swap2<0>(XL, XH);
    bfly2<true>(XL, XH, f0);
    // ---- store recovery rows < m
#pragma unroll
    for (int m = 0; m < 2; m++) {
        const uint32_t r = (HI ? 0u : c * CM_N) + S0::row(lane, m);
        if (r < a.out_rows) {
            uint32_t* p = (uint32_t*)(out + (size_t)r * a.S_out);
            p[0] = XL[m];
            p[8] = XH[m];
        }
    }
}

}  // namespace

int col_rows_ok(uint32_t L) { return L >= COL_LMIN && L <= COL_LMAX; }

hipError_t launch_col_multi(const ColArgs& a, bool high, hipStream_t s) {
    if (a.nch == 0 || a.nch > COLM_MAX_CHUNKS) return hipErrorInvalidValue;
    if (a.qrow == 0 || a.nstripes == 0 || a.out_rows == 0) return hipSuccess;
    const int bytes = (int)(a.nch * 2 * CM_TAB_BYTES + (high ? a.nch * CM_N * 8 : 0));
    const auto fn = high ? colm_kernel<true> : colm_kernel<false>;
    // the LDS limit is a per-device attribute: set it for the current device
    // the first time this process launches there (engines on several GPUs)
    constexpr int MAX_DEV = 64;
    static bool attr[MAX_DEV][2] = {};  // (idempotent: a racing second call sets it again)
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    if (dev < 0 || dev >= MAX_DEV || !attr[dev][high]) {
        const int most = (int)(COLM_MAX_CHUNKS * 2 * CM_TAB_BYTES + COLM_MAX_CHUNKS * CM_N * 8);
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, most);
        if (e != hipSuccess) return e;
        if (dev >= 0 && dev < MAX_DEV) attr[dev][high] = true;
    }
    hipLaunchKernelGGL(fn, dim3(a.qrow * a.nstripes), dim3(64 * a.nch), bytes, s, a);
    return hipGetLastError();
}

hipError_t launch_col(const ColArgs& a, uint32_t L, int mode, hipStream_t s) {
    if (L < COL_LMIN || L > COL_LGEN || mode < COL_ENC || mode > COL_ENC_FFTX) return hipErrorInvalidValue;
    if (L == COL_LGEN && mode != COL_DEC_GEN) return hipErrorInvalidValue;
    // multi-chunk encodes: radix-2 form, one stripe, nch <= COL_MAX_CHUNKS
    const bool chunks = mode >= COL_ENC_IFFT || a.nch > 1;
    if (chunks && (L < COL_LCHUNK || L > COL_LMAX || a.nstripes != 1 || a.nch == 0 || a.nch > COL_MAX_CHUNKS ||
                   (mode != COL_ENC && mode < COL_ENC_IFFT)))
        return hipErrorInvalidValue;
    if (a.qrow == 0 || a.nstripes == 0 || a.out_rows == 0) return hipSuccess;
    typedef void (*ColFn)(ColArgs);
#define RS16_COL_ROW(L)                                                                                   \
    {col_kernel<L, COL_ENC>, L >= 9 ? col_kernel<L, COL_DEC_EWORK> : nullptr, col_kernel<L, COL_DEC_EVAL>, \
     col_kernel<L, COL_DEC_GEN>}
    static const ColFn fns[6][4] = {RS16_COL_ROW(6),  RS16_COL_ROW(7), RS16_COL_ROW(8), RS16_COL_ROW(9),
                                    RS16_COL_ROW(10), {nullptr, nullptr, nullptr, col_kernel<11, COL_DEC_GEN>}};
#undef RS16_COL_ROW
    static const int lds[6] = {ColSmem<6>::BYTES, ColSmem<7>::BYTES,  ColSmem<8>::BYTES,
                               ColSmem<9>::BYTES, ColSmem<10>::BYTES, ColSmem<11>::BYTES};
    ColFn fn = mode <= COL_DEC_GEN ? fns[L - COL_LMIN][mode] : nullptr;
    if (!fn && !chunks) return hipErrorInvalidValue;  // (the ework decoder needs 4 waves: L >= 9)
    uint32_t threads = (1u << L) / 4, rows = 1;
    if (chunks) {
        static const ColFn fnc[3][3] = {{col2_kernel<8, COL_ENC>, col2_kernel<8, COL_ENC_IFFT>, col2_kernel<8, COL_ENC_FFTX>},
                                        {col2_kernel<9, COL_ENC>, col2_kernel<9, COL_ENC_IFFT>, col2_kernel<9, COL_ENC_FFTX>},
                                        {col2_kernel<10, COL_ENC>, col2_kernel<10, COL_ENC_IFFT>, col2_kernel<10, COL_ENC_FFTX>}};
        fn = fnc[L - COL_LCHUNK][mode == COL_ENC ? 0 : mode - COL_ENC_IFFT + 1];
        threads = (1u << L) / 2;
        rows = mode == COL_ENC_FFTX ? 1 : a.nch;  // (one grid row per chunk)
    } else if (mode != COL_DEC_EWORK && L >= 8 && !(a.diag & DIAG_COL_RADIX4)) {
        // the encode and the half decode of 2^8 .. 2^10 rows: the radix-2
        // form (2 rows per thread), unless RS16_DIAG_COL_RADIX4
        static const ColFn fns2[4][3] = {
            {col2_kernel<8, COL_ENC>, col2_kernel<8, COL_DEC_EVAL>, col2_kernel<8, COL_DEC_GEN>},
            {col2_kernel<9, COL_ENC>, col2_kernel<9, COL_DEC_EVAL>, col2_kernel<9, COL_DEC_GEN>},
            {col2_kernel<10, COL_ENC>, col2_kernel<10, COL_DEC_EVAL>, col2_kernel<10, COL_DEC_GEN>},
            {nullptr, nullptr, col2_kernel<11, COL_DEC_GEN>}};
        fn = fns2[L - 8][mode == COL_ENC ? 0 : (mode == COL_DEC_EVAL ? 1 : 2)];
        threads = (1u << L) / 2;
    }
    int bytes = lds[L - COL_LMIN];
    if (chunks) {
        static const int enc[3] = {ColSmem<8>::ELOG, ColSmem<9>::ELOG, ColSmem<10>::ELOG};
        static const int ifo[3] = {ColSmem<8>::B, ColSmem<9>::B, ColSmem<10>::B};
        bytes = (mode == COL_ENC_IFFT ? ifo : enc)[L - COL_LCHUNK];
    }
    if (bytes > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(fn, dim3(a.qrow * a.nstripes, rows), dim3(threads), bytes, s, a);
    return hipGetLastError();
}

}  // namespace rs16
