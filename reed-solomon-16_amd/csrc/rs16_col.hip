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
// latency-bound kernels of 128-256 one-wave workgroups.  Here
// every quad column (8 bytes of each row: 4 elements, an independent set of
// codewords, src/algorithm.md:18-32) is one workgroup that keeps the whole
// column -- 2^L rows x 8 bytes, 8 KiB at L = 10 -- resident for all 2L layers:
//
//   * 2^L / 4 threads (4 waves at L = 10, one per SIMD), 4 rows per thread.
//     Layers go in radix-4 blocks over two row bits (b0, b1): the thread's
//     4 rows are its index with b0 / b1 inserted, so both layers of a block
//     are in registers; between blocks the rows move through an 8 KiB LDS
//     image (one barrier per block: every thread writes back exactly the
//     rows it read).  The image is XOR-swizzled (row bits 5, 6 into bits
//     0-4) so that every block's b64 accesses are bank-conflict free.
//   * The 2 (2^L - 1) twiddle tables of the codec (80-byte v_perm tables,
//     rs16_gf.hpp) are staged once into LDS: both directions except the FFT's
//     last layer (2^(L-1) tables), which is written over the IFFT's first
//     layer once that block is done -- 128 KiB at L = 10.
//   * The IFFT's last block and the FFT's first share their row bits: no
//     exchange between the two directions.
//   * Rows are loaded straight into the first block's layout and stored from
//     the last one's (rows 4t .. 4t + 3); a workgroup reads all of its rows
//     before it writes any, so in / out may alias (the work-buffer API).
//   * Workgroups are dealt to XCDs so that the 16 quad columns of a 128-byte
//     line run on one XCD (one HBM fetch per line and XCD).
#include "rs16_internal.hpp"
#include "rs16_fwht.hpp"

namespace rs16 {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// LDS index of row r in the image (uint2 units): bits 5 and 6 are XORed
// into bits 0-4 so that the 32 lanes of a b64 access hit 32 distinct bank
// pairs for every block's row pattern (block bits (0,1): lane bits -> row
// bits 2-6; (2,3): 0,1,4,5,6; (4,5): 0-3,6; (6,7), (8,9): 0-4).
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

// LDS layout (bytes): [image 2^L x 8][A: (2^L - 1) x 80][B: (2^(L-1) - 1) x 80]
// A holds the IFFT's tables in tile-group order (layer kb at 2^L - 2^(L-kb),
// group j = row >> (kb + 1)), later the FFT's layer-0 tables in [0, 2^(L-1));
// B holds the FFT's layers 1.. (tile group t at t - 2^(L-1)).
template <int L> struct ColSmem {
    static constexpr int N = 1 << L;
    static constexpr int IMG = N * 8;
    static constexpr int A = IMG;
    static constexpr int B = A + (N - 1) * 80;
    static constexpr int TABS_END = B + (N / 2 - 1) * 80;
    // decoder: the erasure logs of the 2^(L+1) work rows (eval_poly's last H_lo, done here)
    static constexpr int ELOG = TABS_END;
    static constexpr int bytes(bool dec) { return TABS_END + (dec ? 2 * N * 4 : 0); }
};

// Twiddle (skew index) of tile group t of a 2^L-row transform at skew delta.
template <int L> __device__ __forceinline__ uint32_t group_skew(uint32_t t, uint32_t delta) {
    const int kb = L - 32 + __clz((uint32_t)((1 << L) - 1) - t);
    const uint32_t j = t - ((1u << L) - (1u << (L - kb)));
    return (j << (kb + 1)) + (1u << kb) + delta - 1u;
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

// LDS byte offset of the table of layer kb for row r, direction FFT or not.
template <int L, bool FFT> __device__ __forceinline__ uint32_t tab_off(int kb, uint32_t r) {
    constexpr int N = 1 << L;
    const uint32_t t = (uint32_t)(N - (N >> kb)) + (r >> (kb + 1));
    if (!FFT || kb == 0) return ColSmem<L>::A + t * 80u;
    return ColSmem<L>::B + (t - N / 2) * 80u;
}

// The twiddle tables of one block: the layers on row bits B0 (if D0) and B1
// (if D1) of the thread's 4 rows (register m <-> bit B0 = m & 1, bit B1 =
// m >> 1).  Read from LDS one block ahead of their use.
struct BlockTabs {
    uint32_t w0[20], w2[20], w1[20];  // layer B0: pairs (0,1), (2,3); layer B1: pairs (0,2), (1,3)
};
template <int L, bool FFT, int B0, int B1, bool D0, bool D1>
__device__ __forceinline__ void load_tabs(BlockTabs& w, uint32_t t, const uint8_t* smem) {
    const uint32_t r0 = brow<B0, B1>(t, 0), r2 = brow<B0, B1>(t, 2);
    if (D0) {
        lds_table(w.w0, smem, tab_off<L, FFT>(B0, r0));
        lds_table(w.w2, smem, tab_off<L, FFT>(B0, r2));
    }
    if (D1) lds_table(w.w1, smem, tab_off<L, FFT>(B1, r0));
}
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

// Diagnostic timeline (-DRS16_STAMPS=1 builds only, scripts/stamps.py):
// thread 0 stores s_memtime at phase i to stamps[block * 16 + i] (14 / 15:
// s_memrealtime at start / end, 12 / 13: HW_ID / XCC_ID).
#ifndef RS16_STAMPS
#define RS16_STAMPS 0
#endif
__device__ __forceinline__ void cstamp(const ColArgs& a, int i) {
#if RS16_STAMPS
    if (a.stamps && threadIdx.x == 0) {
        uint64_t* p = a.stamps + blockIdx.x * 16;
        p[i] = __builtin_amdgcn_s_memtime();
        if (i == 0) {
            p[14] = __builtin_amdgcn_s_memrealtime();
            p[12] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            p[13] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        }
        if (i == 11) p[15] = __builtin_amdgcn_s_memrealtime();
    }
#else
    (void)a;
    (void)i;
#endif
}

template <int L, bool DEC>
__global__ __launch_bounds__((1 << L) / 4) void col_kernel(ColArgs a) {
    constexpr int N = 1 << L, NT = N / 4;
    constexpr int NTAB = N - 1;               // twiddle tables per direction
    constexpr int CPL = (5 * NTAB + NT - 1) / NT;  // 16-byte table chunks per thread per direction (20)
    constexpr int LATE = 5 * (N / 2) / NT;    // the FFT's layer-0 chunks: i < LATE (10)
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t t = threadIdx.x;
    cstamp(a, 0);

    // workgroup -> (stripe, quad column), XCD-aware: consecutive columns on
    // one XCD (workgroups are dealt to the 8 XCDs round-robin)
    const uint32_t total = a.qrow * a.nstripes;
    uint32_t g = blockIdx.x;
    if ((total & 7u) == 0) g = (g & 7u) * (total >> 3) + (g >> 3);
    const uint32_t st = g / a.qrow, q = g - st * a.qrow;
    const uint32_t offL = (q >> 3) * 64u + (q & 7u) * 4u;
    const uint8_t* in = a.in + st * a.bs_in + offL;
    uint8_t* out = a.out + st * a.bs_out + offL;

    // ---- requests: rows, the decoder's erasure data, then the twiddle tables
    uint32_t XL[4], XH[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const uint32_t r = 4 * t + m;
        // (a row that is not read comes from the zero page, RS16_ZERO_BYTES;
        // the decoder zeroes rows that were not received with its multiply)
        const uint32_t* p = (const uint32_t*)(r < a.in_rows ? in + (size_t)r * a.S_in : a.zero + (offL & 0x7FFFu));
        XL[m] = p[0];
        XH[m] = p[8];
    }
    // decoder: eval_poly's output before its last 256-point FWHT (a.elog =
    // the engine's ework): wave w finishes the blocks of rows [512 w, 512 w + 512)
    uint32_t zv[2][4];
    bool rcv[4] = {true, true, true, true};
    if constexpr (DEC) {
        const uint32_t w = t >> 6, lane = t & 63;
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int j = 0; j < 4; j++) zv[b][j] = a.elog[(2 * w + b) * 256 + lane + 64 * j];
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint32_t r = 4 * t + m;
            rcv[m] = r < a.in_rows && (!a.flags || a.flags[r] != 0);
        }
    }
    u32x4 s1[CPL], s2[CPL];
    const u32x4* skew_tab = (const u32x4*)a.skew_tab;
#pragma unroll
    for (int i = 0; i < CPL; i++) {
        const uint32_t c = t + (uint32_t)i * NT;
        if (c < 5 * NTAB) s1[i] = skew_tab[(size_t)group_skew<L>(c / 5, a.skew_ifft) * (TAB_DWORDS / 4) + c % 5];
    }
    uint32_t gt[DEC ? 4 : 1][20];
    uint32_t ev[4] = {0, 0, 0, 0};
    if constexpr (DEC) {
        // the last H_lo of eval_poly (src/engine.rs:207-218) for the work
        // rows this codec reads: erasure logs of rows [0, 2^(L+1)) in LDS
        uint32_t* elds = (uint32_t*)(smem + ColSmem<L>::ELOG);
        const uint32_t w = t >> 6, lane = t & 63;
#pragma unroll
        for (int b = 0; b < 2; b++) {
            fwht256_wave(zv[b]);
#pragma unroll
            for (int j = 0; j < 4; j++) elds[(2 * w + b) * 256 + lane + 64 * j] = zv[b][j];
        }
        __syncthreads();
        // gather multipliers: the v_perm table of each received row's log
        // (MULTIPLY SHARDS, rate_high.rs:203-228: other rows times zero)
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint32_t r = 4 * t + m;
            glb_table(gt[m], a.mul_tab, rcv[m] ? elds[a.base_in + r] : ZERO_ENTRY);
            ev[m] = elds[a.base_out + r];
        }
    }
#pragma unroll
    for (int i = 0; i < CPL; i++) {
        const uint32_t c = t + (uint32_t)i * NT;
        if (c < 5 * NTAB) s2[i] = skew_tab[(size_t)group_skew<L>(c / 5, a.skew_fft) * (TAB_DWORDS / 4) + c % 5];
    }

    cstamp(a, 1);
    // ---- stage the IFFT's tables into A (the FFT's after the first block)
#pragma unroll
    for (int i = 0; i < CPL; i++) {
        const uint32_t c = t + (uint32_t)i * NT;
        if (c < 5 * NTAB) *(u32x4*)(smem + ColSmem<L>::A + (c / 5) * 80 + (c % 5) * 16) = s1[i];
    }
    if constexpr (DEC) {
#pragma unroll
        for (int m = 0; m < 4; m++) {
            uint32_t zl = 0, zh = 0;
            mul_xor(zl, zh, XL[m], XH[m], gt[m]);
            XL[m] = zl;
            XH[m] = zh;
        }
    }
    __syncthreads();
    cstamp(a, 2);
    // FFT tables, written between the barriers of the first exchange: layer 0
    // over the IFFT's layer 0 (dead by then), layers >= 1 into B
    auto stage_fft = [&]() {
#pragma unroll
        for (int i = 0; i < CPL; i++) {
            const uint32_t c = t + (uint32_t)i * NT;
            if (i < LATE) *(u32x4*)(smem + ColSmem<L>::A + (c / 5) * 80 + (c % 5) * 16) = s2[i];
            else if (c < 5 * NTAB) *(u32x4*)(smem + ColSmem<L>::B + (c / 5 - N / 2) * 80 + (c % 5) * 16) = s2[i];
        }
    };

    // ---- IFFT (layers 0 .. L-1) then FFT (L-1 .. 0) in radix-4 blocks; the
    // next block's tables are read before each exchange's barrier
    BlockTabs ta, tb;
    load_tabs<L, false, 0, 1, true, true>(ta, t, smem);
    compute<false, true, true>(XL, XH, ta);
    cstamp(a, 3);
    load_tabs<L, false, 2, 3, true, true>(tb, t, smem);
    exchange<0, 1, 2, 3>(XL, XH, t, smem, stage_fft);
    compute<false, true, true>(XL, XH, tb);
    load_tabs<L, false, 4, 5, true, true>(ta, t, smem);
    exchange<2, 3, 4, 5>(XL, XH, t, smem);
    compute<false, true, true>(XL, XH, ta);
    cstamp(a, 4);
    load_tabs<L, false, 6, 7, true, true>(tb, t, smem);
    exchange<4, 5, 6, 7>(XL, XH, t, smem);
    compute<false, true, true>(XL, XH, tb);
    if constexpr (L == 10) {
        load_tabs<L, false, 8, 9, true, true>(ta, t, smem);
        exchange<6, 7, 8, 9>(XL, XH, t, smem);
        compute<false, true, true>(XL, XH, ta);
        cstamp(a, 5);
        // the FFT's first block keeps the row bits: no exchange
        load_tabs<L, true, 8, 9, true, true>(tb, t, smem);
        compute<true, true, true>(XL, XH, tb);
        load_tabs<L, true, 6, 7, true, true>(ta, t, smem);
        exchange<8, 9, 6, 7>(XL, XH, t, smem);
    } else {
        static_assert(L == 9, "the column codec covers 2^9 and 2^10 rows");
        load_tabs<L, false, 7, 8, false, true>(ta, t, smem);
        exchange<6, 7, 7, 8>(XL, XH, t, smem);
        compute<false, false, true>(XL, XH, ta);
        cstamp(a, 5);
        load_tabs<L, true, 7, 8, false, true>(tb, t, smem);
        compute<true, false, true>(XL, XH, tb);
        load_tabs<L, true, 6, 7, true, true>(ta, t, smem);
        exchange<7, 8, 6, 7>(XL, XH, t, smem);
    }
    cstamp(a, 6);
    compute<true, true, true>(XL, XH, ta);
    load_tabs<L, true, 4, 5, true, true>(tb, t, smem);
    exchange<6, 7, 4, 5>(XL, XH, t, smem);
    compute<true, true, true>(XL, XH, tb);
    cstamp(a, 7);
    load_tabs<L, true, 2, 3, true, true>(ta, t, smem);
    exchange<4, 5, 2, 3>(XL, XH, t, smem);
    compute<true, true, true>(XL, XH, ta);
    load_tabs<L, true, 0, 1, true, true>(tb, t, smem);
    exchange<2, 3, 0, 1>(XL, XH, t, smem);
    cstamp(a, 8);
    uint32_t rt[DEC ? 4 : 1][20];
    if constexpr (DEC) {
        // reveal multipliers (requested here so the tables are in flight
        // under the last block)
#pragma unroll
        for (int m = 0; m < 4; m++) glb_table(rt[m], a.mul_tab, GF_MODULUS - ev[m]);
    }
    compute<true, true, true>(XL, XH, tb);
    cstamp(a, 9);

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
        if (r < a.out_rows) {
            uint32_t* p = (uint32_t*)(out + (size_t)r * a.S_out);
            __builtin_nontemporal_store(vl, p);
            __builtin_nontemporal_store(vh, p + 8);
        }
    }
    cstamp(a, 10);
#if RS16_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
    cstamp(a, 11);
#endif
}

}  // namespace

int col_rows_ok(uint32_t L) { return L == 9 || L == 10; }

hipError_t launch_col(const ColArgs& a, uint32_t L, bool dec, hipStream_t s) {
    if (!col_rows_ok(L)) return hipErrorInvalidValue;
    if (a.qrow == 0 || a.nstripes == 0 || a.out_rows == 0) return hipSuccess;
    const void* fn;
    int lds;
    if (L == 10) {
        fn = dec ? (const void*)col_kernel<10, true> : (const void*)col_kernel<10, false>;
        lds = ColSmem<10>::bytes(dec);
    } else {
        fn = dec ? (const void*)col_kernel<9, true> : (const void*)col_kernel<9, false>;
        lds = ColSmem<9>::bytes(dec);
    }
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
    }
    dim3 grid(a.qrow * a.nstripes), block((1u << L) / 4);
    if (L == 10) {
        if (dec) hipLaunchKernelGGL((col_kernel<10, true>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((col_kernel<10, false>), grid, block, lds, s, a);
    } else {
        if (dec) hipLaunchKernelGGL((col_kernel<9, true>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((col_kernel<9, false>), grid, block, lds, s, a);
    }
    return hipGetLastError();
}

}  // namespace rs16
