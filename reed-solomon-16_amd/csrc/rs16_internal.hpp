// rs16_internal.hpp -- shared declarations of the MI355X engine (not part of
// the public C ABI; see include/rs16.h for that).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "rs16_gf.hpp"

namespace rs16 {

struct HostTables {
    std::vector<uint16_t> exp, log, skew, log_walsh;
    std::vector<uint32_t> skew_entry;  // GF_ORDER entries: mul-table entry of each twiddle
    std::vector<uint32_t> mul_tab;     // TAB_ENTRIES * TAB_DWORDS
    std::vector<uint32_t> skew_tab;    // GF_ORDER * TAB_DWORDS: mul_tab row of skew_entry[i]
    // Column codec (rs16_col.hip): the 2^L - 1 twiddle tables (20 dwords
    // each, tile-group order) of a 2^L-row transform at skew delta d 2^L,
    // contiguous, for L = COL_LMIN .. COL_LGEN and d < col_img_count(L);
    // image (L, d) at col_img_offset(L, d) dwords.  (The images of one L
    // together are a permutation of the twiddle indices [0, 65535) when d
    // covers every chunk: the multi-chunk codecs of 2^8 .. 2^10 rows.)
    std::vector<uint32_t> col_img;
    // eval_poly of a high-rate decode with n = 2^(L+1) <= 2048 work rows as
    // an n-point XOR convolution (rs16_col.hip): col_v[col_v_offset(n) + k] =
    // n^-1 H_n(W)[k] mod 65535 with W = H_65536(log_walsh).
    std::vector<uint32_t> col_v;
    // the low rate's erasure vector is 1 from row n on (rate_low.rs:183-197):
    // rows [0, n) of the polynomial gain col_k[log2 n] = LogWalsh[0] -
    // sum_{j < n} W[j] mod 65535 (sum over all rows of W = 65536 LogWalsh[0])
    std::vector<uint32_t> col_k;
};
// DEC_MID of an L-bit general decode as a 2^hi x 2^hi matrix of mul-table
// entries (rs16_tables.cpp; the direct middle pass, rs16_engine::mid_matrix)
std::vector<uint32_t> mid_matrix_entries(const HostTables& t, int L);

constexpr uint32_t COL_LMIN = 6, COL_LMAX = 10;
// (and the general decoder's 2^11-row transform, skew delta 0 only)
constexpr uint32_t COL_LGEN = 11;
// L = 8 .. 10 (the radix-2 codec's multi-chunk encodes): every delta d 2^L
// (d < 2^(16 - L)); 6, 7: d = 0, 1; 11: d = 0
constexpr uint32_t COL_LCHUNK = 8;
constexpr uint32_t col_img_count(uint32_t L) {
    return L == COL_LGEN ? 1u : (L >= COL_LCHUNK ? (1u << (16 - L)) : 2u);
}
constexpr size_t col_img_offset(uint32_t L, uint32_t d) {
    size_t off = 0;
    for (uint32_t l = COL_LMIN; l < L; l++) off += (size_t)col_img_count(l) * ((1u << l) - 1) * 20;
    return off + (size_t)d * ((1u << L) - 1) * 20;
}
constexpr size_t COL_IMG_DWORDS = col_img_offset(COL_LGEN + 1, 0);
// n = 2^COL_LMIN .. 2^(COL_LMAX+1): tables of n entries at n - 2^COL_LMIN
constexpr size_t col_v_offset(uint32_t n) { return n - (1u << COL_LMIN); }
constexpr size_t COL_V_DWORDS = col_v_offset(4u << COL_LMAX);
const HostTables& host_tables();

// ---------------------------------------------------------------------------
// Pass kernels.  A "pass" applies a contiguous range of FFT/IFFT layers to
// tiles of 2^T rows (T <= 8) x Q quads (Q = 32 for T > 4, else 64; a quad is
// 8 bytes of a row, rs16_gf.hpp), one workgroup per (tile, slab of Q quads).
// Tile t covers
// rows  b_low + (k << lo) + (b_high << (lo+T)),  k in [0, 2^T),
// b_low = t mod 2^lo, b_high = t >> lo, i.e. lo = 0 gives contiguous tiles
// and lo > 0 gives strided tiles over bits [lo, lo+T) of the row index.
// ---------------------------------------------------------------------------
enum Prog : int {
    GEN_FFT = 0,   // plain load -> FFT layers -> plain store
    GEN_IFFT,      // plain load -> IFFT layers -> plain store
    ENC_FIRST,     // gather originals (rows >= a_count are zero) -> IFFT -> store
    ENC_MID,       // load -> IFFT (skew_ifft) -> FFT (skew_fft) -> store
    ENC_LAST,      // load -> FFT -> store rows < out_rows
    ENC_SINGLE,    // gather -> IFFT -> FFT -> store rows < out_rows
    DEC_FIRST,     // gather received rows * erasure logs -> IFFT -> store
    DEC_MID,       // load -> IFFT -> (I + in-tile formal derivative) -> FFT -> store
    DEC_LAST,      // u + L(z) -> FFT -> reveal lost originals -> store them
    DEC_SINGLE,    // gather*e -> IFFT -> formal derivative -> FFT -> reveal -> store
    // Half-transform decode (every original lost; see rs16_engine.cpp):
    DEC_HALF_LAST,    // load -> FFT -> reveal -> store lost originals
    DEC_HALF_SINGLE,  // gather*e -> IFFT -> FFT -> reveal -> store (one pass)
    NUM_PROGS
};
// Profiling ids (rs16_engine_set_profiling): the programs, then the passes
// of the half-transform decode that reuse DEC_FIRST / ENC_MID kernels, then
// the eval_poly kernels of a decode.
enum ProfId : int {
    PROF_DEC_HALF_FIRST = NUM_PROGS,
    PROF_DEC_HALF_MID,
    PROF_EVAL_POLY,
    PROF_COL_ENC,  // one-launch codec (rs16_col.hip): encode
    PROF_COL_DEC,  // one-launch codec: half-transform decode
    PROF_DEC_MID_DIRECT,  // the general decode's middle pass as a direct product (mid_direct_kernel)
    PROF_DEC_TILE_LAST,   // the general decode's last pass, one wave per quad column (tile_last_kernel)
    NUM_PROF
};

struct PassArgs {
    uint8_t* out;              // plain store base (row 0 of the transform)
    const uint8_t* in;         // plain load base (DEC_LAST: z)
    const uint8_t* in2;        // DEC_LAST: u
    const uint8_t* seg_a;      // gather source for rows [0, a_count)
    const uint8_t* seg_b;      // gather source for rows [chunk, chunk + b_count)
    const uint8_t* flags_a;    // received flags of segment A (nullptr: all present)
    const uint8_t* flags_b;    // received flags of segment B
    uint8_t* rest;             // restored-originals output (row 0 = original 0)
    const uint32_t* elog;      // erasure logs by row (eval_poly output)
    const uint32_t* skew_tab;   // v_perm table of every twiddle index: GF_ORDER x TAB_DWORDS
    const uint32_t* mul_tab;    // v_perm table of every log (TAB_ENTRIES x TAB_DWORDS)
    // Row strides (bytes) of in / in2, out, seg_a / seg_b and rest: equal to
    // the row width for work arrays, the caller's shard_bytes for its arrays
    // when the pass works on a column slice of them.
    uint64_t S_in, S_out, S_seg, S_rest;
    uint32_t qrow;             // quads per row of the slice = width / 8
    uint32_t nslab;            // ceil(qrow / Q), set by launch_pass
    // The launch covers ntiles tiles x nslab slabs = items, one workgroup
    // per item (set_item maps workgroups to items XCD-aware).  Set by launch_pass.
    uint32_t ntiles;
    uint32_t lo;               // tile bit offset
    uint32_t a_count, chunk, b_count;
    uint32_t skew_ifft, skew_fft;
    uint32_t out_rows;         // ENC_LAST / ENC_SINGLE
    uint32_t rest_seg_b;       // originals are segment B (high rate) or A (low rate)
    // Decode work row of pass row 0 on the gather side (received rows, their
    // erasure logs) and on the reveal side (lost originals, their logs):
    // 0 except in the half-transform decode.
    uint32_t row_base_in, row_base_out;
    uint32_t tile_base;        // first tile index of this launch
    // DEC_MID output pruning: only tile rows k in [need_lo, need_hi) are
    // consumed downstream; FFT groups and stores outside it are skipped.
    // need_hi == 0: no pruning.
    uint32_t need_lo, need_hi;
    // Set by launch_pass: every lane's byte offset within its wave's row
    // (row-set offset x stride + quad offset) fits in 32 bits, and no wave's
    // rows straddle the decoder's segment boundary, so HBM addresses are an
    // SGPR row base + a 32-bit lane offset (else 64-bit lane offsets).
    uint32_t voff32;
    uint32_t fd_lds;  // DEC_MID: in-tile formal derivative through LDS only (DIAG_FD_LDS)
    // Decode zero tiles: zflags[t] = 1 when DEC_FIRST tile t holds no received
    // row (then it is all zero after the erasure multiply and is neither
    // computed nor stored).  Written with rbits by the eval_poly kernels from
    // the received flags; read by DEC_FIRST (skip), DEC_MID (row r -> flag
    // r >> lo) and DEC_LAST; nullptr: no skipping.
    const uint8_t* zflags;
    // Received rows of the decode as a bitmap (bit r & 31 of word r >> 5), so
    // that a tile's flags are two scalar loads (rows of segments A and B).
    const uint32_t* rbits;
    // Branch-free loads: a row that is not read (absent / zero / out-of-slab
    // lanes) is read from `zero` (RS16_ZERO_BYTES of zeros, at offset
    // offL & 0x7FFF), so every load of an item is unconditional and the
    // compiler's vmcnt waits for the staged tables stay exact.
    const uint8_t* zero;
    // eval_poly with its last 256-point FWHT (row bits 0-7) left undone
    // (launch_eval_poly_from_flags, last_lo = false): DEC_FIRST / DEC_LAST at
    // T = 8 finish it for their tile's rows in LDS.  nullptr: use elog.
    const uint32_t* ework;
    // Lost originals' row range [lostrange[0], lostrange[1]) of a general
    // decode, written by the eval_poly kernels from the received flags
    // (nullptr: not pruned).  DEC_MID narrows [need_lo, need_hi) to the last
    // pass's tiles that hold a lost original; DEC_LAST workgroups of other
    // tiles return at once (their rows would only be stored if lost).
    const uint32_t* lostrange;
    // diagnostic timeline buffer (RS16_STAMPS builds; nullptr otherwise)
    uint64_t* stamps;
    // Independent stripes in one launch (rs16_encode_device_batch,
    // rs16_decode_device_batch): tiles [s * stripe_tiles, (s + 1) *
    // stripe_tiles) belong to stripe s, which reads / writes in, in2, out,
    // seg_a, seg_b and rest displaced by s times bs_in, bs_in2, bs_out,
    // bs_seg, bs_seg_b, bs_rest bytes; its twiddles and decode metadata are
    // those of tile (tile - s * stripe_tiles) (+ tile_base).  stripe_tiles ==
    // 0: one stripe.
    uint32_t stripe_tiles;
    uint64_t bs_in, bs_out, bs_seg, bs_in2, bs_seg_b, bs_rest;
    // Plain loads read row (r & in_rows_mask) of `in` (0: row r): the low-rate
    // encoder's FFTs of every recovery chunk read the one transformed chunk
    // of originals instead of copies of it.
    uint32_t in_rows_mask;
    // Batched stripes with losses of their own (rs16_decode_device_batch_varied):
    // stripe s also reads flags_a / flags_b displaced by s bs_fa / bs_fb
    // bytes and its own decode metadata -- elog / ework + s bs_elog words,
    // rbits + s bs_rbits words, zflags + s bs_zflags bytes, lostrange + s
    // bs_lost words (ErasureSpec's per-stripe outputs).  All 0: shared.
    uint64_t bs_fa, bs_fb;
    uint32_t bs_elog, bs_rbits, bs_zflags, bs_lost;
    // the engine's diagnostic switches (DiagFlags; host side: launch_pass)
    uint32_t diag;
    // ENC_FIRST / ENC_LAST as the passes of a decode with identity erasure
    // multipliers (rs16_engine::identity_logs): no eval_poly kernel read the
    // received flags, so these passes count them for rs16_decode_check.  Pass
    // row r (< 2^L of the half this launch covers) is decode work row r +
    // cnt_base with flag byte cnt_flags[r] (nullptr: received); the received
    // count of each 64-row chunk goes to rcount[2 (row >> 6) + cnt_seg] and 0
    // to the other segment's slot (ErasureSpec::rcount layout).  rcount
    // nullptr: not counted.
    uint32_t* rcount;
    const uint8_t* cnt_flags;
    uint32_t cnt_base, cnt_seg;
    // DEC_MID: mid_direct_kernel runs before it and produces U itself when
    // the consumed tile rows (from lostrange) are at most mid_direct; those
    // DEC_MID workgroups return at once (0: no direct kernel)
    uint32_t mid_direct;
    // DEC_LAST at 2^8-row tiles: when tl_max > 0 the lost originals' tiles
    // (lostrange) are the last pass of tile_last_kernel if they span at most
    // tl_max tiles, else of the 8-wave DEC_LAST items; each launch checks on
    // the device and returns at once when the other one covers the stripe
    // (0: DEC_LAST alone, no tile_last_kernel launch)
    uint32_t tl_max;
};

// One-launch codec for 2^9 / 2^10-row transforms (rs16_col.hip): one
// workgroup per quad column (x stripe) runs the whole encode or
// half-transform decode with the column resident in registers / LDS.
//   ENC: out[0, out_rows) = FFT_skew_fft(IFFT_skew_ifft(rows [0, in_rows) of in, zero above))
//   DEC: x[r] = received(r) ? in[r] * e[base_in + r] : 0 (received: r < in_rows
//        and flags[r], flags nullptr = all), out[r] = FFT(IFFT(x))[r] *
//        (65535 - e[base_out + r]) for r < out_rows; e = the erasure logs of
//        the 2^(L+1) work rows, whose last 256-point FWHT the kernel does
//        itself: elog = eval_poly's output without it (the engine's ework)
struct ColArgs {
    const uint8_t* img_ifft;    // the transforms' table images (HostTables::col_img)
    const uint8_t* img_fft;
    // decoder computing eval_poly itself (high rate, COL_DEC_EVAL): the
    // originals' received flags / count (segment B), HostTables::col_v of
    // n = 2^(L+1), and the per-64-row received counts (ErasureSpec::rcount)
    const uint8_t* flags_o;
    uint32_t o_rows;
    const uint32_t* vtab;
    uint32_t* rcount;
    uint32_t chunk;             // decoder: first row of segment B
    // erasure vector: rows [in_rows, chunk) = e_pad, rows from chunk + o_rows
    // on = e_tail, and e_k added to every log (low rate: e_pad 0, e_tail 1,
    // e_k = HostTables::col_k; high rate: 1, 0, 0)
    uint32_t e_pad, e_tail, e_k;
    uint32_t rev_a;             // COL_DEC_GEN: the originals are segment A (low rate), else B
    // COL_DEC_GEN: the received originals (segment B rows, stride S_in, stripe stride bs_in_b)
    const uint8_t* in_b;
    uint64_t bs_in_b;
    const uint8_t* in;
    const uint8_t* flags;
    uint8_t* out;
    const uint32_t* elog;
    const uint32_t* skew_tab;
    const uint32_t* mul_tab;
    const uint8_t* zero;
    uint64_t S_in, S_out;       // row strides of in / out
    uint32_t qrow;              // quad columns per row (width / 8)
    uint32_t nstripes;          // stripes (in / out displaced by bs_in / bs_out bytes each)
    uint32_t in_rows, out_rows;
    uint32_t skew_ifft, skew_fft;
    uint32_t base_in, base_out;
    uint64_t bs_in, bs_out;
    // stripes with losses of their own: flags / flags_o + st bs_flags /
    // bs_flags_o bytes, elog + st bs_elog words (0: shared by all stripes)
    uint64_t bs_flags, bs_flags_o;
    uint32_t bs_elog;
    uint32_t nch;               // launch_col_multi: chunks of 128 rows (one wave each); launch_col: chunks (ColMode)
    uint64_t* stamps;           // RS16_STAMPS builds: phase timeline (rs16_engine_set_stamps)
    uint32_t diag;              // the engine's diagnostic switches (DiagFlags; host side: launch_col)
};
int col_rows_ok(uint32_t L);  // L = log2(rows of the transform) the codec covers
// COL_DEC_GEN: the general high-rate decode of a 2^L-row work buffer (any
// loss pattern; formal derivative in the kernel), polynomial in the kernel
//   COL_ENC_IFFT / COL_ENC_FFTX (2^8 .. 2^10 rows): the high rate's
//   multi-chunk encode in two launches -- the IFFT of every chunk of
//   originals (grid row = chunk, skew_ifft = 2^L: chunk c at delta (c + 1)
//   2^L) stored whole, then the FFT (skew 0) of the XOR of nch chunks
// ColArgs::nch > 1 with COL_ENC / COL_ENC_IFFT: one grid row per chunk (COL_ENC:
// the low rate's recovery chunks, FFT of chunk c at delta (c + 1) 2^L)
enum ColMode : int { COL_ENC = 0, COL_DEC_EWORK, COL_DEC_EVAL, COL_DEC_GEN, COL_ENC_IFFT, COL_ENC_FFTX };
// the radix-2 multi-chunk encodes take at most this many chunks (more: passes)
constexpr uint32_t COL_MAX_CHUNKS = 64;
hipError_t launch_col(const ColArgs& a, uint32_t L, int mode, hipStream_t s);
// Multi-chunk encodes of 128-row chunks in one launch (colm_kernel): high
// rate (high = 1: nch chunks of originals, one recovery chunk) or low rate
// (one chunk of originals, nch recovery chunks); nch <= COLM_MAX_CHUNKS
constexpr uint32_t COLM_L = 7, COLM_MAX_CHUNKS = 16;
hipError_t launch_col_multi(const ColArgs& a, bool high, hipStream_t s);

// Per-engine diagnostic switches (rs16_engine_set_diagnostics, include/rs16.h):
// alternative code paths kept for tests and measurements, never needed for
// correct results.  0 = the shipped behaviour.  They travel with the launch
// arguments (PassArgs / ColArgs / ErasureSpec::diag); there is no process-wide
// state.
enum DiagFlags : int {
    DIAG_FORCE_VOFF64 = 1,    // 64-bit lane offsets in every pass (PassArgs::voff32 = 0)
    DIAG_EVAL_TWO_KERNEL = 2, // eval_poly: two-kernel form even when the one-kernel form applies
    DIAG_EVAL_FULL = 4,       // eval_poly: the full 65536-point form even for n <= 2048
    DIAG_NO_COLUMN = 8,       // 2^9 / 2^10-row transforms through the pass codec (rs16_col.hip off)
    DIAG_FORCE_COLUMN = 16,   // ... through the column codec at any width (rs16_engine::col_max_quads, col_max_chunk_rows ignored)
    DIAG_TILE_LAST = 32,      // the general decode's T = 8 last pass as tile_last_kernel at any loss count
    DIAG_NO_TILE_LAST = 64,   // ... always as the 8-wave pass (DEC_LAST items)
    DIAG_FD_LDS = 128,        // DEC_MID's in-tile formal derivative always through the LDS image (tile_fd)
    DIAG_COL_RADIX4 = 256,    // column codec: the 4-rows-per-thread form for every transform (col_kernel)
    DIAG_NO_IDENTITY = 512,   // whole-half erasures: eval_poly and the per-row multipliers anyway (identity_logs)
    DIAG_NO_MID_DIRECT = 1024, // the general decode's middle pass always as DEC_MID (no mid_direct_kernel)
};

constexpr size_t RS16_ZERO_BYTES = 65536;

// Launch `num_tiles` tiles (x nslab slabs) of program P with tile bits T.
hipError_t launch_pass(int prog, int T, const PassArgs& a, uint32_t num_tiles, hipStream_t s);
// DEC_LAST at T = 8 as one wave per quad column of a tile (rs16_pass.hip
// tile_last_kernel): `num_tiles` tiles (x stripes, PassArgs::stripe_tiles)
// from a.tile_base, rows at lo = 0.
hipError_t launch_tile_last(const PassArgs& a, uint32_t num_tiles, hipStream_t s);
// The general decode's middle pass as a direct product (rs16_pass.hip
// mid_direct_kernel): U rows [need_lo, need_hi) of every tile column j from
// the live Z rows and mtab (rs16_engine::mid_tables: 2^hi x 2^hi v_perm
// tables of mid_matrix_entries, 80 bytes each, row-major), for `ns`
// stripes; a stripe whose consumed rows exceed MID_DIRECT_MAX does nothing
// (DEC_MID computes it).
constexpr uint32_t MID_DIRECT_MAX = 4;
// tile_last_kernel is the general decode's last pass when the lost originals
// span at most this many 256-row tiles (scripts/probe_general.py: 16 tiles
// 18.6 against 24.0 us for the 8-wave items, 32 tiles 28.3 against 24.7)
constexpr uint32_t TILE_LAST_MAX = 16;
hipError_t launch_mid_direct(const PassArgs& a, const uint32_t* mtab, uint32_t hi, uint32_t ns, hipStream_t s);

// Elementwise / small kernels.
hipError_t launch_mul(uint8_t* x, size_t bytes, uint32_t entry, const uint32_t* mul_tab, hipStream_t s);
hipError_t launch_xor(uint8_t* x, const uint8_t* y, size_t bytes, hipStream_t s);
// w[0, chunk_bytes) ^= the nch - 1 chunks behind it / chunk 0 copied into them
hipError_t launch_xor_chunks(uint8_t* w, size_t chunk_bytes, uint32_t nch, hipStream_t s);
hipError_t launch_copy_chunks(uint8_t* w, size_t chunk_bytes, uint32_t nch, hipStream_t s);
hipError_t launch_formal_derivative(uint8_t* out, const uint8_t* in, size_t shard_count, size_t S, hipStream_t s);

// FWHT / eval_poly.  `work` is a u32[65536] scratch.
struct ErasureSpec {           // builds the erasure vector of rate_{high,low}.rs decode
    const uint8_t* flags_a;    // received flags of segment A
    const uint8_t* flags_b;    // received flags of segment B
    uint32_t a_count, chunk, b_count;
    uint32_t pad_fill;         // value of rows [a_count, chunk)   (1 for high rate)
    uint32_t tail_fill;        // value of rows >= chunk + b_count (1 for low rate)
    // Decode pass metadata written by the same kernels (nullptr: none):
    // rbits = received-row bitmap of rows [0, n); zflags[t] = 1 when rows
    // [t << zlo, (t + 1) << zlo) hold no received row (t < n >> zlo <= 256).
    uint32_t* rbits;
    uint8_t* zflags;
    uint32_t n, zlo;
    // Lost-original rows (rows of the originals' segment -- B when orig_b,
    // else A -- without a received flag): lostpart[2 b], lostpart[2 b + 1] =
    // the first / one past the last lost row of block b (~0u / 0 if none),
    // reduced to lostrange[0..1] = [first lost row, last lost row + 1)
    // ({~0u, 0} if none).  nullptr: not computed.
    uint32_t* lostpart;
    uint32_t* lostrange;
    uint32_t orig_b;
    // Received rows per 64-row chunk of rows [0, n), by segment:
    // rcount[2 c] = rows of segment A, rcount[2 c + 1] = rows of segment B
    // (rs16_decode_check compares their sums with the caller's counts).
    uint32_t* rcount;
    uint64_t* stamps;          // RS16_STAMPS builds: eval timeline (rs16_engine_set_stamps)
    // Stripes with losses of their own (rs16_decode_device_batch_varied):
    // nstripes > 1 evaluates stripe y in grid row y, with its flags at
    // flags_a / flags_b + y bs_fa / bs_fb bytes and its outputs displaced by
    // y times bs_work (work / out words), bs_elog (last_lo output words),
    // bs_rbits (words), bs_zflags (bytes), bs_lost (lostpart / lostrange
    // words).  rcount must be nullptr then.  0 / 1: one stripe.
    uint32_t nstripes;
    uint64_t bs_fa, bs_fb;
    uint32_t bs_work, bs_elog, bs_rbits, bs_zflags, bs_lost;
    uint32_t diag;             // the engine's diagnostic switches (DiagFlags; host side)
};
hipError_t launch_eval_poly_from_flags(const ErasureSpec& e, uint32_t* work, uint32_t* out_elog,
                                       const uint16_t* log_walsh, hipStream_t s, bool last_lo);
// high-rate decodes with n <= 2048 rows (tail_fill == 0): 2 kernels, rows [0, n) of out_elog
hipError_t launch_eval_poly_small(const ErasureSpec& e, uint32_t n, uint32_t* work, uint32_t* out_elog,
                                  const uint16_t* log_walsh, hipStream_t s, bool last_lo);
hipError_t launch_eval_poly_u16(uint16_t* data, uint32_t* work, const uint16_t* log_walsh, hipStream_t s);
hipError_t launch_fwht_u16(uint16_t* data, uint32_t* work, hipStream_t s);

}  // namespace rs16
