// rs16_engine.hpp -- host-side engine object and pass drivers (internal).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "../../include/rs16.h"
#include "rs16_internal.hpp"

namespace rs16 {

// Grow-only device buffer.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t bytes);
    void release();
};
// Grow-only page-locked host buffer (hipHostMalloc): DMA-rate H2D / D2H.
struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t bytes);
    void release();
};
// An event recorded on a stream and not yet waited for on the host.
struct Pending {
    hipEvent_t ev = nullptr;
    bool busy = false;
    hipError_t record(hipStream_t s);
    hipError_t wait();  // host-side: returns once the recorded work is done
    void release();
};

// Status helper: every internal call returns an rs16 code and fills err.
int set_error(rs16_error* err, int code, uint64_t v0 = 0, uint64_t v1 = 0, uint64_t v2 = 0);
int hip_fail(rs16_error* err, hipError_t e);
#define RS16_HIP(call)                                 \
    do {                                               \
        hipError_t _e = (call);                        \
        if (_e != hipSuccess) return hip_fail(err, _e); \
    } while (0)
#define RS16_PASS(...)                                       \
    do {                                                     \
        if (int _rc = this->pass(__VA_ARGS__, err)) return _rc; \
    } while (0)
// the same under profiling id PROF
#define RS16_PASS_AS(PROF, ...)                                     \
    do {                                                            \
        if (int _rc = this->pass(__VA_ARGS__, err, PROF)) return _rc; \
    } while (0)

size_t next_pow2(size_t x);
inline int ilog2(size_t x) { int l = 0; while (((size_t)1 << l) < x) l++; return l; }

// Geometry of a decode (both rates): segment A = rows [0, a_count),
// segment B = rows [chunk, chunk + b_count), transform of n rows.
struct DecodeGeom {
    bool high;
    uint32_t a_count, chunk, b_count, n;
    // Received shard counts of the two segments when the caller knows them
    // (0: the whole segment is lost, so its first-pass tiles need no launch).
    size_t a_recv = 1, b_recv = 1;
};
DecodeGeom decode_geom(bool high, size_t k, size_t m);

}  // namespace rs16

struct rs16_encoder;
struct rs16_decoder;

struct rs16_engine {
    int device = 0;
    int flags = 0;  // rs16_engine_new_ex flags (RS16_ENGINE_OWN_QUEUE)
    hipStream_t stream = nullptr;
    // diagnostic switches of this engine (rs16::DiagFlags, rs16_engine_set_diagnostics)
    int diag = 0;
    uint32_t* d_skew_tab = nullptr;  // v_perm table per twiddle index (8 MiB)
    uint32_t* d_mul_tab = nullptr;
    uint32_t* d_col_img = nullptr;   // column codec table images (HostTables::col_img)
    uint32_t* d_col_v = nullptr;     // column codec eval_poly tables (HostTables::col_v)
    uint16_t* d_log_walsh = nullptr;
    uint8_t* d_zero_sink = nullptr;  // zero page (PassArgs::zero, ColArgs::zero)
    // scratch
    rs16::DevBuf ws_z, ws_u, ws_fd, ws_flags;
    // the general decode's middle pass as v_perm tables of its matrix, per
    // transform size L (mid_tables; built on first use)
    rs16::DevBuf mid_tab[17];
    // The decode's eval_poly outputs / pass metadata (written by decode_eval,
    // read by decode_passes).  `evset` points at the set the next decode uses:
    // ev_main, or one of the pipelined host path's per-lane sets (so that
    // two lanes' decodes never share them).
    struct EvalBufs {
        rs16::DevBuf work32, elog;
        rs16::DevBuf zflag;   // per DEC_FIRST tile, 1 = no received row (tile skipped, rows zero)
        rs16::DevBuf rbits;   // received-row bitmap (65536 bits)
        rs16::DevBuf lost;    // lost-original row range per 256-row block (2 KiB) + overall (8 B)
        rs16::DevBuf rcount;  // received rows per 64-row chunk and segment (ErasureSpec::rcount)
        void release() { work32.release(), elog.release(), zflag.release(), rbits.release(), lost.release(), rcount.release(); }
    };
    EvalBufs ev_main, ev_lane[2];
    EvalBufs* evset = &ev_main;
    // Split decode (rs16_decode_prepare / rs16_decode_device_prepared): the
    // prepared received pattern, whose eval_poly went to ev_main on the
    // prepare's stream; prep_ev marks its end.  While prep_pending, any other
    // use of ev_main first orders itself after prep_ev (guard_eval).
    struct Prepared {
        bool valid = false, nothing = false;
        size_t k = 0, m = 0, S = 0;
        rs16::DecodeGeom g{};
        const uint8_t* fl_a = nullptr;
        const uint8_t* fl_b = nullptr;
        int nslices = 1;
    } prep;
    hipEvent_t prep_ev = nullptr;
    bool prep_pending = false;
    bool preparing = false;
    // order stream s after a pending preparation's eval_poly (whose outputs
    // the caller is about to overwrite or read) and drop the preparation
    // unless it is the one being consumed
    int guard_eval(hipStream_t s, bool consume, rs16_error* err);
    // the last decode's geometry and the received counts it was given (rs16_decode_check)
    rs16::DecodeGeom last_dec{};
    bool last_dec_valid = false;
    // ... or, when that decode had nothing to restore (every original
    // received: no kernel counted anything), a copy of its flags in ws_flags
    // (segment A at 0, B at GF_ORDER), which rs16_decode_check counts itself
    bool last_dec_flags_only = false;
    void forget_decode() { last_dec_valid = last_dec_flags_only = false; }
    // Host-resident pipeline (rs16_encode_host / rs16_decode_host): column
    // slices alternate between two slots, each with its own stream and the
    // device buffers of one slice, so copies and compute of different slices
    // overlap.  hflags: the received flags of a host decode; hev orders the
    // slots after the engine stream.
    struct HostSlot {
        hipStream_t s = nullptr;
        rs16::DevBuf orig, rec, z, u;
        rs16::DevBuf rcount;  // the slot's column decodes' received counts (never ws_rcount)
    };
    HostSlot hslot[2];
    // Column slices of the device-resident one-shot codec: a stripe's shard
    // columns are split into `slices` slices (multiples of 64 bytes; every
    // 64-byte column block is an independent codeword) that run on internal
    // streams forked from and joined back into the caller's stream.  Default
    // 1: measured on MI355X (scripts/probe_fork.py), the fork/join events
    // cost ~8 us of host time each and the cross-queue dependencies erase the
    // overlap (32768:32768 x 1 KiB encode 97 us at 1 slice, 101 us at 2);
    // only fully independent streams (two stripes) gain (+10 %).
    static constexpr int MAX_SLICES = 4;
    int slices = 1;
    hipStream_t sl_stream[MAX_SLICES] = {};  // per call: [0] = caller's stream, [j] = sl_own[j]
    hipStream_t sl_own[MAX_SLICES] = {};
    hipEvent_t sl_fork = nullptr, sl_join[MAX_SLICES] = {};
    int slice_count(size_t S) const;
    int fork(hipStream_t s, int n, rs16_error* err);
    int join(hipStream_t s, int n, rs16_error* err);
    rs16::DevBuf hflags;
    hipEvent_t hev = nullptr;
    // pipelined host stripes (rs16_{en,de}code_host_batch): per lane, the
    // flag bytes' copy out of hp_flags is done
    hipEvent_t hp_ev[2] = {};
    hipEvent_t hp_off = nullptr;  // the first stripe's H2D is done: the other lane's first H2D starts then
    rs16::HostBuf hp_flags;  // page-locked staging of the decode's flag bytes (2 x (k + m))
    int host_pipe_events(rs16_error* err);
    int host_slots(rs16_error* err);

    hipStream_t pick(void* s) const { return s ? (hipStream_t)s : stream; }
    int activate(rs16_error* err);

    // The scratch buffers (ws_*) belong to the engine, not to a stream: a
    // call that uses them on stream s first waits for the engine's previous
    // such call when that ran on another stream, so calls on different
    // streams cannot overwrite each other's scratch.  order(s) at the start
    // of such a call, scratch_done(s) at its end.  A call on a caller's
    // stream records order_ev there before it returns (the stream is never
    // touched again: the caller may destroy it); a call on the engine's own
    // stream records nothing unless a later call on another stream needs it
    // (then it is recorded on the engine stream, which the engine owns), so
    // the one-stream case costs no event.
    enum { LAST_NONE, LAST_ENGINE, LAST_CALLER } last = LAST_NONE;
    hipEvent_t order_ev = nullptr;
    int order(hipStream_t s, rs16_error* err);
    int scratch_done(hipStream_t s, rs16_error* err);

    // Encoders / decoders created on this engine.  rs16_engine_free releases
    // their device work space and detaches them (eng = nullptr): a detached
    // object answers every call with RS16_INVALID_ARGUMENT and
    // rs16_{en,de}coder_free only frees its host memory.
    std::vector<rs16_encoder*> encoders;
    std::vector<rs16_decoder*> decoders;

    // Pass launch (with optional hipEvent timing on the launch stream under
    // profiling id `prof` (rs16::ProfId; -1 = the program's own id).
    int pass(int prog, int T, const rs16::PassArgs& a, uint32_t tiles, hipStream_t s, rs16_error* err,
             int prof = -1);
    int prof_begin(hipStream_t s, hipEvent_t* ev, rs16_error* err);
    int prof_end(int id, hipStream_t s, hipEvent_t ev, rs16_error* err);
    bool profiling = false;
    // diagnostic timelines (rs16_engine_set_stamps): passes under profiling
    // id stamp_prof get stamp_buf (RS16_STAMPS builds record into it)
    void* stamp_buf = nullptr;
    int stamp_prof = -1;
    bool elog_fused = false;  // last decode_eval left the final 256-point FWHT to the passes (ws_work32)
    bool eval_in_col = false; // last decode_eval left eval_poly to the column codec (COL_DEC_EVAL)
    bool e_ident = false;     // last decode_eval found every erasure log 0 (identity_logs): no eval_poly kernel
    struct ProfRec {
        int id;
        hipEvent_t a, b;
    };
    std::vector<ProfRec> prof_pending;
    std::vector<hipEvent_t> ev_pool;
    double prof_ms[rs16::NUM_PROF] = {};
    uint64_t prof_n[rs16::NUM_PROF] = {};
    int prof_collect(rs16_error* err);

    // Engine ops on device shard arrays (validated by the C ABI layer).
    int fft(uint8_t* data, size_t S, size_t pos, size_t size, size_t skew_delta, hipStream_t s, rs16_error* err);
    int ifft(uint8_t* data, size_t S, size_t pos, size_t size, size_t skew_delta, hipStream_t s, rs16_error* err);

    // Fused HighRate single-chunk encode: originals rows [0,k) of d_orig ->
    // recovery rows [0,m) of d_rec, using Z (chunk rows) as work.
    // S = row width worked on (a column slice of the caller's arrays when
    // S < S_user), S_user = row stride of d_orig / d_rec (Z: stride S).
    int encode_high_fused(size_t k, size_t m, size_t S, size_t S_user, const uint8_t* d_orig, uint8_t* d_rec, uint8_t* Z,
                          hipStream_t s, rs16_error* err, size_t nstripes = 1, size_t bs_orig = 0, size_t bs_rec = 0);
    // Fused decode (both rates): seg_a / seg_b gather sources with device
    // flags; lost originals written to rest; Z, U work (n rows each; Z may
    // alias the sources when they live at their work positions).
    // S = row width, S_user = row stride of seg_a / seg_b / rest (Z, U: stride S)
    int decode_fused(const rs16::DecodeGeom& g, size_t S, size_t S_user, const uint8_t* seg_a, const uint8_t* flags_a,
                     const uint8_t* seg_b, const uint8_t* flags_b, uint8_t* rest, uint8_t* Z, uint8_t* U,
                     hipStream_t s, rs16_error* err);
    // decode_fused = decode_eval (erasure logs into ws_elog) + decode_passes.
    // S / nstripes: the width of the decode_passes launches that follow (0:
    // unknown); when the column codec will run them as a high-rate half
    // decode it computes eval_poly itself and no kernel is launched here.
    // vary > 1: nstripes = vary stripes with losses of their own, stripe i's
    // flags at flags_a / flags_b + i bs_fa / bs_fb bytes: one grid row of the
    // eval kernels per stripe, per-stripe metadata (VARY_* strides below),
    // which the decode_passes that follow read (var_* state).
    // Every erasure log of the decode is 0 (a whole-half erasure, DESIGN.md
    // 3.13): the multipliers are identities and eval_poly is not launched.
    bool identity_logs(const rs16::DecodeGeom& g, uint32_t vary) const;
    // Device tables of the L-bit general decode's middle-pass matrix
    // (mid_matrix_entries), uploaded on first use.
    int mid_tables(int L, const uint32_t** out, rs16_error* err);
    int decode_eval(const rs16::DecodeGeom& g, const uint8_t* flags_a, const uint8_t* flags_b, hipStream_t s,
                    rs16_error* err, size_t S = 0, size_t nstripes = 1, uint32_t vary = 0, size_t bs_fa = 0,
                    size_t bs_fb = 0);
    // per-stripe decode metadata of a batch with losses of its own
    static constexpr uint32_t VARY_WORK = rs16::GF_ORDER, VARY_RBITS = rs16::GF_ORDER / 32, VARY_ZFLAGS = 256,
                              VARY_LOST = 520;
    uint32_t var_ns = 0;           // last decode_eval: stripes with losses of their own (0: shared)
    uint64_t var_bs_fa = 0, var_bs_fb = 0;
    // rcount: where a column decode that evaluates the polynomial itself
    // writes the received counts (ErasureSpec::rcount layout): ws_rcount on
    // the call's own stream, a buffer of their own for concurrent slots.
    int decode_passes(const rs16::DecodeGeom& g, size_t S, size_t S_user, const uint8_t* seg_a, const uint8_t* flags_a,
                      const uint8_t* seg_b, const uint8_t* flags_b, uint8_t* rest, uint8_t* Z, uint8_t* U,
                      uint32_t* rcount, hipStream_t s, rs16_error* err, size_t nstripes = 1, size_t bs_a = 0,
                      size_t bs_b = 0, size_t bs_rest = 0);
    // The half-transform decode applies (every original lost, originals
    // segment = one half of the work rows).
    static bool half_decode(const rs16::DecodeGeom& g);
    // One-launch codec (rs16_col.hip) for transforms of 2^9 / 2^10 rows:
    // used when the launch has at most col_max_quads quad columns (x
    // stripes); wider launches take the pass codec, whose tiles share each
    // twiddle table over 32 quad columns.
    uint32_t col_max_quads = 256;  // (measured: scripts/probe_col.py)
    bool col_ok(int L, size_t S, size_t nstripes, bool gen = false) const;  // gen: the general decode (up to 2^11 rows)
    // Multi-chunk encodes of 2^8 .. 2^10-row chunks in the column codec: at
    // most col_max_chunk_rows rows in all (more take the passes: every
    // workgroup stages its own twiddle tables, and the low rate's repeats the
    // IFFT, so the column form's cost grows faster with the chunk count;
    // break-even 6-8 chunks of 1024 rows, scripts/probe_chunks.py)
    uint32_t col_max_chunk_rows = 6144;
    bool col_chunks_ok(int L, uint32_t nch, size_t S, bool high) const;
    int col(const rs16::ColArgs& a, int L, int mode, hipStream_t s, rs16_error* err);
    int col_multi(size_t k, size_t m, size_t S, size_t S_user, const uint8_t* d_orig, uint8_t* d_rec, uint32_t nch,
                  bool high, hipStream_t s, rs16_error* err);
    int col_tables(hipStream_t s, rs16_error* err);
    rs16::ColArgs col_args() const;
    // Multi-chunk encoders (high rate with k > chunk, low rate): every chunk's
    // transform in one batched set of launches.  d_orig rows have pitch
    // S_user, Z is the work space (work_count x S; may be d_orig), the
    // recovery rows [0, m) go to d_rec (pitch S_user; may be Z).
    int encode_high_multi(size_t k, size_t m, size_t S, size_t S_user, const uint8_t* d_orig, uint8_t* d_rec,
                          uint8_t* Z, hipStream_t s, rs16_error* err);
    // U: chunk x S bytes for the transformed originals, owned by the call's
    // stream (the engine's ws_u on the engine-ordered paths, a slot's own
    // buffer on concurrent slots); required -- there is no fallback.
    int encode_low_multi(size_t k, size_t m, size_t S, size_t S_user, const uint8_t* d_orig, uint8_t* d_rec,
                         uint8_t* Z, uint8_t* U, hipStream_t s, rs16_error* err);
    int fft_to_recovery(size_t m, size_t S, size_t S_user, const uint8_t* src, uint8_t* Z, uint8_t* d_rec,
                        size_t chunk, uint32_t nch, uint32_t skew, hipStream_t s, rs16_error* err);
};
