// rs16_api.cpp -- C ABI (include/rs16.h): errors, rate selection, the
// encoder/decoder state machines (EncoderWork / DecoderWork semantics of
// src/rate/{encoder,decoder}_work.rs) with HBM-resident work space, and the
// device-resident one-shot codec.
#include <atomic>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "rs16_engine.hpp"

using namespace rs16;

// ---------------------------------------------------------------------------
// Errors -- Display of src/lib.rs:130-222.
// ---------------------------------------------------------------------------
extern "C" size_t rs16_error_message(const rs16_error* e, char* buf, size_t len) {
    char tmp[256];
    unsigned long long a = e->v0, b = e->v1, c = e->v2;
    switch (e->code) {
    case RS16_OK: snprintf(tmp, sizeof tmp, "ok"); break;
    case RS16_DIFFERENT_SHARD_SIZE:
        snprintf(tmp, sizeof tmp, "different shard size: expected %llu bytes, got %llu bytes", a, b);
        break;
    case RS16_DUPLICATE_ORIGINAL_SHARD_INDEX: snprintf(tmp, sizeof tmp, "duplicate original shard index: %llu", a); break;
    case RS16_DUPLICATE_RECOVERY_SHARD_INDEX: snprintf(tmp, sizeof tmp, "duplicate recovery shard index: %llu", a); break;
    case RS16_INVALID_ORIGINAL_SHARD_INDEX:
        snprintf(tmp, sizeof tmp, "invalid original shard index: %llu >= original_count %llu", b, a);
        break;
    case RS16_INVALID_RECOVERY_SHARD_INDEX:
        snprintf(tmp, sizeof tmp, "invalid recovery shard index: %llu >= recovery_count %llu", b, a);
        break;
    case RS16_INVALID_SHARD_SIZE:
        snprintf(tmp, sizeof tmp, "invalid shard size: %llu bytes (must non-zero and multiple of 64)", a);
        break;
    case RS16_NOT_ENOUGH_SHARDS:
        snprintf(tmp, sizeof tmp, "not enough shards: %llu original + %llu recovery < %llu original_count", b, c, a);
        break;
    case RS16_TOO_FEW_ORIGINAL_SHARDS:
        snprintf(tmp, sizeof tmp, "too few original shards: got %llu shards while original_count is %llu", b, a);
        break;
    case RS16_TOO_MANY_ORIGINAL_SHARDS:
        snprintf(tmp, sizeof tmp, "too many original shards: got more than original_count (%llu) shards", a);
        break;
    case RS16_UNSUPPORTED_SHARD_COUNT:
        snprintf(tmp, sizeof tmp, "unsupported shard count: %llu original shards with %llu recovery shards", a, b);
        break;
    case RS16_DEVICE_ERROR:
        // v0 = hipError_t, or 1000 + ncclResult_t for an RCCL call (rs16_comm.cpp)
        if (a >= 1000)
            snprintf(tmp, sizeof tmp, "device error: RCCL: %s", ncclGetErrorString((ncclResult_t)(a - 1000)));
        else
            snprintf(tmp, sizeof tmp, "device error: %s", hipGetErrorString((hipError_t)a));
        break;
    case RS16_INVALID_ARGUMENT: snprintf(tmp, sizeof tmp, "invalid argument"); break;
    default: snprintf(tmp, sizeof tmp, "unknown error %d", e->code); break;
    }
    size_t n = strlen(tmp);
    if (buf && len) {
        size_t c2 = std::min(n, len - 1);
        memcpy(buf, tmp, c2);
        buf[c2] = 0;
    }
    return n;
}

extern "C" void rs16_host_mul(const void* in, void* out, size_t bytes, uint16_t log_m) {
    const uint32_t* t = &host_tables().mul_tab[(size_t)log_m * TAB_DWORDS];
    const uint8_t* src = (const uint8_t*)in;
    uint8_t* dst = (uint8_t*)out;
    for (size_t q = 0; q < bytes / 8; q++) {
        const size_t off = (q >> 3) * 64 + (q & 7) * 4;
        uint32_t yl, yh, ol = 0, oh = 0;
        memcpy(&yl, src + off, 4);
        memcpy(&yh, src + off + 32, 4);
        mul_xor(ol, oh, yl, yh, t);
        memcpy(dst + off, &ol, 4);
        memcpy(dst + off + 32, &oh, 4);
    }
}

extern "C" int rs16_engine_set_profiling(rs16_engine* e, int enable, rs16_error* err) {
    if (int rc = e->activate(err)) return rc;
    if (int rc = e->prof_collect(err)) return rc;
    e->profiling = enable != 0;
    return set_error(err, RS16_OK);
}
extern "C" int rs16_engine_profile_read(rs16_engine* e, int prog, double* total_ms, uint64_t* launches,
                                        rs16_error* err) {
    if (prog < 0 || prog >= NUM_PROF) return set_error(err, RS16_INVALID_ARGUMENT);
    if (int rc = e->activate(err)) return rc;
    if (int rc = e->prof_collect(err)) return rc;
    if (total_ms) *total_ms = e->prof_ms[prog];
    if (launches) *launches = e->prof_n[prog];
    return set_error(err, RS16_OK);
}
extern "C" void rs16_engine_profile_reset(rs16_engine* e) {
    rs16_error err;
    (void)e->activate(&err);
    (void)e->prof_collect(&err);
    for (int i = 0; i < NUM_PROF; i++) e->prof_ms[i] = 0, e->prof_n[i] = 0;
}
extern "C" int rs16_engine_set_stamps(rs16_engine* e, void* d_buf, int prog, rs16_error* err) {
    if (prog < -1 || prog >= NUM_PROF) return set_error(err, RS16_INVALID_ARGUMENT);
    e->stamp_buf = d_buf;
    e->stamp_prof = prog;
    return set_error(err, RS16_OK);
}
extern "C" int rs16_engine_set_slices(rs16_engine* e, int n, rs16_error* err) {
    if (n < 1 || n > rs16_engine::MAX_SLICES) return set_error(err, RS16_INVALID_ARGUMENT);
    e->slices = n;
    return set_error(err, RS16_OK);
}
// The received counts of the engine's last decode against the device flags
// (the eval_poly kernels count the received rows per 64-row chunk).
extern "C" int rs16_decode_check(rs16_engine* e, void* stream, rs16_error* err) {
    if (!e->last_dec_valid && !e->last_dec_flags_only) return set_error(err, RS16_OK);
    if (int rc = e->activate(err)) return rc;
    RS16_HIP(hipStreamSynchronize(e->pick(stream)));
    const DecodeGeom& g = e->last_dec;
    uint64_t a = 0, b = 0;
    if (e->last_dec_flags_only) {
        // nothing was restored and no kernel counted: count the copy of the
        // flags the decode took (note_flags_only; segment A / B sizes)
        std::vector<uint8_t> f(2 * (size_t)GF_ORDER);
        RS16_HIP(hipMemcpy(f.data(), e->ws_flags.p, f.size(), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < g.a_count; i++) a += f[i] != 0;
        for (uint32_t i = 0; i < g.b_count; i++) b += f[GF_ORDER + i] != 0;
    } else {
        const size_t chunks = ((size_t)g.n + 63) / 64;
        std::vector<uint32_t> c(2 * chunks);
        RS16_HIP(hipMemcpy(c.data(), e->ev_main.rcount.p, c.size() * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < chunks; i++) a += c[2 * i], b += c[2 * i + 1];
    }
    // (orig_recv, rec_recv) as the caller gave them to rs16_decode_device
    const uint64_t want_o = g.high ? g.b_recv : g.a_recv, want_r = g.high ? g.a_recv : g.b_recv;
    const uint64_t got_o = g.high ? b : a, got_r = g.high ? a : b;
    if (got_o != want_o || got_r != want_r) return set_error(err, RS16_INVALID_ARGUMENT, got_o, got_r);
    return set_error(err, RS16_OK);
}
static constexpr int DIAG_ALL = DIAG_FORCE_VOFF64 | DIAG_EVAL_TWO_KERNEL | DIAG_EVAL_FULL | DIAG_NO_COLUMN |
                                DIAG_FORCE_COLUMN | DIAG_TILE_LAST | DIAG_NO_TILE_LAST | DIAG_FD_LDS |
                                DIAG_COL_RADIX4 | DIAG_NO_IDENTITY | DIAG_NO_MID_DIRECT;
extern "C" int rs16_engine_set_diagnostics(rs16_engine* e, int flags) {
    const int old = e->diag;
    e->diag = flags & DIAG_ALL;
    return old;
}
// Deprecated process-wide form (the round-4 ABI): the flags every engine
// created afterwards starts with.  Existing engines keep their own.
static std::atomic<int> g_default_diag{0};
extern "C" int rs16_set_diagnostics(int flags) { return g_default_diag.exchange(flags & DIAG_ALL); }
extern "C" int rs16_prog_count(void) { return NUM_PROF; }
extern "C" const char* rs16_prog_name(int prog) {
    static const char* names[] = {"GEN_FFT",   "GEN_IFFT",   "ENC_FIRST",     "ENC_MID",
                                  "ENC_LAST",  "ENC_SINGLE", "DEC_FIRST",     "DEC_MID",
                                  "DEC_LAST",  "DEC_SINGLE", "DEC_HALF_LAST", "DEC_HALF_SINGLE",
                                  "DEC_HALF_FIRST", "DEC_HALF_MID", "EVAL_POLY", "COL_ENC", "COL_DEC",
                                  "DEC_MID_DIRECT", "DEC_TILE_LAST"};
    static_assert(sizeof names / sizeof names[0] == NUM_PROF, "profiling names");
    return (prog >= 0 && prog < NUM_PROF) ? names[prog] : "?";
}

extern "C" const char* rs16_version(void) { return "rs16-mi355x 0.1 gfx950 (v_perm GF(2^16) engine)"; }

// ---------------------------------------------------------------------------
// Rates.
// ---------------------------------------------------------------------------
static bool high_supports(size_t k, size_t m) {  // src/rate/rate_high.rs:19-25
    return k > 0 && m > 0 && k < GF_ORDER && m < GF_ORDER && next_pow2(m) + k <= GF_ORDER;
}
static bool low_supports(size_t k, size_t m) {  // src/rate/rate_low.rs:19-25
    return k > 0 && m > 0 && k < GF_ORDER && m < GF_ORDER && next_pow2(k) + m <= GF_ORDER;
}

extern "C" int rs16_use_high_rate(size_t k, size_t m, rs16_error* err) {  // rate_default.rs:15-64
    if (k > GF_ORDER || m > GF_ORDER) return set_error(err, RS16_UNSUPPORTED_SHARD_COUNT, k, m), -1;
    const size_t kp = next_pow2(k), mp = next_pow2(m);
    const size_t smaller = std::min(kp, mp), larger = std::max(k, m);
    if (k == 0 || m == 0 || smaller + larger > GF_ORDER) return set_error(err, RS16_UNSUPPORTED_SHARD_COUNT, k, m), -1;
    set_error(err, RS16_OK);
    if (kp < mp) return 0;
    if (kp > mp) return 1;
    return k <= m ? 1 : 0;
}

extern "C" int rs16_supports(int rate, size_t k, size_t m) {
    if (rate == RS16_RATE_HIGH) return high_supports(k, m);
    if (rate == RS16_RATE_LOW) return low_supports(k, m);
    return rs16_use_high_rate(k, m, nullptr) >= 0;
}

extern "C" int rs16_validate(int rate, size_t k, size_t m, size_t S, rs16_error* err) {  // src/rate.rs:91-106
    if (!rs16_supports(rate, k, m)) return set_error(err, RS16_UNSUPPORTED_SHARD_COUNT, k, m);
    if (S == 0 || (S & 63) != 0) return set_error(err, RS16_INVALID_SHARD_SIZE, S);
    return set_error(err, RS16_OK);
}

extern "C" size_t rs16_encoder_work_count(int high, size_t k, size_t m) {
    const size_t chunk = high ? next_pow2(m) : next_pow2(k);
    const size_t n = high ? k : m;
    return (n + chunk - 1) / chunk * chunk;
}
extern "C" size_t rs16_decoder_work_count(int high, size_t k, size_t m) {
    return high ? next_pow2(next_pow2(m) + k) : next_pow2(next_pow2(k) + m);
}

// Resolve the rate of a (rate kind, k, m) request and validate it, the way
// DefaultRate{En,De}coder::new / reset and {High,Low}Rate*::reset_work do.
static int resolve_rate(int rate, size_t k, size_t m, size_t S, bool* high, rs16_error* err) {
    if (rate == RS16_RATE_DEFAULT) {
        int h = rs16_use_high_rate(k, m, err);
        if (h < 0) return err ? err->code : RS16_UNSUPPORTED_SHARD_COUNT;
        *high = h == 1;
    } else if (rate == RS16_RATE_HIGH || rate == RS16_RATE_LOW) {
        *high = rate == RS16_RATE_HIGH;
    } else {
        return set_error(err, RS16_INVALID_ARGUMENT);
    }
    return rs16_validate(*high ? RS16_RATE_HIGH : RS16_RATE_LOW, k, m, S, err);
}

// ---------------------------------------------------------------------------
// Engine.
// ---------------------------------------------------------------------------
static void detach(rs16_encoder* enc);
static void detach(rs16_decoder* dec);

extern "C" rs16_engine* rs16_engine_new(int device, rs16_error* err) { return rs16_engine_new_ex(device, 0, err); }

extern "C" rs16_engine* rs16_engine_new_ex(int device, int flags, rs16_error* err) {
    if (flags & ~RS16_ENGINE_OWN_QUEUE) return set_error(err, RS16_INVALID_ARGUMENT), nullptr;
    int ndev = 0;
    hipError_t he = hipGetDeviceCount(&ndev);
    if (he != hipSuccess) return hip_fail(err, he), nullptr;
    if (device < 0 || device >= ndev) return set_error(err, RS16_INVALID_ARGUMENT), nullptr;
    rs16_engine* e = new (std::nothrow) rs16_engine();
    if (!e) return set_error(err, RS16_INVALID_ARGUMENT), nullptr;
    e->device = device;
    e->diag = g_default_diag.load();
    const HostTables& t = host_tables();
    auto fail = [&](hipError_t x) {
        hip_fail(err, x);
        rs16_engine_free(e);
        return (rs16_engine*)nullptr;
    };
    if ((he = hipSetDevice(device)) != hipSuccess) return fail(he);
    if (flags & RS16_ENGINE_OWN_QUEUE) {
        // A stream with a CU mask gets a hardware queue of its own (the HIP
        // runtime shares its GPU_MAX_HW_QUEUES queues only among unmasked
        // streams); the mask enables every CU.
        int cus = 0;
        if ((he = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess) return fail(he);
        std::vector<uint32_t> mask(((size_t)cus + 31) / 32, 0xFFFFFFFFu);
        if (cus % 32) mask.back() = (1u << (cus % 32)) - 1;
        if ((he = hipExtStreamCreateWithCUMask(&e->stream, (uint32_t)mask.size(), mask.data())) != hipSuccess)
            return fail(he);
    } else if ((he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking)) != hipSuccess) {
        return fail(he);
    }
    e->flags = flags;
    if ((he = hipMalloc(&e->d_skew_tab, (size_t)GF_ORDER * TAB_DWORDS * 4)) != hipSuccess) return fail(he);
    if ((he = hipMalloc(&e->d_mul_tab, t.mul_tab.size() * 4)) != hipSuccess) return fail(he);
    if ((he = hipMalloc(&e->d_log_walsh, GF_ORDER * 2)) != hipSuccess) return fail(he);
    if ((he = hipMalloc(&e->d_zero_sink, RS16_ZERO_BYTES)) != hipSuccess) return fail(he);
    if ((he = hipMemset(e->d_zero_sink, 0, RS16_ZERO_BYTES)) != hipSuccess) return fail(he);
    if ((he = hipMemcpy(e->d_skew_tab, t.skew_tab.data(), t.skew_tab.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return fail(he);
    if ((he = hipMemcpy(e->d_mul_tab, t.mul_tab.data(), t.mul_tab.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return fail(he);
    if ((he = hipMemcpy(e->d_log_walsh, t.log_walsh.data(), GF_ORDER * 2, hipMemcpyHostToDevice)) != hipSuccess) return fail(he);
    set_error(err, RS16_OK);
    return e;
}

extern "C" void rs16_engine_free(rs16_engine* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    // The streams this engine's work can be on: its own, the slice and
    // host-pipeline streams, and the last caller stream that used its scratch
    // (through order_ev).  Other engines and unrelated work are not waited for.
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    for (int j = 0; j < rs16_engine::MAX_SLICES; j++)
        if (e->sl_own[j]) (void)hipStreamSynchronize(e->sl_own[j]);
    for (auto& sl : e->hslot)
        if (sl.s) (void)hipStreamSynchronize(sl.s);
    if (e->last == rs16_engine::LAST_CALLER && e->order_ev) (void)hipEventSynchronize(e->order_ev);
    for (rs16_encoder* c : e->encoders) detach(c);
    for (rs16_decoder* c : e->decoders) detach(c);
    e->ws_z.release();
    e->ws_u.release();
    e->ws_fd.release();
    for (auto& b : e->mid_tab) b.release();
    e->ev_main.release();
    for (auto& l : e->ev_lane) l.release();
    e->ws_flags.release();
    e->hp_flags.release();
    for (auto& sl : e->hslot) {
        if (sl.s) (void)hipStreamSynchronize(sl.s), (void)hipStreamDestroy(sl.s);
        sl.orig.release(), sl.rec.release(), sl.z.release(), sl.u.release();
    }
    e->hflags.release();
    if (e->hev) (void)hipEventDestroy(e->hev);
    if (e->prep_ev) (void)hipEventDestroy(e->prep_ev);
    for (auto& ev : e->hp_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (e->hp_off) (void)hipEventDestroy(e->hp_off);
    if (e->order_ev) (void)hipEventDestroy(e->order_ev);
    for (int j = 0; j < rs16_engine::MAX_SLICES; j++) {
        if (e->sl_own[j]) (void)hipStreamDestroy(e->sl_own[j]);
        if (e->sl_join[j]) (void)hipEventDestroy(e->sl_join[j]);
    }
    if (e->sl_fork) (void)hipEventDestroy(e->sl_fork);
    if (e->d_skew_tab) (void)hipFree(e->d_skew_tab);
    if (e->d_mul_tab) (void)hipFree(e->d_mul_tab);
    if (e->d_col_img) (void)hipFree(e->d_col_img);
    if (e->d_col_v) (void)hipFree(e->d_col_v);
    if (e->d_log_walsh) (void)hipFree(e->d_log_walsh);
    if (e->d_zero_sink) (void)hipFree(e->d_zero_sink);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

extern "C" int rs16_engine_device(const rs16_engine* e) { return e->device; }
extern "C" void* rs16_engine_stream(const rs16_engine* e) { return (void*)e->stream; }
extern "C" int rs16_engine_synchronize(rs16_engine* e, void* stream, rs16_error* err) {
    if (int rc = e->activate(err)) return rc;
    RS16_HIP(hipStreamSynchronize(e->pick(stream)));
    return set_error(err, RS16_OK);
}

// ---- engine ops -----------------------------------------------------------
static bool is_pow2(size_t x) { return x && !(x & (x - 1)); }

static int check_transform(size_t shard_count, size_t S, size_t pos, size_t size, size_t trunc, size_t skew_delta,
                           rs16_error* err) {
    if (S == 0 || (S & 63) || !is_pow2(size) || size > GF_ORDER || trunc > size || pos + size > shard_count)
        return set_error(err, RS16_INVALID_ARGUMENT);
    // largest twiddle index touched: (size - 2) + skew_delta must be < GF_MODULUS
    if (size >= 2 && size - 2 + skew_delta >= GF_MODULUS) return set_error(err, RS16_INVALID_ARGUMENT);
    return RS16_OK;
}

extern "C" int rs16_engine_fft(rs16_engine* e, void* data, size_t shard_count, size_t S, size_t pos, size_t size,
                               size_t trunc, size_t skew_delta, void* stream, rs16_error* err) {
    if (int rc = check_transform(shard_count, S, pos, size, trunc, skew_delta, err)) return rc;
    if (int rc = e->activate(err)) return rc;
    if (int rc = e->fft((uint8_t*)data, S, pos, size, skew_delta, e->pick(stream), err)) return rc;
    return set_error(err, RS16_OK);
}
extern "C" int rs16_engine_fft_skew_end(rs16_engine* e, void* data, size_t shard_count, size_t S, size_t pos,
                                        size_t size, size_t trunc, void* stream, rs16_error* err) {
    return rs16_engine_fft(e, data, shard_count, S, pos, size, trunc, pos + size, stream, err);
}
extern "C" int rs16_engine_ifft(rs16_engine* e, void* data, size_t shard_count, size_t S, size_t pos, size_t size,
                                size_t trunc, size_t skew_delta, void* stream, rs16_error* err) {
    if (int rc = check_transform(shard_count, S, pos, size, trunc, skew_delta, err)) return rc;
    if (int rc = e->activate(err)) return rc;
    if (int rc = e->ifft((uint8_t*)data, S, pos, size, skew_delta, e->pick(stream), err)) return rc;
    return set_error(err, RS16_OK);
}
extern "C" int rs16_engine_ifft_skew_end(rs16_engine* e, void* data, size_t shard_count, size_t S, size_t pos,
                                         size_t size, size_t trunc, void* stream, rs16_error* err) {
    return rs16_engine_ifft(e, data, shard_count, S, pos, size, trunc, pos + size, stream, err);
}
extern "C" int rs16_engine_fwht(rs16_engine* e, uint16_t* d, size_t trunc, void* stream, rs16_error* err) {
    if (trunc > GF_ORDER) return set_error(err, RS16_INVALID_ARGUMENT);
    if (int rc = e->activate(err)) return rc;
    if (int rc = e->order(e->pick(stream), err)) return rc;
    if (int rc = e->guard_eval(e->pick(stream), false, err)) return rc;
    RS16_HIP(e->evset->work32.reserve(GF_ORDER * 4));
    RS16_HIP(launch_fwht_u16(d, (uint32_t*)e->evset->work32.p, e->pick(stream)));
    if (int rc = e->scratch_done(e->pick(stream), err)) return rc;
    return set_error(err, RS16_OK);
}
extern "C" int rs16_engine_eval_poly(rs16_engine* e, uint16_t* d, size_t trunc, void* stream, rs16_error* err) {
    if (trunc > GF_ORDER) return set_error(err, RS16_INVALID_ARGUMENT);
    if (int rc = e->activate(err)) return rc;
    if (int rc = e->order(e->pick(stream), err)) return rc;
    if (int rc = e->guard_eval(e->pick(stream), false, err)) return rc;
    RS16_HIP(e->evset->work32.reserve(GF_ORDER * 4));
    RS16_HIP(launch_eval_poly_u16(d, (uint32_t*)e->evset->work32.p, e->d_log_walsh, e->pick(stream)));
    if (int rc = e->scratch_done(e->pick(stream), err)) return rc;
    return set_error(err, RS16_OK);
}
extern "C" int rs16_engine_mul(rs16_engine* e, void* x, size_t bytes, uint16_t log_m, void* stream, rs16_error* err) {
    if (bytes & 63) return set_error(err, RS16_INVALID_ARGUMENT);
    if (int rc = e->activate(err)) return rc;
    RS16_HIP(launch_mul((uint8_t*)x, bytes, log_m, e->d_mul_tab, e->pick(stream)));
    return set_error(err, RS16_OK);
}
extern "C" int rs16_engine_xor(rs16_engine* e, void* x, const void* y, size_t bytes, void* stream, rs16_error* err) {
    if (bytes & 63) return set_error(err, RS16_INVALID_ARGUMENT);
    if (int rc = e->activate(err)) return rc;
    RS16_HIP(launch_xor((uint8_t*)x, (const uint8_t*)y, bytes, e->pick(stream)));
    return set_error(err, RS16_OK);
}
extern "C" int rs16_engine_xor_within(rs16_engine* e, void* data, size_t shard_count, size_t S, size_t x, size_t y,
                                      size_t count, void* stream, rs16_error* err) {
    if ((S & 63) || x + count > shard_count || y + count > shard_count || (x < y ? x + count > y : y + count > x))
        return set_error(err, RS16_INVALID_ARGUMENT);
    uint8_t* d = (uint8_t*)data;
    return rs16_engine_xor(e, d + x * S, d + y * S, count * S, stream, err);
}
extern "C" int rs16_engine_formal_derivative(rs16_engine* e, void* data, size_t n, size_t S, void* stream,
                                             rs16_error* err) {
    if ((S & 63) || S == 0 || !is_pow2(n)) return set_error(err, RS16_INVALID_ARGUMENT);
    if (int rc = e->activate(err)) return rc;
    hipStream_t s = e->pick(stream);
    if (int rc = e->order(s, err)) return rc;
    RS16_HIP(e->ws_fd.reserve(n * S));
    RS16_HIP(launch_formal_derivative((uint8_t*)e->ws_fd.p, (const uint8_t*)data, n, S, s));
    RS16_HIP(hipMemcpyAsync(data, e->ws_fd.p, n * S, hipMemcpyDeviceToDevice, s));
    if (int rc = e->scratch_done(s, err)) return rc;
    return set_error(err, RS16_OK);
}

// ---------------------------------------------------------------------------
// Host staging of the Rate-level API.  The reference copies every added shard
// into its work buffer (src/rate/encoder_work.rs:49-69,
// src/rate/decoder_work.rs:62-116) and serves results out of it
// (EncoderResult::recovery / DecoderResult::restored_original).  Here a shard
// added from host memory is copied (host memcpy, no HIP call) into a
// page-locked image of the work buffer; runs of consecutive rows stream to
// HBM in DMA copies of >= STREAM_BYTES while the caller keeps adding, the
// rest goes at encode()/decode(); the results come back in one DMA copy into
// the page-locked image, and the result accessors wait for it.  encode() and
// decode() return once everything is enqueued on the engine stream.
// ---------------------------------------------------------------------------
static constexpr size_t STREAM_BYTES = (size_t)1 << 20;

// ---------------------------------------------------------------------------
// Encoder -- EncoderWork (src/rate/encoder_work.rs) + Rate encoders.
// ---------------------------------------------------------------------------
struct rs16_encoder {
    rs16_engine* eng;  // nullptr once the engine was freed (detached)
    int rate_kind;
    bool high = true;
    // encoded: an EncoderResult is alive (encode ran, result not dropped).
    // The encode works in place, so a second encode before the drop would
    // read recovery rows as originals; the reference's borrow rules rule
    // that out at compile time (src/rate.rs:157-166), here it is an error.
    bool encoded = false;
    size_t k = 0, m = 0, S = 0, work_count = 0, received = 0;
    DevBuf work;
    // Host staging: h_in holds the rows added from host memory (row = the
    // shard's position, as the reference's work buffer); rows [run0,
    // received) are there but not yet copied to `work`.  h_out receives the
    // recovery rows.  in_done: the last H2D out of h_in (h_in may be
    // rewritten once it completed); out_done: the D2H into h_out.
    HostBuf h_in, h_out;
    size_t run0 = 0;
    bool host_round = false;  // a shard of this round came from host memory
    bool out_on_host = false;  // the D2H of this round's recovery rows is issued
    Pending in_done, out_done;
};

static void detach(rs16_encoder* enc) {
    enc->work.release();
    enc->h_in.release();
    enc->h_out.release();
    enc->in_done.release();
    enc->out_done.release();
    enc->eng = nullptr;
}
template <class V, class T> static void forget(V& v, T* x) { v.erase(std::remove(v.begin(), v.end(), x), v.end()); }

static void encoder_new_round(rs16_encoder* enc) {
    enc->received = 0;
    enc->encoded = false;
    enc->run0 = 0;
    enc->host_round = false;
    enc->out_on_host = false;
}

static int encoder_reset_impl(rs16_encoder* enc, size_t k, size_t m, size_t S, rs16_error* err) {
    if (!enc->eng) return set_error(err, RS16_INVALID_ARGUMENT);
    bool high;
    if (int rc = resolve_rate(enc->rate_kind, k, m, S, &high, err)) return rc;
    const size_t wc = rs16_encoder_work_count(high, k, m);
    if (int rc = enc->eng->activate(err)) return rc;
    RS16_HIP(enc->work.reserve(wc * S));
    enc->high = high;
    enc->k = k;
    enc->m = m;
    enc->S = S;
    enc->work_count = wc;
    encoder_new_round(enc);
    return set_error(err, RS16_OK);
}

extern "C" rs16_encoder* rs16_encoder_new(rs16_engine* eng, int rate, size_t k, size_t m, size_t S, rs16_error* err) {
    if (!eng) return set_error(err, RS16_INVALID_ARGUMENT), nullptr;
    rs16_encoder* enc = new (std::nothrow) rs16_encoder();
    if (!enc) return set_error(err, RS16_INVALID_ARGUMENT), nullptr;
    enc->eng = eng;
    enc->rate_kind = rate;
    eng->encoders.push_back(enc);
    if (encoder_reset_impl(enc, k, m, S, err)) {
        rs16_encoder_free(enc);
        return nullptr;
    }
    return enc;
}
extern "C" void rs16_encoder_free(rs16_encoder* enc) {
    if (!enc) return;
    if (rs16_engine* e = enc->eng) {
        (void)hipSetDevice(e->device);
        (void)hipStreamSynchronize(e->stream);
        detach(enc);
        forget(e->encoders, enc);
    }
    delete enc;
}
extern "C" int rs16_encoder_reset(rs16_encoder* enc, size_t k, size_t m, size_t S, rs16_error* err) {
    return encoder_reset_impl(enc, k, m, S, err);
}
// Copy the staged host rows [run0, upto) to the device work rows.
static int encoder_stream(rs16_encoder* enc, size_t upto, rs16_error* err) {
    if (upto <= enc->run0) return RS16_OK;
    const size_t S = enc->S;
    RS16_HIP(hipMemcpyAsync((uint8_t*)enc->work.p + enc->run0 * S, (const uint8_t*)enc->h_in.p + enc->run0 * S,
                            (upto - enc->run0) * S, hipMemcpyHostToDevice, enc->eng->stream));
    enc->run0 = upto;
    return RS16_OK;
}
static int encoder_add(rs16_encoder* enc, const void* shard, size_t len, bool device, rs16_error* err) {
    if (!enc->eng) return set_error(err, RS16_INVALID_ARGUMENT);
    if (enc->received == enc->k) return set_error(err, RS16_TOO_MANY_ORIGINAL_SHARDS, enc->k);
    if (len != enc->S) return set_error(err, RS16_DIFFERENT_SHARD_SIZE, enc->S, len);
    const size_t r = enc->received, S = enc->S;
    if (device) {
        if (int rc = enc->eng->activate(err)) return rc;
        if (int rc = encoder_stream(enc, r, err)) return rc;  // (host rows before it)
        RS16_HIP(hipMemcpyAsync((uint8_t*)enc->work.p + r * S, shard, len, hipMemcpyDeviceToDevice, enc->eng->stream));
        enc->run0 = r + 1;
    } else {
        if (r == 0) {
            // the previous round's copies out of h_in must be done
            RS16_HIP(enc->in_done.wait());
            RS16_HIP(enc->h_in.reserve(enc->k * S));
        }
        memcpy((uint8_t*)enc->h_in.p + r * S, shard, len);
        enc->host_round = true;
        if ((r + 1 - enc->run0) * S >= STREAM_BYTES) {
            if (int rc = enc->eng->activate(err)) return rc;
            if (int rc = encoder_stream(enc, r + 1, err)) return rc;
        }
    }
    enc->received = r + 1;
    return set_error(err, RS16_OK);
}
extern "C" int rs16_encoder_add_original_shard(rs16_encoder* enc, const void* shard, size_t len, rs16_error* err) {
    return encoder_add(enc, shard, len, false, err);
}
extern "C" int rs16_encoder_add_original_shard_device(rs16_encoder* enc, const void* d, size_t len, rs16_error* err) {
    return encoder_add(enc, d, len, true, err);
}
// D2H of every recovery row into h_out (once per round).
static int encoder_fetch(rs16_encoder* enc, rs16_error* err) {
    if (enc->out_on_host) return RS16_OK;
    RS16_HIP(enc->h_out.reserve(enc->m * enc->S));
    RS16_HIP(hipMemcpyAsync(enc->h_out.p, enc->work.p, enc->m * enc->S, hipMemcpyDeviceToHost, enc->eng->stream));
    RS16_HIP(enc->out_done.record(enc->eng->stream));
    enc->out_on_host = true;
    return RS16_OK;
}
extern "C" int rs16_encoder_encode(rs16_encoder* enc, rs16_error* err) {
    if (!enc->eng || enc->encoded) return set_error(err, RS16_INVALID_ARGUMENT);
    if (enc->received != enc->k) return set_error(err, RS16_TOO_FEW_ORIGINAL_SHARDS, enc->k, enc->received);
    rs16_engine* e = enc->eng;
    if (int rc = e->activate(err)) return rc;
    if (int rc = e->order(e->stream, err)) return rc;
    if (enc->host_round) {
        if (int rc = encoder_stream(enc, enc->received, err)) return rc;
        RS16_HIP(enc->in_done.record(e->stream));
    }
    uint8_t* w = (uint8_t*)enc->work.p;
    const size_t chunk = next_pow2(enc->m);
    int rc;
    if (enc->high && enc->k <= chunk)
        rc = e->encode_high_fused(enc->k, enc->m, enc->S, enc->S, w, w, w, e->stream, err);
    else if (enc->high)
        rc = e->encode_high_multi(enc->k, enc->m, enc->S, enc->S, w, w, w, e->stream, err);
    else
        rc = e->ws_u.reserve(next_pow2(enc->k) * enc->S) == hipSuccess
                 ? e->encode_low_multi(enc->k, enc->m, enc->S, enc->S, w, w, w, (uint8_t*)e->ws_u.p, e->stream, err)
                 : hip_fail(err, hipErrorOutOfMemory);
    if (rc) return rc;
    if (int rc2 = e->scratch_done(e->stream, err)) return rc2;
    // a host round gets its results back in one copy, right behind the passes
    if (enc->host_round)
        if (int rc2 = encoder_fetch(enc, err)) return rc2;
    enc->encoded = true;
    return set_error(err, RS16_OK);
}
extern "C" const void* rs16_encoder_recovery_device(rs16_encoder* enc, size_t index) {
    return enc->eng && enc->encoded && index < enc->m ? (const uint8_t*)enc->work.p + index * enc->S : nullptr;
}
static const void* encoder_recovery_host(rs16_encoder* enc, size_t index, rs16_error* err) {
    if (!(enc->eng && enc->encoded && index < enc->m)) return set_error(err, RS16_OK), nullptr;
    // (the common case -- rows already copied back -- makes no HIP call)
    if (enc->out_on_host && !enc->out_done.busy)
        return set_error(err, RS16_OK), (const uint8_t*)enc->h_out.p + index * enc->S;
    if (enc->eng->activate(err) || encoder_fetch(enc, err)) return nullptr;
    hipError_t he = enc->out_done.wait();
    if (he != hipSuccess) return hip_fail(err, he), nullptr;
    set_error(err, RS16_OK);
    return (const uint8_t*)enc->h_out.p + index * enc->S;
}
extern "C" const void* rs16_encoder_recovery(rs16_encoder* enc, size_t index, rs16_error* err) {
    return encoder_recovery_host(enc, index, err);
}
extern "C" int rs16_encoder_recovery_copy(rs16_encoder* enc, size_t index, void* dst, size_t len, rs16_error* err) {
    if (!rs16_encoder_recovery_device(enc, index)) return set_error(err, RS16_OK), 0;
    if (len < enc->S) return set_error(err, RS16_INVALID_ARGUMENT), -1;
    const void* src = encoder_recovery_host(enc, index, err);
    if (!src) return -1;
    memcpy(dst, src, enc->S);
    return 1;
}
extern "C" void rs16_encoder_result_drop(rs16_encoder* enc) { encoder_new_round(enc); }
extern "C" int rs16_encoder_is_high_rate(const rs16_encoder* enc) { return enc->high; }

// ---------------------------------------------------------------------------
// Decoder -- DecoderWork (src/rate/decoder_work.rs) + Rate decoders.
// ---------------------------------------------------------------------------
struct rs16_decoder {
    rs16_engine* eng;  // nullptr once the engine was freed (detached)
    int rate_kind;
    bool high = true;
    // decoded: a DecoderResult is alive.  The decode restores in place, so
    // adding shards or decoding again before the drop is an error (the
    // reference's borrow rules, src/rate.rs:235-244).
    bool decoded = false;
    size_t k = 0, m = 0, S = 0, work_count = 0;
    size_t orig_base = 0, rec_base = 0, orig_recv = 0, rec_recv = 0;
    std::vector<uint8_t> received;  // by work position
    DevBuf work, ubuf, flags;       // work = shards (z), ubuf = second work array (u)
    // Host staging: h_img is a page-locked image of the work layout.  hrow[pos]
    // = 1: row pos was added from host memory and is not yet on the device;
    // [run_lo, run_hi) is the latest stretch of consecutive host rows (it
    // streams to HBM once it reaches STREAM_BYTES).  h_flags: the received
    // flags of the two segments, for the device.
    HostBuf h_img, h_flags, h_out;  // h_out: restored originals, row = original index
    std::vector<uint8_t> hrow;
    size_t run_lo = 0, run_hi = 0;
    bool host_round = false, dev_round = false, out_on_host = false;
    Pending in_done, out_done;
};

static void detach(rs16_decoder* d) {
    d->work.release();
    d->ubuf.release();
    d->flags.release();
    d->h_img.release();
    d->h_flags.release();
    d->h_out.release();
    d->in_done.release();
    d->out_done.release();
    d->eng = nullptr;
}

static void decoder_new_round(rs16_decoder* d) {
    d->decoded = false;
    d->orig_recv = d->rec_recv = 0;
    std::fill(d->received.begin(), d->received.end(), 0);
    std::fill(d->hrow.begin(), d->hrow.end(), 0);
    d->run_lo = d->run_hi = 0;
    d->host_round = d->dev_round = d->out_on_host = false;
}

static int decoder_reset_impl(rs16_decoder* d, size_t k, size_t m, size_t S, rs16_error* err) {
    if (!d->eng) return set_error(err, RS16_INVALID_ARGUMENT);
    bool high;
    if (int rc = resolve_rate(d->rate_kind, k, m, S, &high, err)) return rc;
    const size_t wc = rs16_decoder_work_count(high, k, m);
    if (int rc = d->eng->activate(err)) return rc;
    RS16_HIP(d->work.reserve(wc * S));
    RS16_HIP(d->ubuf.reserve(wc * S));
    RS16_HIP(d->flags.reserve(GF_ORDER * 2));
    d->high = high;
    d->k = k;
    d->m = m;
    d->S = S;
    d->work_count = wc;
    d->orig_base = high ? next_pow2(m) : 0;  // rate_high.rs:279-299 / rate_low.rs:279-299
    d->rec_base = high ? 0 : next_pow2(k);
    d->received.assign(std::max(d->received.size(), wc), 0);
    d->hrow.assign(std::max(d->hrow.size(), wc), 0);
    decoder_new_round(d);
    return set_error(err, RS16_OK);
}

extern "C" rs16_decoder* rs16_decoder_new(rs16_engine* eng, int rate, size_t k, size_t m, size_t S, rs16_error* err) {
    if (!eng) return set_error(err, RS16_INVALID_ARGUMENT), nullptr;
    rs16_decoder* d = new (std::nothrow) rs16_decoder();
    if (!d) return set_error(err, RS16_INVALID_ARGUMENT), nullptr;
    d->eng = eng;
    d->rate_kind = rate;
    eng->decoders.push_back(d);
    if (decoder_reset_impl(d, k, m, S, err)) {
        rs16_decoder_free(d);
        return nullptr;
    }
    return d;
}
extern "C" void rs16_decoder_free(rs16_decoder* d) {
    if (!d) return;
    if (rs16_engine* e = d->eng) {
        (void)hipSetDevice(e->device);
        (void)hipStreamSynchronize(e->stream);
        detach(d);
        forget(e->decoders, d);
    }
    delete d;
}
extern "C" int rs16_decoder_reset(rs16_decoder* d, size_t k, size_t m, size_t S, rs16_error* err) {
    return decoder_reset_impl(d, k, m, S, err);
}
// Copy host rows [lo, hi) of the image to the device work rows.
static int decoder_stream(rs16_decoder* d, size_t lo, size_t hi, rs16_error* err) {
    const size_t S = d->S;
    RS16_HIP(hipMemcpyAsync((uint8_t*)d->work.p + lo * S, (const uint8_t*)d->h_img.p + lo * S, (hi - lo) * S,
                            hipMemcpyHostToDevice, d->eng->stream));
    std::fill(d->hrow.begin() + lo, d->hrow.begin() + hi, 0);
    return RS16_OK;
}
// Every host row not yet on the device: maximal runs of such rows, or one
// copy of their whole span when they are scattered (rows in between were
// not received, and their device contents are never read -- unless a row
// in between came from device memory: then run by run).
static int decoder_stream_all(rs16_decoder* d, rs16_error* err) {
    const size_t wc = d->work_count;
    std::vector<std::pair<size_t, size_t>> runs;
    for (size_t i = 0; i < wc;) {
        if (!d->hrow[i]) {
            i++;
            continue;
        }
        size_t j = i;
        while (j < wc && d->hrow[j]) j++;
        runs.push_back({i, j});
        i = j;
    }
    if (runs.empty()) return RS16_OK;
    if (runs.size() > 32 && !d->dev_round) return decoder_stream(d, runs.front().first, runs.back().second, err);
    for (auto& r : runs)
        if (int rc = decoder_stream(d, r.first, r.second, err)) return rc;
    return RS16_OK;
}
static int decoder_add(rs16_decoder* d, bool original, size_t index, const void* shard, size_t len, bool device,
                       rs16_error* err) {
    if (!d->eng || d->decoded) return set_error(err, RS16_INVALID_ARGUMENT);
    const size_t count = original ? d->k : d->m;
    const size_t pos = (original ? d->orig_base : d->rec_base) + index;
    if (index >= count)
        return set_error(err, original ? RS16_INVALID_ORIGINAL_SHARD_INDEX : RS16_INVALID_RECOVERY_SHARD_INDEX, count,
                         index);
    if (d->received[pos])
        return set_error(err, original ? RS16_DUPLICATE_ORIGINAL_SHARD_INDEX : RS16_DUPLICATE_RECOVERY_SHARD_INDEX,
                         index);
    if (len != d->S) return set_error(err, RS16_DIFFERENT_SHARD_SIZE, d->S, len);
    const size_t S = d->S;
    if (device) {
        if (int rc = d->eng->activate(err)) return rc;
        RS16_HIP(hipMemcpyAsync((uint8_t*)d->work.p + pos * S, shard, len, hipMemcpyDeviceToDevice, d->eng->stream));
        d->dev_round = true;
    } else {
        if (!d->host_round) {
            // the previous round's copies out of the image must be done
            RS16_HIP(d->in_done.wait());
            RS16_HIP(d->h_img.reserve(d->work_count * S));
            d->host_round = true;
        }
        memcpy((uint8_t*)d->h_img.p + pos * S, shard, len);
        d->hrow[pos] = 1;
        if (pos == d->run_hi && d->run_hi > d->run_lo) d->run_hi++;
        else d->run_lo = pos, d->run_hi = pos + 1;
        if ((d->run_hi - d->run_lo) * S >= STREAM_BYTES) {
            if (int rc = d->eng->activate(err)) return rc;
            if (int rc = decoder_stream(d, d->run_lo, d->run_hi, err)) return rc;
            d->run_lo = d->run_hi;
        }
    }
    (original ? d->orig_recv : d->rec_recv)++;
    d->received[pos] = 1;
    return set_error(err, RS16_OK);
}
extern "C" int rs16_decoder_add_original_shard(rs16_decoder* d, size_t i, const void* s, size_t len, rs16_error* err) {
    return decoder_add(d, true, i, s, len, false, err);
}
extern "C" int rs16_decoder_add_recovery_shard(rs16_decoder* d, size_t i, const void* s, size_t len, rs16_error* err) {
    return decoder_add(d, false, i, s, len, false, err);
}
extern "C" int rs16_decoder_add_original_shard_device(rs16_decoder* d, size_t i, const void* s, size_t len,
                                                      rs16_error* err) {
    return decoder_add(d, true, i, s, len, true, err);
}
extern "C" int rs16_decoder_add_recovery_shard_device(rs16_decoder* d, size_t i, const void* s, size_t len,
                                                      rs16_error* err) {
    return decoder_add(d, false, i, s, len, true, err);
}
// D2H of the lost originals' rows into h_out (one copy of their span;
// received rows inside it come back as scratch, and are never read there).
static int decoder_fetch(rs16_decoder* d, rs16_error* err) {
    if (d->out_on_host) return RS16_OK;
    size_t lo = d->k, hi = 0;
    for (size_t i = 0; i < d->k; i++)
        if (!d->received[d->orig_base + i]) lo = std::min(lo, i), hi = i + 1;
    if (hi > lo) {
        const size_t S = d->S;
        RS16_HIP(d->h_out.reserve(d->k * S));
        RS16_HIP(hipMemcpyAsync((uint8_t*)d->h_out.p + lo * S, (const uint8_t*)d->work.p + (d->orig_base + lo) * S,
                                (hi - lo) * S, hipMemcpyDeviceToHost, d->eng->stream));
        RS16_HIP(d->out_done.record(d->eng->stream));
    }
    d->out_on_host = true;
    return RS16_OK;
}
extern "C" int rs16_decoder_decode(rs16_decoder* d, rs16_error* err) {
    if (!d->eng || d->decoded) return set_error(err, RS16_INVALID_ARGUMENT);
    // (the Rate decoder counts its own received set, as the reference does:
    // there is nothing for rs16_decode_check, which serves rs16_decode_device)
    d->eng->forget_decode();
    // decode_begin (src/rate/decoder_work.rs:120-139)
    if (d->orig_recv + d->rec_recv < d->k)
        return set_error(err, RS16_NOT_ENOUGH_SHARDS, d->k, d->orig_recv, d->rec_recv);
    if (d->orig_recv == d->k) return d->decoded = true, set_error(err, RS16_OK);  // nothing to do
    rs16_engine* e = d->eng;
    if (int rc = e->activate(err)) return rc;
    if (int rc = e->order(e->stream, err)) return rc;
    if (int rc = decoder_stream_all(d, err)) return rc;
    DecodeGeom g = decode_geom(d->high, d->k, d->m);
    g.a_recv = d->high ? d->rec_recv : d->orig_recv;
    g.b_recv = d->high ? d->orig_recv : d->rec_recv;
    // Received flags of the two segments -> device (bytes, one per row), out
    // of the page-locked staging (written once the previous round's copies
    // out of it are done).
    if (!d->host_round) RS16_HIP(d->in_done.wait());
    RS16_HIP(d->h_flags.reserve(GF_ORDER * 2));
    uint8_t* hf = (uint8_t*)d->h_flags.p;
    memcpy(hf, d->received.data(), g.a_count);
    memcpy(hf + GF_ORDER, d->received.data() + g.chunk, g.b_count);
    uint8_t* fl = (uint8_t*)d->flags.p;
    RS16_HIP(hipMemcpyAsync(fl, hf, g.a_count, hipMemcpyHostToDevice, e->stream));
    RS16_HIP(hipMemcpyAsync(fl + GF_ORDER, hf + GF_ORDER, g.b_count, hipMemcpyHostToDevice, e->stream));
    RS16_HIP(d->in_done.record(e->stream));
    uint8_t* w = (uint8_t*)d->work.p;
    if (int rc = e->decode_fused(g, d->S, d->S, w, fl, w + (size_t)g.chunk * d->S, fl + GF_ORDER, w + d->orig_base * d->S,
                                 w, (uint8_t*)d->ubuf.p, e->stream, err))
        return rc;
    e->forget_decode();
    if (int rc = e->scratch_done(e->stream, err)) return rc;
    if (d->host_round)
        if (int rc = decoder_fetch(d, err)) return rc;
    d->decoded = true;
    return set_error(err, RS16_OK);
}
extern "C" const void* rs16_decoder_restored_original_device(rs16_decoder* d, size_t index) {
    const size_t pos = d->orig_base + index;
    if (d->eng && d->decoded && index < d->k && !d->received[pos]) return (const uint8_t*)d->work.p + pos * d->S;
    return nullptr;
}
static const void* decoder_restored_host(rs16_decoder* d, size_t index, rs16_error* err) {
    if (!rs16_decoder_restored_original_device(d, index)) return set_error(err, RS16_OK), nullptr;
    if (d->out_on_host && !d->out_done.busy) return set_error(err, RS16_OK), (const uint8_t*)d->h_out.p + index * d->S;
    if (d->eng->activate(err) || decoder_fetch(d, err)) return nullptr;
    hipError_t he = d->out_done.wait();
    if (he != hipSuccess) return hip_fail(err, he), nullptr;
    set_error(err, RS16_OK);
    return (const uint8_t*)d->h_out.p + index * d->S;
}
extern "C" const void* rs16_decoder_restored_original(rs16_decoder* d, size_t index, rs16_error* err) {
    return decoder_restored_host(d, index, err);
}
extern "C" int rs16_decoder_restored_original_copy(rs16_decoder* d, size_t index, void* dst, size_t len,
                                                   rs16_error* err) {
    if (!rs16_decoder_restored_original_device(d, index)) return set_error(err, RS16_OK), 0;
    if (len < d->S) return set_error(err, RS16_INVALID_ARGUMENT), -1;
    const void* src = decoder_restored_host(d, index, err);
    if (!src) return -1;
    memcpy(dst, src, d->S);
    return 1;
}
extern "C" void rs16_decoder_result_drop(rs16_decoder* d) {  // DecoderWork::reset_received
    decoder_new_round(d);
}
extern "C" int rs16_decoder_is_high_rate(const rs16_decoder* d) { return d->high; }

// ---------------------------------------------------------------------------
// Device-resident one-shot codec.
// ---------------------------------------------------------------------------
// Device encode of one stripe (or column slice) with work space Z of
// work_count x S bytes, on stream s.
// Z: work_count x S, U: next_pow2(k) x S for the low rate (the transformed
// originals) -- both owned by stream s for the call: the engine's ws_z /
// ws_u on the engine-ordered paths (order() / scratch_done()), a slot's own
// buffers on concurrent slots.
static int encode_dev(rs16_engine* e, bool high, size_t k, size_t m, size_t S, const uint8_t* d_orig, uint8_t* d_rec,
                      uint8_t* Z, uint8_t* U, hipStream_t s, rs16_error* err) {
    if (high && k <= next_pow2(m)) return e->encode_high_fused(k, m, S, S, d_orig, d_rec, Z, s, err);
    return high ? e->encode_high_multi(k, m, S, S, d_orig, d_rec, Z, s, err)
                : e->encode_low_multi(k, m, S, S, d_orig, d_rec, Z, U, s, err);
}
// The engine's own low-rate scratch for an engine-ordered call.
static uint8_t* engine_u(rs16_engine* e, bool high, size_t k, size_t S, rs16_error* err, int* rc) {
    *rc = RS16_OK;
    if (high) return nullptr;
    if (hipError_t he = e->ws_u.reserve(next_pow2(k) * S)) return *rc = hip_fail(err, he), nullptr;
    return (uint8_t*)e->ws_u.p;
}

extern "C" int rs16_encode_device(rs16_engine* e, size_t k, size_t m, size_t S, const void* d_original,
                                  void* d_recovery, void* stream, rs16_error* err) {
    bool high;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    if (int rc = e->activate(err)) return rc;
    hipStream_t s = e->pick(stream);
    if (int rc = e->order(s, err)) return rc;
    const size_t wc = rs16_encoder_work_count(high, k, m);
    RS16_HIP(e->ws_z.reserve(wc * S));
    const int n = (high && k <= next_pow2(m)) ? e->slice_count(S) : 1;
    if (n == 1) {
        int urc;
        uint8_t* U = engine_u(e, high, k, S, err, &urc);
        if (urc) return urc;
        if (int rc = encode_dev(e, high, k, m, S, (const uint8_t*)d_original, (uint8_t*)d_recovery,
                                (uint8_t*)e->ws_z.p, U, s, err))
            return rc;
        if (int rc = e->scratch_done(s, err)) return rc;
        return set_error(err, RS16_OK);
    }
    // column slices on the engine's slice streams (work space: wc x width each)
    if (int rc = e->fork(s, n, err)) return rc;
    const size_t blocks = S / 64;
    for (int j = 0, b0 = 0; j < n; j++) {
        const size_t b1 = blocks * (j + 1) / n, off = b0 * 64, w = (b1 - b0) * 64;
        if (int rc = e->encode_high_fused(k, m, w, S, (const uint8_t*)d_original + off, (uint8_t*)d_recovery + off,
                                          (uint8_t*)e->ws_z.p + wc * off, e->sl_stream[j], err))
            return rc;
        b0 = (int)b1;
    }
    if (int rc = e->join(s, n, err)) return rc;
    if (int rc = e->scratch_done(s, err)) return rc;
    return set_error(err, RS16_OK);
}

// Many independent stripes of one geometry in one call: stripe i's originals
// at d_original + i original_stride, its recovery at d_recovery + i
// recovery_stride.  High-rate stripes with k <= chunk (every k <= m) run
// batched -- each pass launch covers all stripes -- so small stripes fill the
// chip; other shapes encode stripe by stripe.
extern "C" int rs16_encode_device_batch(rs16_engine* e, size_t k, size_t m, size_t S, size_t nstripes,
                                        const void* d_original, size_t original_stride, void* d_recovery,
                                        size_t recovery_stride, void* stream, rs16_error* err) {
    bool high;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    if (nstripes == 0) return set_error(err, RS16_OK);
    // (strides in whole 64-byte blocks, as shard sizes: every row stays aligned)
    if (!d_original || !d_recovery || original_stride < k * S || recovery_stride < m * S || original_stride % 64 ||
        recovery_stride % 64)
        return set_error(err, RS16_INVALID_ARGUMENT);
    const size_t chunk = next_pow2(m);
    // one launch holds < 2^32 tiles; stay far below
    if (nstripes > ((size_t)1 << 20)) return set_error(err, RS16_INVALID_ARGUMENT);
    if (int rc = e->activate(err)) return rc;
    hipStream_t s = e->pick(stream);
    if (int rc = e->order(s, err)) return rc;
    const size_t wc = rs16_encoder_work_count(high, k, m);
    const uint8_t* o = (const uint8_t*)d_original;
    uint8_t* r = (uint8_t*)d_recovery;
    if (high && k <= chunk) {
        RS16_HIP(e->ws_z.reserve(nstripes * chunk * S));
        if (int rc = e->encode_high_fused(k, m, S, S, o, r, (uint8_t*)e->ws_z.p, s, err, nstripes, original_stride,
                                          recovery_stride))
            return rc;
    } else {
        RS16_HIP(e->ws_z.reserve(wc * S));
        int urc;
        uint8_t* U = engine_u(e, high, k, S, err, &urc);
        if (urc) return urc;
        for (size_t i = 0; i < nstripes; i++)
            if (int rc = encode_dev(e, high, k, m, S, o + i * original_stride, r + i * recovery_stride,
                                    (uint8_t*)e->ws_z.p, U, s, err))
                return rc;
    }
    if (int rc = e->scratch_done(s, err)) return rc;
    return set_error(err, RS16_OK);
}

// ---------------------------------------------------------------------------
// Host-resident one-shot codec: shards start and end in host memory.
// ---------------------------------------------------------------------------
int rs16_engine::host_slots(rs16_error* err) {
    for (auto& sl : hslot)
        if (!sl.s) RS16_HIP(hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking));
    if (!hev) RS16_HIP(hipEventCreateWithFlags(&hev, hipEventDisableTiming));
    if (int rc = order(stream, err)) return rc;
    // start after the caller's earlier work on the engine stream
    RS16_HIP(hipEventRecord(hev, stream));
    for (auto& sl : hslot) RS16_HIP(hipStreamWaitEvent(sl.s, hev, 0));
    return RS16_OK;
}

// Column slice width: a multiple of 64 (every 64-byte column block is an
// independent codeword, src/algorithm.md:6-32); default: the whole shard.
// Measured on MI355X at 32768:32768 x 1 KiB (scripts/host_slices.py):
// 1024 / 512 / 256 / 128-byte slices take 1.33 / 1.40 / 1.97 / 3.16 ms per
// encode -- the pitched (2-D) pinned copies lose more than the overlap wins.
static size_t host_slice(size_t S, size_t slice) {
    if (slice == 0) slice = S;
    slice = std::max<size_t>(64, slice / 64 * 64);
    return std::min(slice, S);
}

extern "C" int rs16_encode_host(rs16_engine* e, size_t k, size_t m, size_t S, const void* h_original,
                                void* h_recovery, size_t slice_bytes, rs16_error* err) {
    bool high;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    if (int rc = e->activate(err)) return rc;
    const size_t W = host_slice(S, slice_bytes), wc = rs16_encoder_work_count(high, k, m);
    for (auto& sl : e->hslot) {
        RS16_HIP(sl.orig.reserve(k * W));
        RS16_HIP(sl.rec.reserve(m * W));
        RS16_HIP(sl.z.reserve(wc * W));
        if (!high) RS16_HIP(sl.u.reserve(next_pow2(k) * W));  // (the two slots run concurrently)
    }
    if (int rc = e->host_slots(err)) return rc;
    for (size_t off = 0, j = 0; off < S; off += W, j++) {
        const size_t w = std::min(W, S - off);
        auto& sl = e->hslot[j & 1];
        RS16_HIP(hipMemcpy2DAsync(sl.orig.p, w, (const uint8_t*)h_original + off, S, w, k, hipMemcpyHostToDevice,
                                  sl.s));
        if (int rc = encode_dev(e, high, k, m, w, (const uint8_t*)sl.orig.p, (uint8_t*)sl.rec.p, (uint8_t*)sl.z.p,
                                high ? nullptr : (uint8_t*)sl.u.p, sl.s, err))
            return rc;
        RS16_HIP(hipMemcpy2DAsync((uint8_t*)h_recovery + off, S, sl.rec.p, w, w, m, hipMemcpyDeviceToHost, sl.s));
    }
    for (auto& sl : e->hslot) RS16_HIP(hipStreamSynchronize(sl.s));
    if (int rc = e->scratch_done(e->stream, err)) return rc;
    return set_error(err, RS16_OK);
}

extern "C" int rs16_decode_host(rs16_engine* e, size_t k, size_t m, size_t S, void* h_original,
                                const uint8_t* original_received, const void* h_recovery,
                                const uint8_t* recovery_received, size_t slice_bytes, rs16_error* err) {
    bool high;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    size_t orig_recv = 0, rec_recv = 0;
    for (size_t i = 0; i < k; i++) orig_recv += original_received[i] != 0;
    for (size_t i = 0; i < m; i++) rec_recv += recovery_received[i] != 0;
    if (orig_recv + rec_recv < k) return set_error(err, RS16_NOT_ENOUGH_SHARDS, k, orig_recv, rec_recv);
    if (orig_recv == k) return set_error(err, RS16_OK);
    if (int rc = e->activate(err)) return rc;
    DecodeGeom g = decode_geom(high, k, m);
    g.a_recv = high ? rec_recv : orig_recv;
    g.b_recv = high ? orig_recv : rec_recv;
    const size_t W = host_slice(S, slice_bytes);
    for (auto& sl : e->hslot) {
        RS16_HIP(sl.orig.reserve(k * W));
        RS16_HIP(sl.rec.reserve(m * W));
        RS16_HIP(sl.z.reserve((size_t)g.n * W));
        RS16_HIP(sl.u.reserve((size_t)g.n * W));
        RS16_HIP(sl.rcount.reserve(GF_ORDER / 64 * 8));
    }
    // received flags -> device; erasure logs once, shared by every slice
    if (int rc = e->order(e->stream, err)) return rc;
    RS16_HIP(e->hflags.reserve(k + m));
    uint8_t* d_of = (uint8_t*)e->hflags.p;
    uint8_t* d_rf = d_of + k;
    RS16_HIP(hipMemcpyAsync(d_of, original_received, k, hipMemcpyHostToDevice, e->stream));
    RS16_HIP(hipMemcpyAsync(d_rf, recovery_received, m, hipMemcpyHostToDevice, e->stream));
    const uint8_t* fa = high ? d_rf : d_of;
    const uint8_t* fb = high ? d_of : d_rf;
    if (int rc = e->decode_eval(g, fa, fb, e->stream, err, W)) return rc;
    if (int rc = e->host_slots(err)) return rc;
    for (size_t off = 0, j = 0; off < S; off += W, j++) {
        const size_t w = std::min(W, S - off);
        auto& sl = e->hslot[j & 1];
        if (rec_recv)
            RS16_HIP(hipMemcpy2DAsync(sl.rec.p, w, (const uint8_t*)h_recovery + off, S, w, m, hipMemcpyHostToDevice,
                                      sl.s));
        if (orig_recv)
            RS16_HIP(hipMemcpy2DAsync(sl.orig.p, w, (const uint8_t*)h_original + off, S, w, k,
                                      hipMemcpyHostToDevice, sl.s));
        const uint8_t* o = (const uint8_t*)sl.orig.p;
        const uint8_t* r = (const uint8_t*)sl.rec.p;
        if (int rc = e->decode_passes(g, w, w, high ? r : o, fa, high ? o : r, fb, (uint8_t*)sl.orig.p,
                                      (uint8_t*)sl.z.p, (uint8_t*)sl.u.p, (uint32_t*)sl.rcount.p, sl.s, err))
            return rc;
        // restored originals land in place; received rows come back unchanged
        RS16_HIP(hipMemcpy2DAsync((uint8_t*)h_original + off, S, sl.orig.p, w, w, k, hipMemcpyDeviceToHost, sl.s));
    }
    for (auto& sl : e->hslot) RS16_HIP(hipStreamSynchronize(sl.s));
    if (int rc = e->scratch_done(e->stream, err)) return rc;
    // (the counts came from the host flags themselves: nothing for rs16_decode_check)
    e->forget_decode();
    return set_error(err, RS16_OK);
}

// ---------------------------------------------------------------------------
// Host-resident stripes, pipelined.  Two lanes, each a stream with device
// buffers and codec scratch of its own (hslot[b]: rows, Z, U; ev_lane[b]:
// the decode's eval_poly outputs): stripe i runs on lane i & 1 as
// H2D -> codec -> D2H in stream order, so while one lane copies a stripe's
// outputs back the other copies the next stripe's inputs in -- both link
// directions busy -- and no event crosses between streams (the copy engines'
// waits on other queues' events stalled the pipeline for milliseconds at a
// time, profiles/r05_hostbatch_trace.txt).
// ---------------------------------------------------------------------------
namespace {
// Contiguous runs of rows whose flag equals `want` (rows [0, n)), each one
// copy; more than max_runs of them: one copy of the span from the first to
// the last such row.
template <class F>
int copy_runs(const uint8_t* flags, size_t n, bool want, size_t max_runs, F copy) {
    size_t runs = 0, first = n, last = 0;
    for (size_t i = 0; i < n; i++) {
        if ((flags[i] != 0) != want) continue;
        if (i == 0 || (flags[i - 1] != 0) != want) runs++;
        first = std::min(first, i);
        last = i + 1;
    }
    if (runs == 0) return RS16_OK;
    if (runs > max_runs) return copy(first, last - first);
    for (size_t i = 0; i < n;) {
        if ((flags[i] != 0) != want) {
            i++;
            continue;
        }
        size_t j = i;
        while (j < n && (flags[j] != 0) == want) j++;
        if (int rc = copy(i, j - i)) return rc;
        i = j;
    }
    return RS16_OK;
}
constexpr size_t HP_MAX_RUNS = 64;
// the engine's decode scratch set, restored on every exit path
struct EvalSet {
    rs16_engine* e;
    explicit EvalSet(rs16_engine* eng, int lane) : e(eng) { e->evset = &e->ev_lane[lane]; }
    ~EvalSet() { e->evset = &e->ev_main; }
};
}  // namespace

int rs16_engine::host_pipe_events(rs16_error* err) {
    for (auto& ev : hp_ev)
        if (!ev) RS16_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    if (!hp_off) RS16_HIP(hipEventCreateWithFlags(&hp_off, hipEventDisableTiming));
    return RS16_OK;
}

extern "C" int rs16_encode_host_batch(rs16_engine* e, size_t k, size_t m, size_t S, size_t nstripes,
                                      const void* h_original, size_t original_stride, void* h_recovery,
                                      size_t recovery_stride, rs16_error* err) {
    bool high;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    if (nstripes == 0) return set_error(err, RS16_OK);
    if (!h_original || !h_recovery || original_stride < k * S || recovery_stride < m * S)
        return set_error(err, RS16_INVALID_ARGUMENT);
    if (int rc = e->activate(err)) return rc;
    const size_t wc = rs16_encoder_work_count(high, k, m);
    for (auto& sl : e->hslot) {
        RS16_HIP(sl.orig.reserve(k * S));
        RS16_HIP(sl.rec.reserve(m * S));
        RS16_HIP(sl.z.reserve(wc * S));
        if (!high) RS16_HIP(sl.u.reserve(next_pow2(k) * S));
    }
    if (int rc = e->host_pipe_events(err)) return rc;
    if (int rc = e->host_slots(err)) return rc;  // (lanes after the engine stream's earlier work)
    for (size_t i = 0; i < nstripes; i++) {
        auto& sl = e->hslot[i & 1];
        uint8_t* d_o = (uint8_t*)sl.orig.p;
        uint8_t* d_r = (uint8_t*)sl.rec.p;
        // lane 1 starts half a period late (its first H2D after lane 0's), so
        // that from then on one lane's D2H meets the other's H2D, not its D2H
        if (i == 1) RS16_HIP(hipStreamWaitEvent(sl.s, e->hp_off, 0));
        RS16_HIP(hipMemcpyAsync(d_o, (const uint8_t*)h_original + i * original_stride, k * S, hipMemcpyHostToDevice,
                                sl.s));
        if (i == 0) RS16_HIP(hipEventRecord(e->hp_off, sl.s));
        if (int rc = encode_dev(e, high, k, m, S, d_o, d_r, (uint8_t*)sl.z.p, high ? nullptr : (uint8_t*)sl.u.p, sl.s,
                                err))
            return rc;
        RS16_HIP(hipMemcpyAsync((uint8_t*)h_recovery + i * recovery_stride, d_r, m * S, hipMemcpyDeviceToHost, sl.s));
    }
    for (auto& sl : e->hslot) RS16_HIP(hipStreamSynchronize(sl.s));
    if (int rc = e->scratch_done(e->stream, err)) return rc;
    return set_error(err, RS16_OK);
}

extern "C" int rs16_decode_host_batch(rs16_engine* e, size_t k, size_t m, size_t S, size_t nstripes,
                                      void* h_original, size_t original_stride, const uint8_t* original_received,
                                      size_t original_received_stride, const void* h_recovery,
                                      size_t recovery_stride, const uint8_t* recovery_received,
                                      size_t recovery_received_stride, rs16_error* err) {
    bool high;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    if (nstripes == 0) return set_error(err, RS16_OK);
    if (!h_original || !h_recovery || !original_received || !recovery_received || original_stride < k * S ||
        recovery_stride < m * S || original_received_stride < k || recovery_received_stride < m)
        return set_error(err, RS16_INVALID_ARGUMENT);
    // every stripe's counts first (src/rate/decoder_work.rs:120-139): a stripe
    // with too few shards fails the call before anything moves
    std::vector<size_t> ocnt(nstripes), rcnt(nstripes);
    for (size_t i = 0; i < nstripes; i++) {
        const uint8_t* fo = original_received + i * original_received_stride;
        const uint8_t* fr = recovery_received + i * recovery_received_stride;
        size_t o = 0, r = 0;
        for (size_t j = 0; j < k; j++) o += fo[j] != 0;
        for (size_t j = 0; j < m; j++) r += fr[j] != 0;
        if (o + r < k) return set_error(err, RS16_NOT_ENOUGH_SHARDS, k, o, r);
        ocnt[i] = o;
        rcnt[i] = r;
    }
    if (int rc = e->activate(err)) return rc;
    const DecodeGeom g0 = decode_geom(high, k, m);
    for (auto& sl : e->hslot) {
        RS16_HIP(sl.orig.reserve(k * S));
        RS16_HIP(sl.rec.reserve(m * S));
        RS16_HIP(sl.z.reserve((size_t)g0.n * S));
        RS16_HIP(sl.u.reserve((size_t)g0.n * S));
        RS16_HIP(sl.rcount.reserve(GF_ORDER / 64 * 8));
    }
    RS16_HIP(e->hflags.reserve(2 * (k + m)));
    RS16_HIP(e->hp_flags.reserve(2 * (k + m)));
    if (int rc = e->host_pipe_events(err)) return rc;
    if (int rc = e->host_slots(err)) return rc;
    auto& ev = e->hp_ev;
    int first_lane = -1;  // (lane offset: see rs16_encode_host_batch)
    bool offset_pending = true;
    for (size_t i = 0; i < nstripes; i++) {
        if (ocnt[i] == k) continue;  // nothing lost: nothing moves, nothing runs
        const int b = (int)(i & 1);
        if (first_lane >= 0 && offset_pending && b != first_lane) {
            RS16_HIP(hipStreamWaitEvent(e->hslot[b].s, e->hp_off, 0));
            offset_pending = false;
        }
        auto& sl = e->hslot[b];
        uint8_t* d_o = (uint8_t*)sl.orig.p;
        uint8_t* d_r = (uint8_t*)sl.rec.p;
        uint8_t* d_of = (uint8_t*)e->hflags.p + b * (k + m);
        uint8_t* d_rf = d_of + k;
        const uint8_t* fo = original_received + i * original_received_stride;
        const uint8_t* fr = recovery_received + i * recovery_received_stride;
        uint8_t* ho = (uint8_t*)h_original + i * original_stride;
        const uint8_t* hr = (const uint8_t*)h_recovery + i * recovery_stride;
        // ---- in: the flags (through page-locked staging: a pageable source
        // would make the copy synchronous; the lane's staging slot was last
        // read by its previous stripe's copy) and the received rows
        uint8_t* hf = (uint8_t*)e->hp_flags.p + b * (k + m);
        RS16_HIP(hipEventSynchronize(ev[b]));
        memcpy(hf, fo, k);
        memcpy(hf + k, fr, m);
        RS16_HIP(hipMemcpyAsync(d_of, hf, k + m, hipMemcpyHostToDevice, sl.s));
        RS16_HIP(hipEventRecord(ev[b], sl.s));
        if (int rc = copy_runs(fr, m, true, HP_MAX_RUNS, [&](size_t r0, size_t nr) -> int {
                RS16_HIP(hipMemcpyAsync(d_r + r0 * S, hr + r0 * S, nr * S, hipMemcpyHostToDevice, sl.s));
                return RS16_OK;
            }))
            return rc;
        if (int rc = copy_runs(fo, k, true, HP_MAX_RUNS, [&](size_t r0, size_t nr) -> int {
                RS16_HIP(hipMemcpyAsync(d_o + r0 * S, ho + r0 * S, nr * S, hipMemcpyHostToDevice, sl.s));
                return RS16_OK;
            }))
            return rc;
        if (first_lane < 0) {
            RS16_HIP(hipEventRecord(e->hp_off, sl.s));
            first_lane = b;
        }
        // ---- codec, with the lane's own eval_poly outputs
        {
            EvalSet lane(e, b);
            DecodeGeom g = g0;
            g.a_recv = high ? rcnt[i] : ocnt[i];
            g.b_recv = high ? ocnt[i] : rcnt[i];
            const uint8_t* fa = high ? d_rf : d_of;
            const uint8_t* fb = high ? d_of : d_rf;
            if (int rc = e->decode_eval(g, fa, fb, sl.s, err, S)) return rc;
            if (int rc = e->decode_passes(g, S, S, high ? d_r : d_o, fa, high ? d_o : d_r, fb, d_o, (uint8_t*)sl.z.p,
                                          (uint8_t*)sl.u.p, (uint32_t*)sl.rcount.p, sl.s, err))
                return rc;
        }
        // ---- out: the restored originals (in place in the lane's rows)
        if (int rc = copy_runs(fo, k, false, HP_MAX_RUNS, [&](size_t r0, size_t nr) -> int {
                RS16_HIP(hipMemcpyAsync(ho + r0 * S, d_o + r0 * S, nr * S, hipMemcpyDeviceToHost, sl.s));
                return RS16_OK;
            }))
            return rc;
    }
    for (auto& sl : e->hslot) RS16_HIP(hipStreamSynchronize(sl.s));
    if (int rc = e->scratch_done(e->stream, err)) return rc;
    e->forget_decode();  // (the counts came from the host flags: nothing for rs16_decode_check)
    return set_error(err, RS16_OK);
}

// ---------------------------------------------------------------------------
// Several GPUs in one process: the byte columns of one stripe are split over
// the engines (every 64-byte column block is an independent codeword,
// src/algorithm.md:18-32); each engine copies its column
// slice in with a pitched DMA copy, runs the device codec on it and copies
// it back, all engines concurrently.  No exchange between the GPUs.
// ---------------------------------------------------------------------------
// Column slice of engine j of n: rs16_column_slice (rs16_comm.cpp), the
// partition the RCCL scatter / gather and rs16/columns.py use.
static void multi_slice(size_t S, int n, int j, size_t* off, size_t* w) { (void)rs16_column_slice(S, n, j, off, w); }
static int multi_check(rs16_engine* const* engines, int n, rs16_error* err) {
    if (!engines || n < 1) return set_error(err, RS16_INVALID_ARGUMENT);
    for (int j = 0; j < n; j++)
        if (!engines[j]) return set_error(err, RS16_INVALID_ARGUMENT);
    return RS16_OK;
}
static int multi_sync(rs16_engine* const* engines, int n, rs16_error* err) {
    for (int j = 0; j < n; j++) {
        rs16_engine* e = engines[j];
        if (int rc = e->activate(err)) return rc;
        RS16_HIP(hipStreamSynchronize(e->stream));
        if (int rc = e->scratch_done(e->stream, err)) return rc;
    }
    return RS16_OK;
}

extern "C" int rs16_encode_host_multi(rs16_engine* const* engines, int n, size_t k, size_t m, size_t S,
                                      const void* h_original, void* h_recovery, rs16_error* err) {
    if (int rc = multi_check(engines, n, err)) return rc;
    bool high;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    const size_t wc = rs16_encoder_work_count(high, k, m);
    for (int j = 0; j < n; j++) {
        size_t off, w;
        multi_slice(S, n, j, &off, &w);
        if (w == 0) continue;
        rs16_engine* e = engines[j];
        if (int rc = e->activate(err)) return rc;
        if (int rc = e->order(e->stream, err)) return rc;
        auto& sl = e->hslot[0];
        RS16_HIP(sl.orig.reserve(k * w));
        RS16_HIP(sl.rec.reserve(m * w));
        RS16_HIP(sl.z.reserve(wc * w));
        if (!high) RS16_HIP(sl.u.reserve(next_pow2(k) * w));
        RS16_HIP(hipMemcpy2DAsync(sl.orig.p, w, (const uint8_t*)h_original + off, S, w, k, hipMemcpyHostToDevice,
                                  e->stream));
        if (int rc = encode_dev(e, high, k, m, w, (const uint8_t*)sl.orig.p, (uint8_t*)sl.rec.p, (uint8_t*)sl.z.p,
                                high ? nullptr : (uint8_t*)sl.u.p, e->stream, err))
            return rc;
        RS16_HIP(hipMemcpy2DAsync((uint8_t*)h_recovery + off, S, sl.rec.p, w, w, m, hipMemcpyDeviceToHost,
                                  e->stream));
    }
    if (int rc = multi_sync(engines, n, err)) return rc;
    return set_error(err, RS16_OK);
}

extern "C" int rs16_decode_host_multi(rs16_engine* const* engines, int n, size_t k, size_t m, size_t S,
                                      void* h_original, const uint8_t* original_received, const void* h_recovery,
                                      const uint8_t* recovery_received, rs16_error* err) {
    if (int rc = multi_check(engines, n, err)) return rc;
    bool high;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    size_t orig_recv = 0, rec_recv = 0;
    for (size_t i = 0; i < k; i++) orig_recv += original_received[i] != 0;
    for (size_t i = 0; i < m; i++) rec_recv += recovery_received[i] != 0;
    if (orig_recv + rec_recv < k) return set_error(err, RS16_NOT_ENOUGH_SHARDS, k, orig_recv, rec_recv);
    if (orig_recv == k) return set_error(err, RS16_OK);
    DecodeGeom g = decode_geom(high, k, m);
    g.a_recv = high ? rec_recv : orig_recv;
    g.b_recv = high ? orig_recv : rec_recv;
    for (int j = 0; j < n; j++) {
        size_t off, w;
        multi_slice(S, n, j, &off, &w);
        if (w == 0) continue;
        rs16_engine* e = engines[j];
        if (int rc = e->activate(err)) return rc;
        if (int rc = e->order(e->stream, err)) return rc;
        auto& sl = e->hslot[0];
        RS16_HIP(sl.orig.reserve(k * w));
        RS16_HIP(sl.rec.reserve(m * w));
        RS16_HIP(sl.z.reserve((size_t)g.n * w));
        RS16_HIP(sl.u.reserve((size_t)g.n * w));
        RS16_HIP(sl.rcount.reserve(GF_ORDER / 64 * 8));
        RS16_HIP(e->hflags.reserve(k + m));
        uint8_t* d_of = (uint8_t*)e->hflags.p;
        uint8_t* d_rf = d_of + k;
        RS16_HIP(hipMemcpyAsync(d_of, original_received, k, hipMemcpyHostToDevice, e->stream));
        RS16_HIP(hipMemcpyAsync(d_rf, recovery_received, m, hipMemcpyHostToDevice, e->stream));
        const uint8_t* fa = high ? d_rf : d_of;
        const uint8_t* fb = high ? d_of : d_rf;
        if (int rc = e->decode_eval(g, fa, fb, e->stream, err, w)) return rc;
        if (rec_recv)
            RS16_HIP(hipMemcpy2DAsync(sl.rec.p, w, (const uint8_t*)h_recovery + off, S, w, m, hipMemcpyHostToDevice,
                                      e->stream));
        if (orig_recv)
            RS16_HIP(hipMemcpy2DAsync(sl.orig.p, w, (const uint8_t*)h_original + off, S, w, k, hipMemcpyHostToDevice,
                                      e->stream));
        const uint8_t* o = (const uint8_t*)sl.orig.p;
        const uint8_t* r = (const uint8_t*)sl.rec.p;
        if (int rc = e->decode_passes(g, w, w, high ? r : o, fa, high ? o : r, fb, (uint8_t*)sl.orig.p,
                                      (uint8_t*)sl.z.p, (uint8_t*)sl.u.p, (uint32_t*)sl.rcount.p, e->stream, err))
            return rc;
        RS16_HIP(hipMemcpy2DAsync((uint8_t*)h_original + off, S, sl.orig.p, w, w, k, hipMemcpyDeviceToHost,
                                  e->stream));
    }
    if (int rc = multi_sync(engines, n, err)) return rc;
    for (int j = 0; j < n; j++) engines[j]->forget_decode();  // (host flags: nothing to check)
    return set_error(err, RS16_OK);
}

// A decode with nothing to restore (every original received) launches no
// kernel that counts the flags: the flags are copied, as they are at the
// decode's place in stream order, into the engine's ws_flags (segment A at
// 0, B at GF_ORDER), and rs16_decode_check counts that copy -- the caller may
// free or reuse its arrays after the call.  A NULL flag array counts as no
// received rows (the kernels read NULL flags as "none received" too).
static int note_flags_only(rs16_engine* e, const DecodeGeom& g, const uint8_t* fl_a, const uint8_t* fl_b,
                           void* stream, rs16_error* err) {
    e->forget_decode();
    if (int rc = e->activate(err)) return rc;
    hipStream_t s = e->pick(stream);
    if (int rc = e->order(s, err)) return rc;
    RS16_HIP(e->ws_flags.reserve(2 * (size_t)GF_ORDER));
    uint8_t* f = (uint8_t*)e->ws_flags.p;
    if (fl_a) RS16_HIP(hipMemcpyAsync(f, fl_a, g.a_count, hipMemcpyDeviceToDevice, s));
    else RS16_HIP(hipMemsetAsync(f, 0, g.a_count, s));
    if (fl_b) RS16_HIP(hipMemcpyAsync(f + GF_ORDER, fl_b, g.b_count, hipMemcpyDeviceToDevice, s));
    else RS16_HIP(hipMemsetAsync(f + GF_ORDER, 0, g.b_count, s));
    if (int rc = e->scratch_done(s, err)) return rc;
    e->last_dec = g;
    e->last_dec_flags_only = true;
    return set_error(err, RS16_OK);
}

// The passes of a device decode whose eval_poly is in ev_main (decode_eval
// on stream s or a preparation ordered before s), per column slice.
static int decode_device_passes(rs16_engine* e, const DecodeGeom& g, size_t S, void* d_original,
                                const void* d_recovery, const uint8_t* fl_a, const uint8_t* fl_b, int n, hipStream_t s,
                                rs16_error* err) {
    RS16_HIP(e->ws_z.reserve((size_t)g.n * S));
    RS16_HIP(e->ws_u.reserve((size_t)g.n * S));
    const uint8_t* orig = (const uint8_t*)d_original;
    const uint8_t* rec = (const uint8_t*)d_recovery;
    const uint8_t* seg_a = g.high ? rec : orig;
    const uint8_t* seg_b = g.high ? orig : rec;
    if (n == 1) {
        if (int rc = e->decode_passes(g, S, S, seg_a, fl_a, seg_b, fl_b, (uint8_t*)d_original, (uint8_t*)e->ws_z.p,
                                      (uint8_t*)e->ws_u.p, (uint32_t*)e->ev_main.rcount.p, s, err))
            return rc;
        if (int rc = e->scratch_done(s, err)) return rc;
        return set_error(err, RS16_OK);
    }
    if (int rc = e->fork(s, n, err)) return rc;
    const size_t blocks = S / 64;
    for (int j = 0, b0 = 0; j < n; j++) {
        const size_t b1 = blocks * (j + 1) / n, off = b0 * 64, w = (b1 - b0) * 64;
        // (decode_eval was told the slices are narrower than S: no column
        // decode evaluates the polynomial itself; with identity multipliers
        // the first slice's passes count the received rows)
        uint32_t* rc_j = j == 0 && e->e_ident ? (uint32_t*)e->ev_main.rcount.p : nullptr;
        if (int rc = e->decode_passes(g, w, S, seg_a + off, fl_a, seg_b + off, fl_b, (uint8_t*)d_original + off,
                                      (uint8_t*)e->ws_z.p + (size_t)g.n * off, (uint8_t*)e->ws_u.p + (size_t)g.n * off,
                                      rc_j, e->sl_stream[j], err))
            return rc;
        b0 = (int)b1;
    }
    if (int rc = e->join(s, n, err)) return rc;
    if (int rc = e->scratch_done(s, err)) return rc;
    return set_error(err, RS16_OK);
}

extern "C" int rs16_decode_device(rs16_engine* e, size_t k, size_t m, size_t S, void* d_original,
                                  const uint8_t* d_original_received, const void* d_recovery,
                                  const uint8_t* d_recovery_received, size_t orig_recv, size_t rec_recv, void* stream,
                                  rs16_error* err) {
    bool high;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    e->forget_decode();  // (whatever happens below, the previous decode is not checked again)
    if (orig_recv > k || rec_recv > m) return set_error(err, RS16_INVALID_ARGUMENT);
    if (orig_recv + rec_recv < k) return set_error(err, RS16_NOT_ENOUGH_SHARDS, k, orig_recv, rec_recv);
    DecodeGeom g = decode_geom(high, k, m);
    g.a_recv = high ? rec_recv : orig_recv;
    g.b_recv = high ? orig_recv : rec_recv;
    const uint8_t* fl_a = high ? d_recovery_received : d_original_received;
    const uint8_t* fl_b = high ? d_original_received : d_recovery_received;
    if (orig_recv == k) return note_flags_only(e, g, fl_a, fl_b, stream, err);
    if (int rc = e->activate(err)) return rc;
    hipStream_t s = e->pick(stream);
    if (int rc = e->order(s, err)) return rc;
    // erasure logs once, then the passes per column slice on the slice streams
    // (one slice: the column codec may compute them itself, decode_eval)
    const int n = e->slice_count(S);
    if (int rc = e->decode_eval(g, fl_a, fl_b, s, err, n == 1 ? S : 0)) return rc;
    return decode_device_passes(e, g, S, d_original, d_recovery, fl_a, fl_b, n, s, err);
}

// Split decode (include/rs16.h): the flag-dependent half of
// rs16_decode_device -- validation and eval_poly of the received pattern
// (src/rate/rate_high.rs:168-202, src/engine.rs:207-218) -- on one stream,
// the passes on another.  The received pattern of a decode is known before
// its shards are (a storage system knows which devices failed), so the
// erasure locator can be computed while the shards are still being produced
// or copied.  The preparation waits for the engine's earlier
// work (a previous decode still reads the eval outputs) but does not become
// the engine's last call: an encode issued after it on the engine stream runs
// concurrently with it.
extern "C" int rs16_decode_prepare(rs16_engine* e, size_t k, size_t m, size_t S, const uint8_t* d_original_received,
                                   const uint8_t* d_recovery_received, size_t orig_recv, size_t rec_recv,
                                   void* stream, rs16_error* err) {
    bool high;
    e->prep.valid = false;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    e->forget_decode();
    if (orig_recv > k || rec_recv > m) return set_error(err, RS16_INVALID_ARGUMENT);
    if (orig_recv + rec_recv < k) return set_error(err, RS16_NOT_ENOUGH_SHARDS, k, orig_recv, rec_recv);
    rs16_engine::Prepared p;
    p.k = k, p.m = m, p.S = S;
    p.g = decode_geom(high, k, m);
    p.g.a_recv = high ? rec_recv : orig_recv;
    p.g.b_recv = high ? orig_recv : rec_recv;
    p.fl_a = high ? d_recovery_received : d_original_received;
    p.fl_b = high ? d_original_received : d_recovery_received;
    p.nslices = e->slice_count(S);
    p.nothing = orig_recv == k;
    if (!p.nothing) {
        if (int rc = e->activate(err)) return rc;
        hipStream_t s = e->pick(stream);
        if (int rc = e->order(s, err)) return rc;
        if (int rc = e->guard_eval(s, false, err)) return rc;  // (an earlier, unconsumed preparation)
        e->preparing = true;
        const int rc = e->decode_eval(p.g, p.fl_a, p.fl_b, s, err, p.nslices == 1 ? S : 0);
        e->preparing = false;
        if (rc) return rc;
        if (!e->prep_ev) RS16_HIP(hipEventCreateWithFlags(&e->prep_ev, hipEventDisableTiming));
        RS16_HIP(hipEventRecord(e->prep_ev, s));
        e->prep_pending = true;
    }
    p.valid = true;
    e->prep = p;
    return set_error(err, RS16_OK);
}

extern "C" int rs16_decode_device_prepared(rs16_engine* e, size_t k, size_t m, size_t S, void* d_original,
                                           const void* d_recovery, void* stream, rs16_error* err) {
    const rs16_engine::Prepared p = e->prep;
    if (!p.valid || p.k != k || p.m != m || p.S != S) return set_error(err, RS16_INVALID_ARGUMENT);
    e->prep.valid = false;
    if (p.nothing) return note_flags_only(e, p.g, p.fl_a, p.fl_b, stream, err);
    if (int rc = e->activate(err)) return rc;
    hipStream_t s = e->pick(stream);
    if (int rc = e->order(s, err)) return rc;
    if (int rc = e->guard_eval(s, true, err)) return rc;  // after the preparation's eval_poly
    return decode_device_passes(e, p.g, S, d_original, d_recovery, p.fl_a, p.fl_b, p.nslices, s, err);
}

// rs16_decode_device for nstripes independent stripes that lost the same
// shards (one failed device holds the same shard index of every stripe):
// one eval_poly from the shared flags, every pass launch covering all
// stripes; stripe i's originals at d_original + i original_stride (restored
// in place), its recovery at d_recovery + i recovery_stride.
extern "C" int rs16_decode_device_batch(rs16_engine* e, size_t k, size_t m, size_t S, size_t nstripes,
                                        void* d_original, size_t original_stride, const uint8_t* d_original_received,
                                        const void* d_recovery, size_t recovery_stride,
                                        const uint8_t* d_recovery_received, size_t orig_recv, size_t rec_recv,
                                        void* stream, rs16_error* err) {
    bool high;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    e->forget_decode();
    if (orig_recv > k || rec_recv > m) return set_error(err, RS16_INVALID_ARGUMENT);
    if (orig_recv + rec_recv < k) return set_error(err, RS16_NOT_ENOUGH_SHARDS, k, orig_recv, rec_recv);
    if (nstripes == 0) return set_error(err, RS16_OK);
    if (orig_recv == k) {
        DecodeGeom g0 = decode_geom(high, k, m);
        g0.a_recv = high ? rec_recv : orig_recv;
        g0.b_recv = high ? orig_recv : rec_recv;
        return note_flags_only(e, g0, high ? d_recovery_received : d_original_received,
                               high ? d_original_received : d_recovery_received, stream, err);
    }
    if (!d_original || !d_recovery || original_stride < k * S || recovery_stride < m * S || original_stride % 64 ||
        recovery_stride % 64 || nstripes > ((size_t)1 << 20))
        return set_error(err, RS16_INVALID_ARGUMENT);
    if (int rc = e->activate(err)) return rc;
    hipStream_t s = e->pick(stream);
    if (int rc = e->order(s, err)) return rc;
    DecodeGeom g = decode_geom(high, k, m);
    g.a_recv = high ? rec_recv : orig_recv;
    g.b_recv = high ? orig_recv : rec_recv;
    RS16_HIP(e->ws_z.reserve(nstripes * g.n * S));
    RS16_HIP(e->ws_u.reserve(nstripes * g.n * S));
    const uint8_t* orig = (const uint8_t*)d_original;
    const uint8_t* rec = (const uint8_t*)d_recovery;
    const uint8_t* seg_a = high ? rec : orig;
    const uint8_t* seg_b = high ? orig : rec;
    const size_t bs_a = high ? recovery_stride : original_stride, bs_b = high ? original_stride : recovery_stride;
    const uint8_t* fl_a = high ? d_recovery_received : d_original_received;
    const uint8_t* fl_b = high ? d_original_received : d_recovery_received;
    if (int rc = e->decode_eval(g, fl_a, fl_b, s, err, S, nstripes)) return rc;
    if (int rc = e->decode_passes(g, S, S, seg_a, fl_a, seg_b, fl_b, (uint8_t*)d_original, (uint8_t*)e->ws_z.p,
                                  (uint8_t*)e->ws_u.p, (uint32_t*)e->evset->rcount.p, s, err, nstripes, bs_a, bs_b,
                                  original_stride))
        return rc;
    if (int rc = e->scratch_done(s, err)) return rc;
    return set_error(err, RS16_OK);
}

// rs16_decode_device for `nstripes` independent stripes, each with its own
// received set (reed_solomon_16::decode, src/lib.rs:287-344, once per stripe;
// src/rate/decoder_work.rs:62-139 counts every call's own received shards):
// stripe i's flags at d_*_received + i * *_received_stride bytes, its counts
// in the host arrays.  One launch of the eval kernels with a grid row per
// stripe (per-stripe erasure logs, received bitmaps, zero tiles, lost
// ranges), then the pass launches shared by all stripes, each workgroup
// reading its stripe's metadata.  Stripes go in groups of at most 256 (the
// scratch is sized for one group).  Path, per group: the half-transform
// decode when no stripe of it received an original, else the general decode
// for all of them; the first-pass tiles launched are the union over the
// group's stripes.
extern "C" int rs16_decode_device_batch_varied(rs16_engine* e, size_t k, size_t m, size_t S, size_t nstripes,
                                               void* d_original, size_t original_stride,
                                               const uint8_t* d_original_received, size_t original_received_stride,
                                               const void* d_recovery, size_t recovery_stride,
                                               const uint8_t* d_recovery_received, size_t recovery_received_stride,
                                               const size_t* original_received_counts,
                                               const size_t* recovery_received_counts, void* stream, rs16_error* err) {
    bool high;
    if (int rc = resolve_rate(RS16_RATE_DEFAULT, k, m, S, &high, err)) return rc;
    e->forget_decode();
    if (nstripes == 0) return set_error(err, RS16_OK);
    if (!d_original || !d_recovery || !d_original_received || !d_recovery_received || !original_received_counts ||
        !recovery_received_counts || original_stride < k * S || recovery_stride < m * S || original_stride % 64 ||
        recovery_stride % 64 || original_received_stride < k || recovery_received_stride < m ||
        nstripes > ((size_t)1 << 16))
        return set_error(err, RS16_INVALID_ARGUMENT);
    for (size_t i = 0; i < nstripes; i++) {
        const size_t o = original_received_counts[i], r = recovery_received_counts[i];
        if (o > k || r > m) return set_error(err, RS16_INVALID_ARGUMENT);
        if (o + r < k) return set_error(err, RS16_NOT_ENOUGH_SHARDS, k, o, r);  // (the first such stripe)
    }
    if (int rc = e->activate(err)) return rc;
    hipStream_t s = e->pick(stream);
    if (int rc = e->order(s, err)) return rc;
    const uint8_t* rec = (const uint8_t*)d_recovery;
    const size_t bs_a = high ? recovery_stride : original_stride, bs_b = high ? original_stride : recovery_stride;
    const size_t fs_a = high ? recovery_received_stride : original_received_stride;
    const size_t fs_b = high ? original_received_stride : recovery_received_stride;
    // Groups of at most VARY_GROUP stripes: the per-stripe metadata (erasure
    // logs, received bitmaps, ... 0.5 MiB a stripe) and the work rows (2 n S
    // bytes a stripe) are reserved for one group, not for the whole call.
    constexpr size_t VARY_GROUP = 256;
    for (size_t g0 = 0; g0 < nstripes; g0 += VARY_GROUP) {
        const size_t ns = std::min(VARY_GROUP, nstripes - g0);
        size_t max_o = 0, max_r = 0;
        bool any_lost = false;
        for (size_t i = g0; i < g0 + ns; i++) {
            max_o = std::max(max_o, original_received_counts[i]);
            max_r = std::max(max_r, recovery_received_counts[i]);
            any_lost |= original_received_counts[i] < k;
        }
        if (!any_lost) continue;  // nothing to restore in any stripe of the group
        DecodeGeom g = decode_geom(high, k, m);
        // (a segment counts as received when any stripe received a shard of it)
        g.a_recv = high ? max_r : max_o;
        g.b_recv = high ? max_o : max_r;
        RS16_HIP(e->ws_z.reserve(ns * g.n * S));
        RS16_HIP(e->ws_u.reserve(ns * g.n * S));
        uint8_t* og = (uint8_t*)d_original + g0 * original_stride;
        const uint8_t* rg = rec + g0 * recovery_stride;
        const uint8_t* seg_a = high ? rg : og;
        const uint8_t* seg_b = high ? og : rg;
        const uint8_t* fl_a = (high ? d_recovery_received : d_original_received) + g0 * fs_a;
        const uint8_t* fl_b = (high ? d_original_received : d_recovery_received) + g0 * fs_b;
        const uint32_t vary = ns > 1 ? (uint32_t)ns : 0;
        if (int rc = e->decode_eval(g, fl_a, fl_b, s, err, S, ns, vary, fs_a, fs_b)) return rc;
        if (int rc = e->decode_passes(g, S, S, seg_a, fl_a, seg_b, fl_b, og, (uint8_t*)e->ws_z.p, (uint8_t*)e->ws_u.p,
                                      (uint32_t*)e->evset->rcount.p, s, err, ns, bs_a, bs_b, original_stride))
            return rc;
    }
    e->forget_decode();
    if (int rc = e->scratch_done(s, err)) return rc;
    return set_error(err, RS16_OK);
}

// ---------------------------------------------------------------------------
// Device memory helpers.
// ---------------------------------------------------------------------------
extern "C" void* rs16_device_alloc(rs16_engine* e, size_t bytes, rs16_error* err) {
    if (e->activate(err)) return nullptr;
    void* p = nullptr;
    hipError_t he = hipMalloc(&p, bytes ? bytes : 1);
    if (he != hipSuccess) return hip_fail(err, he), nullptr;
    set_error(err, RS16_OK);
    return p;
}
extern "C" void rs16_device_free(rs16_engine* e, void* p) {
    if (!e || !p) return;
    (void)hipSetDevice(e->device);
    (void)hipFree(p);
}
extern "C" void* rs16_stream_create(rs16_engine* e, rs16_error* err) {
    if (e->activate(err)) return nullptr;
    hipStream_t st = nullptr;
    hipError_t he = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (he != hipSuccess) return hip_fail(err, he), nullptr;
    set_error(err, RS16_OK);
    return (void*)st;
}
extern "C" void rs16_stream_destroy(rs16_engine* e, void* st) {
    if (!e || !st) return;
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize((hipStream_t)st);
    (void)hipStreamDestroy((hipStream_t)st);
}
extern "C" void* rs16_host_alloc(rs16_engine* e, size_t bytes, rs16_error* err) {
    if (e->activate(err)) return nullptr;
    void* p = nullptr;
    hipError_t he = hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable);
    if (he != hipSuccess) return hip_fail(err, he), nullptr;
    set_error(err, RS16_OK);
    return p;
}
extern "C" void rs16_host_free(rs16_engine* e, void* p) {
    if (!e || !p) return;
    (void)hipSetDevice(e->device);
    (void)hipHostFree(p);
}
extern "C" int rs16_memcpy_htod(rs16_engine* e, void* dst, const void* src, size_t bytes, void* stream,
                                rs16_error* err) {
    if (int rc = e->activate(err)) return rc;
    hipStream_t s = e->pick(stream);
    RS16_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    RS16_HIP(hipStreamSynchronize(s));
    return set_error(err, RS16_OK);
}
extern "C" int rs16_memcpy_dtoh(rs16_engine* e, void* dst, const void* src, size_t bytes, void* stream,
                                rs16_error* err) {
    if (int rc = e->activate(err)) return rc;
    hipStream_t s = e->pick(stream);
    RS16_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    RS16_HIP(hipStreamSynchronize(s));
    return set_error(err, RS16_OK);
}
extern "C" int rs16_memset_device(rs16_engine* e, void* dst, int value, size_t bytes, void* stream, rs16_error* err) {
    if (int rc = e->activate(err)) return rc;
    RS16_HIP(hipMemsetAsync(dst, value, bytes, e->pick(stream)));
    return set_error(err, RS16_OK);
}
