// rs16_engine.cpp -- engine object: tables in HBM, engine-level transforms
// as HBM passes, and the fused encode/decode pass sequences.
#include <cstdlib>
#include "rs16_engine.hpp"

#include <algorithm>
#include <cstring>

namespace rs16 {

hipError_t DevBuf::reserve(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) cap = bytes;
    return e;
}
void DevBuf::release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
}

hipError_t HostBuf::reserve(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocPortable);
    if (e == hipSuccess) cap = bytes;
    return e;
}
void HostBuf::release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
}

hipError_t Pending::record(hipStream_t s) {
    if (!ev) {
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    hipError_t e = hipEventRecord(ev, s);
    busy = e == hipSuccess;
    return e;
}
hipError_t Pending::wait() {
    if (!busy) return hipSuccess;
    busy = false;
    return hipEventSynchronize(ev);
}
void Pending::release() {
    if (ev) (void)hipEventDestroy(ev);
    ev = nullptr;
    busy = false;
}

int set_error(rs16_error* err, int code, uint64_t v0, uint64_t v1, uint64_t v2) {
    if (err) {
        err->code = code;
        err->v0 = v0;
        err->v1 = v1;
        err->v2 = v2;
    }
    return code;
}
int hip_fail(rs16_error* err, hipError_t e) { return set_error(err, RS16_DEVICE_ERROR, (uint64_t)e); }

size_t next_pow2(size_t x) {
    size_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

DecodeGeom decode_geom(bool high, size_t k, size_t m) {
    DecodeGeom g;
    g.high = high;
    g.a_count = (uint32_t)(high ? m : k);
    g.b_count = (uint32_t)(high ? k : m);
    g.chunk = (uint32_t)next_pow2(g.a_count);
    g.n = (uint32_t)next_pow2((size_t)g.chunk + g.b_count);
    return g;
}

static PassArgs base_args(const rs16_engine* e, size_t S) {
    PassArgs a;
    std::memset(&a, 0, sizeof a);
    a.skew_tab = e->d_skew_tab;
    a.mul_tab = e->d_mul_tab;
    a.zero = e->d_zero_sink;
    a.S_in = a.S_out = a.S_seg = a.S_rest = S;
    a.qrow = (uint32_t)(S / 8);
    a.diag = (uint32_t)e->diag;
    return a;
}

}  // namespace rs16

using namespace rs16;

int rs16_engine::activate(rs16_error* err) {
    RS16_HIP(hipSetDevice(device));
    return RS16_OK;
}

int rs16_engine::slice_count(size_t S) const {
    const int n = slices;
    return (int)std::max<size_t>(1, std::min<size_t>(std::min(n, MAX_SLICES), S / 64));
}

// Slice 0 runs on the caller's stream s itself; slices 1.. on sl_stream[1..]
// (sl_stream[0] = s while a sliced call is being issued).
int rs16_engine::fork(hipStream_t s, int n, rs16_error* err) {
    if (!sl_fork) RS16_HIP(hipEventCreateWithFlags(&sl_fork, hipEventDisableTiming));
    if (n > 1) RS16_HIP(hipEventRecord(sl_fork, s));
    for (int j = 1; j < n; j++) {
        if (!sl_own[j]) RS16_HIP(hipStreamCreateWithFlags(&sl_own[j], hipStreamNonBlocking));
        RS16_HIP(hipStreamWaitEvent(sl_own[j], sl_fork, 0));
    }
    sl_stream[0] = s;
    for (int j = 1; j < MAX_SLICES; j++) sl_stream[j] = sl_own[j];
    return RS16_OK;
}

int rs16_engine::join(hipStream_t s, int n, rs16_error* err) {
    for (int j = 1; j < n; j++) {
        if (!sl_join[j]) RS16_HIP(hipEventCreateWithFlags(&sl_join[j], hipEventDisableTiming));
        RS16_HIP(hipEventRecord(sl_join[j], sl_own[j]));
        RS16_HIP(hipStreamWaitEvent(s, sl_join[j], 0));
    }
    return RS16_OK;
}

int rs16_engine::order(hipStream_t s, rs16_error* err) {
    if (last == LAST_ENGINE && s != stream) {
        if (!order_ev) RS16_HIP(hipEventCreateWithFlags(&order_ev, hipEventDisableTiming));
        RS16_HIP(hipEventRecord(order_ev, stream));
        RS16_HIP(hipStreamWaitEvent(s, order_ev, 0));
    } else if (last == LAST_CALLER) {
        RS16_HIP(hipStreamWaitEvent(s, order_ev, 0));  // (recorded by scratch_done)
    }
    return RS16_OK;
}

int rs16_engine::scratch_done(hipStream_t s, rs16_error* err) {
    if (s == stream) {
        last = LAST_ENGINE;
        return RS16_OK;
    }
    if (!order_ev) RS16_HIP(hipEventCreateWithFlags(&order_ev, hipEventDisableTiming));
    RS16_HIP(hipEventRecord(order_ev, s));
    last = LAST_CALLER;
    return RS16_OK;
}

int rs16_engine::prof_begin(hipStream_t s, hipEvent_t* ev, rs16_error* err) {
    *ev = nullptr;
    if (!profiling) return RS16_OK;
    if (ev_pool.empty()) {
        hipEvent_t e;
        RS16_HIP(hipEventCreate(&e));
        ev_pool.push_back(e);
    }
    *ev = ev_pool.back();
    ev_pool.pop_back();
    RS16_HIP(hipEventRecord(*ev, s));
    return RS16_OK;
}

int rs16_engine::prof_end(int id, hipStream_t s, hipEvent_t ev, rs16_error* err) {
    if (!ev) return RS16_OK;
    if (ev_pool.empty()) {
        hipEvent_t e;
        RS16_HIP(hipEventCreate(&e));
        ev_pool.push_back(e);
    }
    hipEvent_t b = ev_pool.back();
    ev_pool.pop_back();
    RS16_HIP(hipEventRecord(b, s));
    prof_pending.push_back({id, ev, b});
    if (prof_pending.size() > 4096) return prof_collect(err);  // bound the event pool
    return RS16_OK;
}

int rs16_engine::prof_collect(rs16_error* err) {
    for (const ProfRec& r : prof_pending) {
        RS16_HIP(hipEventSynchronize(r.b));
        float ms = 0.f;
        RS16_HIP(hipEventElapsedTime(&ms, r.a, r.b));
        prof_ms[r.id] += ms;
        prof_n[r.id] += 1;
        ev_pool.push_back(r.a);
        ev_pool.push_back(r.b);
    }
    prof_pending.clear();
    return RS16_OK;
}

int rs16_engine::pass(int prog, int T, const PassArgs& a, uint32_t tiles, hipStream_t s, rs16_error* err, int prof) {
    hipEvent_t ev;
    if (prof < 0) prof = prog;
    if (int rc = prof_begin(s, &ev, err)) return rc;
    if (stamp_buf && prof == stamp_prof) {
        PassArgs b = a;
        b.stamps = (uint64_t*)stamp_buf;
        RS16_HIP(launch_pass(prog, T, b, tiles, s));
    } else {
        RS16_HIP(launch_pass(prog, T, a, tiles, s));
    }
    return prof_end(prof, s, ev, err);
}

bool rs16_engine::col_ok(int L, size_t S, size_t nstripes, bool gen) const {
    const bool rows = col_rows_ok((uint32_t)L) || (gen && L == (int)COL_LGEN);
    if (!rows || (diag & DIAG_NO_COLUMN)) return false;
    return (S / 8) * nstripes <= col_max_quads || (diag & DIAG_FORCE_COLUMN);
}

// the radix-2 multi-chunk encodes (launch_col, COL_ENC_IFFT / COL_ENC_FFTX /
// COL_ENC with nch > 1): 2^8 .. 2^10-row chunks, 2 or more of them and at
// most col_max_chunk_rows rows (the high rate's 256 / 512-row chunks: up to
// 8192 rows, which still beat the passes there: 8000:300 30.1 against 33.7
// us, 8000:200 34.0 against 40.9, profiles/r04_probe_chunks.txt)
bool rs16_engine::col_chunks_ok(int L, uint32_t nch, size_t S, bool high) const {
    const size_t rows_max = high && L <= 9 ? std::max<size_t>(col_max_chunk_rows, 8192) : col_max_chunk_rows;
    return L >= (int)COL_LCHUNK && L <= (int)COL_LMAX && nch > 1 && nch <= COL_MAX_CHUNKS &&
           (((size_t)nch << L) <= rows_max || (diag & DIAG_FORCE_COLUMN)) &&
           nch < col_img_count((uint32_t)L) && col_ok(L, S, 1);
}

ColArgs rs16_engine::col_args() const {
    ColArgs a;
    std::memset(&a, 0, sizeof a);
    a.skew_tab = d_skew_tab;
    a.mul_tab = d_mul_tab;
    a.zero = d_zero_sink;
    a.elog = (const uint32_t*)evset->elog.p;
    a.nstripes = 1;
    a.diag = (uint32_t)diag;
    return a;
}

// The column codec's tables (HostTables::col_img / col_v), uploaded on the
// engine's first column launch: engines that never run it allocate nothing.
int rs16_engine::col_tables(hipStream_t s, rs16_error* err) {
    if (d_col_img) return RS16_OK;
    const HostTables& t = host_tables();
    uint32_t *img = nullptr, *v = nullptr;
    RS16_HIP(hipMalloc(&img, COL_IMG_DWORDS * 4));
    if (hipError_t e = hipMalloc(&v, t.col_v.size() * 4)) {
        (void)hipFree(img);
        return hip_fail(err, e);
    }
    hipError_t e = hipMemcpyAsync(img, t.col_img.data(), COL_IMG_DWORDS * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(v, t.col_v.data(), t.col_v.size() * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // (pageable sources: keep no pending copy)
    if (e != hipSuccess) {
        (void)hipFree(img);
        (void)hipFree(v);
        return hip_fail(err, e);
    }
    d_col_img = img;
    d_col_v = v;
    return RS16_OK;
}

int rs16_engine::col(const ColArgs& args, int L, int mode, hipStream_t s, rs16_error* err) {
    const bool dec = mode == COL_DEC_EWORK || mode == COL_DEC_EVAL || mode == COL_DEC_GEN;
    if (int rc = col_tables(s, err)) return rc;
    // the table images of the two transforms (skew deltas 0 / 2^L; the
    // kernel adds the chunk index of a multi-chunk encode to the delta)
    ColArgs a = args;
    const uint32_t N = 1u << L;
    if ((a.skew_ifft != 0 && a.skew_ifft != N) || (a.skew_fft != 0 && a.skew_fft != N) ||
        (a.nch > 1 && a.nch >= col_img_count((uint32_t)L)))
        return hip_fail(err, hipErrorInvalidValue);  // (unreachable: every caller passes 0 or 2^L)
    a.img_ifft = (const uint8_t*)(d_col_img + col_img_offset((uint32_t)L, a.skew_ifft ? 1 : 0));
    a.img_fft = (const uint8_t*)(d_col_img + col_img_offset((uint32_t)L, a.skew_fft ? 1 : 0));
    if (mode == COL_DEC_EVAL) a.vtab = d_col_v + col_v_offset(2u << L);  // (2^(L+1) work rows)
    if (mode == COL_DEC_GEN) a.vtab = d_col_v + col_v_offset(1u << L);   // (2^L work rows)
    hipEvent_t ev;
    const int prof = dec ? PROF_COL_DEC : PROF_COL_ENC;
    if (int rc = prof_begin(s, &ev, err)) return rc;
    if (stamp_buf && stamp_prof == prof) {
        ColArgs b = a;
        b.stamps = (uint64_t*)stamp_buf;
        RS16_HIP(launch_col(b, (uint32_t)L, mode, s));
    } else {
        RS16_HIP(launch_col(a, (uint32_t)L, mode, s));
    }
    return prof_end(prof, s, ev, err);
}

// The multi-chunk encodes of 128-row chunks in one launch (colm_kernel,
// rs16_col.hip): nch chunks of originals (high) or of recovery (low).
int rs16_engine::col_multi(size_t k, size_t m, size_t S, size_t S_user, const uint8_t* d_orig, uint8_t* d_rec,
                           uint32_t nch, bool high, hipStream_t s, rs16_error* err) {
    ColArgs c = col_args();
    c.in = d_orig;
    c.out = d_rec;
    c.S_in = c.S_out = S_user;
    c.qrow = (uint32_t)(S / 8);
    c.in_rows = (uint32_t)k;
    c.out_rows = (uint32_t)m;
    c.nch = nch;
    hipEvent_t ev;
    if (int rc = prof_begin(s, &ev, err)) return rc;
    RS16_HIP(launch_col_multi(c, high, s));
    return prof_end(PROF_COL_ENC, s, ev, err);
}

// Engine::fft over 2^L rows: L <= 8 in one pass; otherwise the high
// (L - L/2) row bits as a strided pass, then the low L/2 bits contiguous.
int rs16_engine::fft(uint8_t* data, size_t S, size_t pos, size_t size, size_t skew_delta, hipStream_t s,
                     rs16_error* err) {
    const int L = ilog2(size);
    if (L == 0) return RS16_OK;
    PassArgs a = base_args(this, S);
    a.in = a.out = data + pos * S;
    a.skew_fft = (uint32_t)skew_delta;
    if (L <= 8) {
        RS16_PASS(GEN_FFT, L, a, 1, s);
        return RS16_OK;
    }
    const int lo = L / 2, hi = L - lo;
    a.lo = lo;
    RS16_PASS(GEN_FFT, hi, a, 1u << lo, s);
    a.lo = 0;
    RS16_PASS(GEN_FFT, lo, a, 1u << hi, s);
    return RS16_OK;
}

int rs16_engine::ifft(uint8_t* data, size_t S, size_t pos, size_t size, size_t skew_delta, hipStream_t s,
                      rs16_error* err) {
    const int L = ilog2(size);
    if (L == 0) return RS16_OK;
    PassArgs a = base_args(this, S);
    a.in = a.out = data + pos * S;
    a.skew_ifft = (uint32_t)skew_delta;
    if (L <= 8) {
        RS16_PASS(GEN_IFFT, L, a, 1, s);
        return RS16_OK;
    }
    const int lo = L / 2, hi = L - lo;
    a.lo = 0;
    RS16_PASS(GEN_IFFT, lo, a, 1u << hi, s);
    a.lo = lo;
    RS16_PASS(GEN_IFFT, hi, a, 1u << lo, s);
    return RS16_OK;
}

// HighRateEncoder::encode for original_count <= chunk (src/rate/rate_high.rs:44-83):
//   recovery = FFT(IFFT(originals zero-padded to chunk, skew = chunk), skew = 0)[0..m)
// as three passes over the 2-D row factorisation (contiguous low bits /
// strided high bits); IFFT-high and FFT-high share the strided pass.
int rs16_engine::encode_high_fused(size_t k, size_t m, size_t S, size_t S_user, const uint8_t* d_orig, uint8_t* d_rec, uint8_t* Z,
                                   hipStream_t s, rs16_error* err, size_t nst, size_t bs_orig, size_t bs_rec) {
    const size_t chunk = next_pow2(m);
    const int L = ilog2(chunk);
    PassArgs a = base_args(this, S);
    a.seg_a = d_orig;
    a.S_seg = S_user;
    a.a_count = (uint32_t)k;
    a.skew_ifft = (uint32_t)chunk;
    a.skew_fft = 0;
    a.out_rows = (uint32_t)m;
    // nst > 1: independent stripes batched in each launch (PassArgs::stripe_tiles);
    // stripe i's originals / recovery at d_orig / d_rec + i bs_orig / bs_rec,
    // its work rows at Z + i chunk S
    const uint32_t ns = (uint32_t)nst;
    auto batch = [&](uint32_t tiles, size_t bs_in, size_t bs_out, size_t bs_seg) {
        a.stripe_tiles = ns > 1 ? tiles : 0;
        a.bs_in = bs_in;
        a.bs_out = bs_out;
        a.bs_seg = bs_seg;
        return tiles * ns;
    };
    if (col_ok(L, S, nst)) {
        // 512 / 1024-row chunks: the whole encode in one launch (rs16_col.hip)
        ColArgs c = col_args();
        c.in = d_orig;
        c.out = d_rec;
        c.S_in = c.S_out = S_user;
        c.qrow = (uint32_t)(S / 8);
        c.nstripes = ns;
        c.bs_in = bs_orig;
        c.bs_out = bs_rec;
        c.in_rows = (uint32_t)k;
        c.out_rows = (uint32_t)m;
        c.skew_ifft = (uint32_t)chunk;
        c.skew_fft = 0;
        return col(c, L, COL_ENC, s, err);
    }
    if (L <= 8) {
        a.out = d_rec;
        a.S_out = S_user;
        RS16_PASS(ENC_SINGLE, L, a, batch(1, 0, bs_rec, bs_orig), s);
        return RS16_OK;
    }
    // odd L: the extra row bit goes to the strided two-direction pass (an
    // 8 / 7 / 8 split measured 2-3 us slower per encode, CHANGELOG.md round 3)
    const int lo = L / 2, hi = L - lo;
    const size_t zs = chunk * S;
    a.out = Z;
    a.lo = 0;
    RS16_PASS(ENC_FIRST, lo, a, batch(1u << hi, 0, zs, bs_orig), s);
    a.in = Z;
    a.lo = lo;
    RS16_PASS(ENC_MID, hi, a, batch(1u << lo, zs, zs, 0), s);
    a.in = Z;
    a.out = d_rec;
    a.S_out = S_user;
    a.lo = 0;
    const uint32_t tiles = (uint32_t)((m + ((size_t)1 << lo) - 1) >> lo);
    RS16_PASS(ENC_LAST, lo, a, batch(tiles, zs, bs_rec, 0), s);
    return RS16_OK;
}

// {High,Low}RateDecoder::decode (src/rate/rate_high.rs:168-247,
// src/rate/rate_low.rs:168-247), all in HBM:
//   e     = eval_poly(erasure vector)                       (3 small kernels)
//   z     = IFFT_low(received * e)                          (pass 1, contiguous)
//   u     = FFT_high((I + H) IFFT_high(z))                  (pass 2, strided)
//   y     = u + L z,  out = reveal(FFT_low(y))              (pass 3, contiguous)
// where the formal derivative FD = I + L + H is split into its low-bit part L
// and high-bit part H (L commutes with the high-bit layers and
// FFT_high o IFFT_high = I), so no separate derivative pass is needed.
int rs16_engine::decode_fused(const DecodeGeom& g, size_t S, size_t S_user, const uint8_t* seg_a, const uint8_t* flags_a,
                              const uint8_t* seg_b, const uint8_t* flags_b, uint8_t* rest, uint8_t* Z, uint8_t* U,
                              hipStream_t s, rs16_error* err) {
    if (int rc = decode_eval(g, flags_a, flags_b, s, err, S)) return rc;
    return decode_passes(g, S, S_user, seg_a, flags_a, seg_b, flags_b, rest, Z, U, (uint32_t*)evset->rcount.p, s, err);
}

int rs16_engine::guard_eval(hipStream_t s, bool consume, rs16_error* err) {
    if (!prep_pending) return RS16_OK;
    RS16_HIP(hipStreamWaitEvent(s, prep_ev, 0));
    prep_pending = false;
    if (!consume) prep.valid = false;
    return RS16_OK;
}

// Erasure logs e = eval_poly(erasure vector) into evset->elog (2-3 small kernels).
int rs16_engine::decode_eval(const DecodeGeom& g, const uint8_t* flags_a, const uint8_t* flags_b, hipStream_t s,
                             rs16_error* err, size_t S, size_t nstripes, uint32_t vary, size_t bs_fa, size_t bs_fb) {
    // (a prepared decode's outputs in ev_main are about to be overwritten)
    if (evset == &ev_main && !preparing)
        if (int rc = guard_eval(s, false, err)) return rc;
    // Any evaluation other than the preparation itself also overwrites the
    // path state below (e_ident, elog_fused, eval_in_col, var_ns) that a
    // prepared decode reads -- whichever eval set it writes to (the
    // pipelined host path's lanes use their own): the preparation is gone.
    if (!preparing) prep.valid = false;
    const size_t nv = vary > 1 ? vary : 1;
    RS16_HIP(evset->work32.reserve(nv * VARY_WORK * 4));
    RS16_HIP(evset->elog.reserve(nv * VARY_WORK * 4));
    RS16_HIP(evset->zflag.reserve(nv * VARY_ZFLAGS));
    RS16_HIP(evset->rbits.reserve(nv * VARY_RBITS * 4));
    RS16_HIP(evset->lost.reserve(nv * VARY_LOST * 4));
    RS16_HIP(evset->rcount.reserve(GF_ORDER / 64 * 8));
    var_ns = vary > 1 ? vary : 0;
    var_bs_fa = vary > 1 ? bs_fa : 0;
    var_bs_fb = vary > 1 ? bs_fb : 0;
    ErasureSpec es{};
    es.flags_a = flags_a;
    es.flags_b = flags_b;
    es.a_count = g.a_count;
    es.chunk = g.chunk;
    es.b_count = g.b_count;
    es.pad_fill = g.high ? 1 : 0;
    es.tail_fill = g.high ? 0 : 1;
    // the pass metadata: received bitmap, and zero flags of the first pass's
    // tiles (2^lo rows, lo = L/2) when the decode takes more than one pass
    const int L = ilog2(g.n);
    es.rbits = (uint32_t*)evset->rbits.p;
    es.zflags = L > 8 ? (uint8_t*)evset->zflag.p : nullptr;
    es.n = g.n;
    es.zlo = (uint32_t)(L / 2);
    // the lost originals' row range prunes the general multi-pass decode
    // (the half-transform decode restores every original: not needed)
    const bool prune = !half_decode(g) && L > 8;
    es.lostpart = prune ? (uint32_t*)evset->lost.p : nullptr;
    es.lostrange = prune ? (uint32_t*)evset->lost.p + 512 : nullptr;
    es.orig_b = g.high ? 1 : 0;
    es.rcount = (uint32_t*)evset->rcount.p;
    es.diag = (uint32_t)diag;
    last_dec = g;
    last_dec_valid = true;
    if (var_ns) {
        // every stripe's own metadata; no received counts (rs16_decode_check
        // covers the single-pattern calls)
        es.nstripes = var_ns;
        es.bs_fa = var_bs_fa;
        es.bs_fb = var_bs_fb;
        es.bs_work = es.bs_elog = VARY_WORK;
        es.bs_rbits = VARY_RBITS;
        es.bs_zflags = VARY_ZFLAGS;
        es.bs_lost = VARY_LOST;
        es.rcount = nullptr;
        last_dec_valid = false;
    }
    // A whole-half erasure: every log is 0, nothing to evaluate (the passes
    // count the received rows for rs16_decode_check)
    e_ident = identity_logs(g, vary);
    if (e_ident) {
        eval_in_col = elog_fused = false;
        return RS16_OK;
    }
    // High-rate half decodes of 2^9 / 2^10-row halves through the column
    // codec: it evaluates the polynomial itself (an n-point XOR convolution,
    // rs16_col.hip) and writes rcount; no kernel here.
    eval_in_col = S && (half_decode(g) ? g.high && col_ok(ilog2(g.n) - 1, S, nstripes)
                                       : col_ok(ilog2(g.n), S, nstripes, true));
    if (eval_in_col) return RS16_OK;
    es.stamps = stamp_prof == PROF_EVAL_POLY ? (uint64_t*)stamp_buf : nullptr;
    hipEvent_t pev;
    if (int rc = prof_begin(s, &pev, err)) return rc;
    // The decode passes that read erasure logs finish eval_poly's last
    // 256-point FWHT themselves, for the 256-row block of their tile's rows
    // (one kernel less) -- except the one-pass half-transform decode, whose
    // gather and reveal rows lie in different blocks.
    const bool small = g.high && g.n <= 2048 && !(diag & DIAG_EVAL_FULL);
    // (the column codec's half decodes of 2^9 / 2^10 rows finish it too)
    elog_fused = !(half_decode(g) && ilog2(g.n) - 1 <= 8);
    if (small) {
        // erasures are zero from row n on: only n/256 live blocks (rs16_misc.hip)
        RS16_HIP(launch_eval_poly_small(es, (uint32_t)g.n, (uint32_t*)evset->work32.p, (uint32_t*)evset->elog.p, d_log_walsh,
                                        s, !elog_fused));
    } else {
        RS16_HIP(launch_eval_poly_from_flags(es, (uint32_t*)evset->work32.p, (uint32_t*)evset->elog.p, d_log_walsh, s,
                                             !elog_fused));
    }
    return prof_end(PROF_EVAL_POLY, s, pev, err);
}

// Half-transform decode.  When every original is lost and the originals'
// segment is one half of the n work rows (high rate: rows [n/2, n) with
// n = 2 chunk; low rate: rows [0, n/2)), the input of the transform is zero
// on that half and only that half of its output is needed.  Then the top
// layer's butterflies and every formal-derivative term cancel on the needed
// half (see DESIGN.md "Half-transform decode"; checked against the
// sequential oracle by tests/test_half_decode.py):
//     FFT(FD(IFFT(x)))[dst half] = FFT_dst(IFFT_src(x[src half]))
// with IFFT_src / FFT_dst the n/2-row transforms over the low L-1 row bits
// with the twiddles of their half (skew_delta = its first row).  So the
// decode is an encode-shaped pipeline on n/2 rows: gather x e -> IFFT ->
// FFT -> reveal, with no formal derivative.
bool rs16_engine::half_decode(const DecodeGeom& g) {
    const bool orig_lost = g.high ? g.b_recv == 0 : g.a_recv == 0;
    return orig_lost && g.n >= 2 && g.n == 2 * (size_t)g.chunk;
}

// Identity multipliers.  When the erased rows are exactly one half of the n
// = 2^(L+1) work rows and the other half is received whole (k = m = n / 2,
// every original lost, every recovery shard received; the low rate adds the
// tail [n, 65536), rate_low.rs:183-197), the erasure log of every work row,
// eval_poly(e)[i] = sum_{j erased} log(i ^ j) mod 65535 (src/engine.rs:207-218
// as an XOR convolution with H(LogWalsh) = log), is the log of the
// subspace polynomial of the erased half at i: 0 for every i (the Cantor
// basis normalizes it to 1 on the complementary coset; checked against the
// oracle for every L in tests/test_eval_identity.py).  Then "MULTIPLY
// SHARDS" (rate_high.rs:203-228) and REVEAL ERASURES (:236-242) multiply by
// exp(0) = 1 and exp(65535) = 1: the passes take the rows as they are.  Only
// the pass form of the half decode (halves of 2^11 rows and more) uses it;
// the counts the caller gave pick it, as they pick the half decode.
bool rs16_engine::identity_logs(const DecodeGeom& g, uint32_t vary) const {
    if ((diag & DIAG_NO_IDENTITY) || vary > 1 || !half_decode(g) || ilog2(g.n) - 1 < 11) return false;
    if (g.a_count != g.chunk || g.b_count != g.chunk) return false;
    return g.high ? g.a_recv == g.a_count : g.b_recv == g.b_count;
}

int rs16_engine::mid_tables(int L, const uint32_t** out, rs16_error* err) {
    DevBuf& b = mid_tab[L];
    if (!b.p) {
        const HostTables& t = host_tables();
        const std::vector<uint32_t> ent = mid_matrix_entries(t, L);
        std::vector<uint32_t> tabs(ent.size() * 20);
        for (size_t i = 0; i < ent.size(); i++)
            std::copy_n(&t.mul_tab[(size_t)ent[i] * TAB_DWORDS], 20, &tabs[i * 20]);
        hipError_t he = b.reserve(tabs.size() * 4);
        if (he == hipSuccess) he = hipMemcpy(b.p, tabs.data(), tabs.size() * 4, hipMemcpyHostToDevice);
        if (he != hipSuccess) {
            b.release();
            return hip_fail(err, he);
        }
    }
    *out = (const uint32_t*)b.p;
    return RS16_OK;
}

// The pass sequence of a decode, given what decode_eval left in evset->elog /
// evset->work32 (erasure logs), evset->rbits (received rows) and evset->zflag (zero tiles).
int rs16_engine::decode_passes(const DecodeGeom& g, size_t S, size_t S_user, const uint8_t* seg_a, const uint8_t* flags_a,
                               const uint8_t* seg_b, const uint8_t* flags_b, uint8_t* rest, uint8_t* Z, uint8_t* U,
                               uint32_t* rcount, hipStream_t s, rs16_error* err, size_t nst, size_t bs_a, size_t bs_b,
                               size_t bs_rest) {
    PassArgs a = base_args(this, S);
    a.S_seg = a.S_rest = S_user;
    a.seg_a = seg_a;
    a.seg_b = seg_b;
    a.flags_a = flags_a;
    a.flags_b = flags_b;
    a.a_count = g.a_count;
    a.chunk = g.chunk;
    a.b_count = g.b_count;
    a.elog = (const uint32_t*)evset->elog.p;
    a.ework = elog_fused ? (const uint32_t*)evset->work32.p : nullptr;
    a.rest = rest;
    a.rest_seg_b = g.high ? 1 : 0;
    a.rbits = (const uint32_t*)evset->rbits.p;
    a.skew_ifft = a.skew_fft = 0;
    if (var_ns) {  // stripes with losses of their own (decode_eval's per-stripe metadata)
        a.bs_fa = var_bs_fa;
        a.bs_fb = var_bs_fb;
        a.bs_elog = VARY_WORK;
        a.bs_rbits = VARY_RBITS;
        a.bs_zflags = VARY_ZFLAGS;
        a.bs_lost = VARY_LOST;
        rcount = nullptr;
    }
    // nst > 1: independent stripes with one erasure pattern (rs16_decode_device_batch):
    // every launch covers all of them (PassArgs::stripe_tiles); stripe i's
    // segments / restored originals at + i bs_a / bs_b / bs_rest, its work
    // rows at Z / U + i n S
    const uint32_t ns = (uint32_t)nst;
    const size_t zs = (size_t)g.n * S;
    a.bs_seg = bs_a;
    a.bs_seg_b = bs_b;
    a.bs_rest = bs_rest;
    auto batch = [&](uint32_t tiles, size_t bs_in, size_t bs_in2, size_t bs_out) {
        a.stripe_tiles = ns > 1 ? tiles : 0;
        a.bs_in = bs_in;
        a.bs_in2 = bs_in2;
        a.bs_out = bs_out;
        return tiles * ns;
    };
    const int L = ilog2(g.n);
    if (half_decode(g)) {
        const uint32_t half = g.n / 2, src = g.high ? 0 : half, dst = g.high ? half : 0;
        const uint32_t orig = g.high ? g.b_count : g.a_count;
        a.row_base_in = a.skew_ifft = src;
        a.row_base_out = a.skew_fft = dst;
        const int Lh = L - 1;
        if (e_ident) {
            // Identity multipliers (identity_logs): gather the received half
            // as it is -> IFFT -> FFT -> its rows are the restored originals,
            // i.e. the encoder's three passes with the half's twiddles; the
            // first and last count the received flags for rs16_decode_check
            const int lo = Lh / 2, hi = Lh - lo;
            a.seg_a = g.high ? seg_a : seg_b;
            a.bs_seg = g.high ? bs_a : bs_b;
            a.a_count = half;
            a.rcount = rcount;
            a.cnt_flags = g.high ? flags_a : flags_b;
            a.cnt_base = src;
            a.cnt_seg = g.high ? 0 : 1;
            a.lo = 0;
            a.out = Z;
            RS16_PASS_AS(PROF_DEC_HALF_FIRST, ENC_FIRST, lo, a, batch(1u << hi, 0, 0, zs), s);
            a.rcount = nullptr;
            a.lo = lo;
            a.in = Z;
            RS16_PASS_AS(PROF_DEC_HALF_MID, ENC_MID, hi, a, batch(1u << lo, zs, 0, zs), s);
            a.lo = 0;
            a.out = rest;
            a.S_out = S_user;
            a.out_rows = orig;
            a.rcount = rcount;
            a.cnt_flags = g.high ? flags_b : flags_a;
            a.cnt_base = dst;
            a.cnt_seg = g.high ? 1 : 0;
            RS16_PASS_AS(DEC_HALF_LAST, ENC_LAST, lo, a, batch((orig + (1u << lo) - 1) >> lo, zs, 0, bs_rest), s);
            return RS16_OK;
        }
        // 2^6 .. 2^10-row halves: the whole decode in one launch (rs16_col.hip)
        // -- high rate with the polynomial in the kernel; the low rate from
        // 2^9 rows on, on eval_poly's output
        const bool col_eval = eval_in_col && g.high;
        if (!col_eval && Lh <= 8) {
            a.ework = nullptr;  // (decode_eval did the whole eval_poly)
            RS16_PASS(DEC_HALF_SINGLE, Lh, a, batch(1, 0, 0, 0), s);
            return RS16_OK;
        }
        if (col_eval || col_ok(Lh, S, ns)) {
            ColArgs c = col_args();
            c.in = g.high ? seg_a : seg_b;
            c.flags = g.high ? flags_a : flags_b;
            c.in_rows = g.high ? g.a_count : g.b_count;
            c.out = rest;
            c.S_in = c.S_out = S_user;
            c.qrow = (uint32_t)(S / 8);
            c.nstripes = ns;
            c.bs_in = g.high ? bs_a : bs_b;
            c.bs_out = bs_rest;
            c.out_rows = orig;
            c.base_in = c.skew_ifft = src;
            c.base_out = c.skew_fft = dst;
            c.chunk = g.chunk;
            c.e_pad = 1;  // (high rate: padding rows erased, nothing above the originals)
            c.bs_flags = g.high ? var_bs_fa : var_bs_fb;
            c.bs_flags_o = var_bs_fb;
            c.bs_elog = var_ns ? VARY_WORK : 0;
            if (col_eval) {
                // eval_poly in the kernel (decode_eval launched nothing)
                c.flags_o = flags_b;
                c.o_rows = g.b_count;
                c.vtab = nullptr;  // (col(): d_col_v + col_v_offset(2^(L+1)))
                c.rcount = rcount;
                return col(c, Lh, COL_DEC_EVAL, s, err);
            }
            c.elog = (const uint32_t*)evset->work32.p;  // (eval_poly without its last H_lo: elog_fused)
            return col(c, Lh, COL_DEC_EWORK, s, err);
        }
        const int lo = Lh / 2, hi = Lh - lo;
        a.lo = 0;
        a.out = Z;
        RS16_PASS_AS(PROF_DEC_HALF_FIRST, DEC_FIRST, lo, a, batch(1u << hi, 0, 0, zs), s);
        a.lo = lo;
        a.in = Z;
        RS16_PASS_AS(PROF_DEC_HALF_MID, ENC_MID, hi, a, batch(1u << lo, zs, 0, zs), s);
        a.lo = 0;
        a.out = nullptr;
        RS16_PASS(DEC_HALF_LAST, lo, a, batch((orig + (1u << lo) - 1) >> lo, zs, 0, 0), s);
        return RS16_OK;
    }
    if (eval_in_col) {
        // up to 2^11 work rows: the whole general decode in one launch,
        // polynomial and formal derivative in the kernel (rs16_col.hip);
        // segment A / B = recovery / originals (high rate) or originals /
        // recovery (low rate, rate_low.rs:168-247)
        ColArgs c = col_args();
        c.in = seg_a;
        c.flags = flags_a;
        c.in_rows = g.a_count;
        c.in_b = seg_b;
        c.bs_in_b = bs_b;
        c.flags_o = flags_b;
        c.o_rows = g.b_count;
        c.chunk = g.chunk;
        c.rev_a = g.high ? 0 : 1;
        c.e_pad = g.high ? 1 : 0;
        c.e_tail = g.high ? 0 : 1;
        c.e_k = g.high ? 0 : host_tables().col_k[L];
        c.out = rest;
        c.S_in = c.S_out = S_user;
        c.qrow = (uint32_t)(S / 8);
        c.nstripes = ns;
        c.bs_in = bs_a;
        c.bs_out = bs_rest;
        c.out_rows = g.high ? g.b_count : g.a_count;
        c.rcount = rcount;
        c.bs_flags = var_bs_fa;
        c.bs_flags_o = var_bs_fb;
        return col(c, L, COL_DEC_GEN, s, err);
    }
    if (L <= 8) {
        RS16_PASS(DEC_SINGLE, L, a, batch(1, 0, 0, 0), s);
        return RS16_OK;
    }
    const int lo = L / 2, hi = L - lo;
    // One flag per DEC_FIRST tile (2^hi <= 256): tiles without a received
    // row are skipped by DEC_FIRST and read as zero by DEC_MID / DEC_LAST.
    a.zflags = (const uint8_t*)evset->zflag.p;
    a.lostrange = (const uint32_t*)evset->lost.p + 512;  // (written by decode_eval)
    // Launch only the tiles that can hold a received row: a segment with no
    // received shard contributes none (its tiles are flagged by block 0).
    const uint32_t tile = 1u << lo, ntiles = 1u << hi;
    uint32_t t0z = ntiles, t1z = 0;
    if (g.a_recv) t0z = 0, t1z = (g.a_count + tile - 1) / tile;
    if (g.b_recv) {
        t0z = std::min(t0z, g.chunk / tile);
        t1z = std::max(t1z, std::min(ntiles, (uint32_t)(((size_t)g.chunk + g.b_count + tile - 1) / tile)));
    }
    if (t1z <= t0z) t0z = 0, t1z = 1;  // (unreachable: a decode has received shards) keep one launch
    a.tile_base = t0z;
    a.lo = 0;
    a.out = Z;
    RS16_PASS(DEC_FIRST, lo, a, batch(t1z - t0z, 0, 0, zs), s);
    a.tile_base = 0;
    // Only tiles that contain original rows are needed in the last pass,
    // so DEC_MID computes and stores only U rows of those tiles (its tile
    // row k is row bits [lo, L) = the last pass's tile index).
    const uint32_t ob = g.high ? g.chunk : 0;
    const uint32_t oc = g.high ? g.b_count : g.a_count;
    const uint32_t t0 = ob >> lo, t1 = (uint32_t)(((size_t)ob + oc + ((size_t)1 << lo) - 1) >> lo);
    a.lo = lo;
    a.in = Z;
    a.out = U;
    a.need_lo = t0;
    a.need_hi = t1;
    const size_t lost = g.high ? (size_t)g.b_count - g.b_recv : (size_t)g.a_count - g.a_recv;
    // Few lost originals: the middle pass's consumed rows may be few enough
    // for the direct product (mid_direct_kernel; DEC_MID then returns for
    // the stripes it covered -- decided on the device from lostrange)
    // (grid z = the stripe: at most 65535 of them in one launch)
    if (!(diag & DIAG_NO_MID_DIRECT) && lost <= ((size_t)MID_DIRECT_MAX << lo) && ns <= 65535) {
        const uint32_t* mt = nullptr;
        if (int rc = mid_tables(L, &mt, err)) return rc;
        batch(1u << lo, zs, 0, zs);  // (stripe displacements of the launch)
        hipEvent_t pev;
        if (int rc = prof_begin(s, &pev, err)) return rc;
        if (stamp_buf && stamp_prof == PROF_DEC_MID_DIRECT) a.stamps = (uint64_t*)stamp_buf;
        RS16_HIP(launch_mid_direct(a, mt, (uint32_t)hi, ns, s));
        a.stamps = nullptr;
        if (int rc = prof_end(PROF_DEC_MID_DIRECT, s, pev, err)) return rc;
        a.mid_direct = MID_DIRECT_MAX;
    }
    RS16_PASS(DEC_MID, hi, a, batch(1u << lo, zs, 0, zs), s);
    a.mid_direct = 0;
    a.need_lo = a.need_hi = 0;
    a.lo = 0;
    a.in = Z;
    a.in2 = U;
    a.out = nullptr;
    a.tile_base = t0;
    // Lost originals in few tiles (lost-range pruning leaves a handful of
    // tiles to this pass): one wave per quad column of each tile
    // (tile_last_kernel) instead of one 8-wave item per 32 quads, whose
    // latency was the pass.  Over more tiles the items win (scattered
    // losses: 128 tiles 81 -> 37 us; break-even 16-32 tiles,
    // scripts/probe_general.py).  How many tiles the lost originals span is
    // known on the device only (lostrange): with <= 2048 lost both kernels
    // are launched and each returns at once where the other one applies.
    const bool tile_last = lo == 8 && !(diag & DIAG_NO_TILE_LAST) && (lost <= 2048 || (diag & DIAG_TILE_LAST));
    if (tile_last) {
        a.tl_max = (diag & DIAG_TILE_LAST) ? (1u << hi) : TILE_LAST_MAX;
        // (the grid: tl_max tiles from the first lost original's, the kernel
        // reads that tile from lostrange; a launch that returns at once costs
        // per workgroup)
        const uint32_t tiles = batch(std::min(t1 - t0, a.tl_max), zs, zs, 0);
        hipEvent_t ev;
        if (int rc = prof_begin(s, &ev, err)) return rc;
        if (stamp_buf && stamp_prof == PROF_DEC_TILE_LAST) a.stamps = (uint64_t*)stamp_buf;
        RS16_HIP(launch_tile_last(a, tiles, s));
        a.stamps = nullptr;
        if (int rc = prof_end(PROF_DEC_TILE_LAST, s, ev, err)) return rc;
        if (diag & DIAG_TILE_LAST) return RS16_OK;  // (every span is tile_last's)
    }
    RS16_PASS(DEC_LAST, lo, a, batch(t1 - t0, zs, zs, 0), s);
    return RS16_OK;
}

// The FFT half of the multi-chunk encoders: FFT of nch chunks of Z (batched
// like the IFFTs below, skew_delta applied to absolute rows), recovery rows
// [0, m) stored to d_rec.
int rs16_engine::fft_to_recovery(size_t m, size_t S, size_t S_user, const uint8_t* src, uint8_t* Z, uint8_t* d_rec,
                                 size_t chunk, uint32_t nch, uint32_t skew, hipStream_t s, rs16_error* err) {
    const int L = ilog2(chunk), lo = L <= 8 ? L : L / 2, hi = L - lo;
    PassArgs a = base_args(this, S);
    a.skew_fft = skew;
    // src != Z: every chunk's FFT reads the one chunk at src (the first pass only)
    const uint32_t mask = src != Z ? (uint32_t)(chunk - 1) : 0u;
    a.in = src;
    a.in_rows_mask = mask;
    if (hi) {
        a.out = Z;
        a.lo = lo;
        RS16_PASS(GEN_FFT, hi, a, nch << lo, s);
        a.in = Z;
        a.in_rows_mask = 0;
    }
    a.out = d_rec;
    a.S_out = S_user;
    a.lo = 0;
    a.out_rows = (uint32_t)m;
    RS16_PASS(ENC_LAST, lo, a, (uint32_t)((m + ((size_t)1 << lo) - 1) >> lo), s);
    return RS16_OK;
}

// HighRateEncoder::encode with more originals than one chunk
// (src/rate/rate_high.rs:44-83): IFFT of every chunk c of the zero-padded
// originals with skew_delta = c chunk + chunk (pos = c chunk), XOR of all of
// them into chunk 0 (xor_within, :56-74), FFT of chunk 0 with skew 0.  The
// twiddle of a layer at relative row r is skew[r + skew_delta + d - 1] =
// skew[(c chunk + r) + chunk + d - 1]: the per-chunk transforms are one
// transform over absolute rows with skew_delta = chunk whose layers stay
// inside a chunk, so every chunk's IFFT runs in the same launches (tiles over
// all chunks; the first pass gathers the originals, rows >= k read as zero),
// then one XOR reduction, then the FFT.
int rs16_engine::encode_high_multi(size_t k, size_t m, size_t S, size_t S_user, const uint8_t* d_orig, uint8_t* d_rec,
                                   uint8_t* Z, hipStream_t s, rs16_error* err) {
    const size_t chunk = next_pow2(m);
    const uint32_t nch = (uint32_t)((k + chunk - 1) / chunk);
    const int L = ilog2(chunk), lo = L <= 8 ? L : L / 2, hi = L - lo;
    if (L == 0) {  // one-row chunks: the single recovery row is the XOR of the originals
        if (Z != d_orig) RS16_HIP(hipMemcpy2DAsync(Z, S, d_orig, S_user, S, k, hipMemcpyDeviceToDevice, s));
        RS16_HIP(launch_xor_chunks(Z, S, nch, s));
        if (d_rec != Z) RS16_HIP(hipMemcpyAsync(d_rec, Z, S, hipMemcpyDeviceToDevice, s));
        return RS16_OK;
    }
    if (L == (int)COLM_L && nch <= COLM_MAX_CHUNKS && col_ok(L, S, 1))
        return col_multi(k, m, S, S_user, d_orig, d_rec, nch, true, s, err);
    if (col_chunks_ok(L, nch, S, true)) {
        // 256 / 512 / 1024-row chunks: every chunk's IFFT into Z (one
        // workgroup per quad column and chunk), then the FFT of their XOR
        ColArgs c = col_args();
        c.in = d_orig;
        c.S_in = S_user;
        c.out = Z;
        c.S_out = S;
        c.qrow = (uint32_t)(S / 8);
        c.in_rows = (uint32_t)k;
        c.out_rows = (uint32_t)(nch * chunk);
        c.skew_ifft = (uint32_t)chunk;
        c.nch = nch;
        if (int rc = col(c, L, COL_ENC_IFFT, s, err)) return rc;
        c.in = Z;
        c.S_in = S;
        c.out = d_rec;
        c.S_out = S_user;
        c.in_rows = (uint32_t)(nch * chunk);
        c.out_rows = (uint32_t)m;
        c.skew_ifft = 0;
        c.skew_fft = 0;
        return col(c, L, COL_ENC_FFTX, s, err);
    }
    PassArgs a = base_args(this, S);
    a.seg_a = d_orig;
    a.S_seg = S_user;
    a.a_count = (uint32_t)k;
    a.skew_ifft = (uint32_t)chunk;
    a.out = Z;
    a.lo = 0;
    RS16_PASS(ENC_FIRST, lo, a, nch << hi, s);
    if (hi) {
        a.in = a.out = Z;
        a.lo = lo;
        RS16_PASS(GEN_IFFT, hi, a, nch << lo, s);
    }
    RS16_HIP(launch_xor_chunks(Z, chunk * S, nch, s));
    return fft_to_recovery(m, S, S_user, Z, Z, d_rec, chunk, 1, 0, s, err);
}

// LowRateEncoder::encode (src/rate/rate_low.rs:44-83): IFFT of the
// zero-padded originals (one chunk, skew 0), copied into every recovery chunk
// c, FFT of each with skew_delta = c chunk + chunk -- batched as above
// (absolute rows, skew_delta = chunk), recovery = rows [0, m).  The copies
// are not made: the transformed chunk goes to the scratch U and the FFT's
// first pass reads it for every chunk (PassArgs::in_rows_mask).
int rs16_engine::encode_low_multi(size_t k, size_t m, size_t S, size_t S_user, const uint8_t* d_orig, uint8_t* d_rec,
                                  uint8_t* Z, uint8_t* U, hipStream_t s, rs16_error* err) {
    const size_t chunk = next_pow2(k);
    const uint32_t nch = (uint32_t)((m + chunk - 1) / chunk);
    const int L = ilog2(chunk), lo = L <= 8 ? L : L / 2, hi = L - lo;
    if (L == 0) {  // one original: every transform is the identity, every recovery row a copy
        if (Z != d_orig) RS16_HIP(hipMemcpyAsync(Z, d_orig, S, hipMemcpyDeviceToDevice, s));
        RS16_HIP(launch_copy_chunks(Z, S, nch, s));
        if (d_rec != Z) RS16_HIP(hipMemcpy2DAsync(d_rec, S_user, Z, S, S, m, hipMemcpyDeviceToDevice, s));
        return RS16_OK;
    }
    if (nch == 1 && col_ok(L, S, 1)) {
        // one recovery chunk of 512 / 1024 rows: one launch (rs16_col.hip)
        ColArgs c = col_args();
        c.in = d_orig;
        c.out = d_rec;
        c.S_in = c.S_out = S_user;
        c.qrow = (uint32_t)(S / 8);
        c.in_rows = (uint32_t)k;
        c.out_rows = (uint32_t)m;
        c.skew_ifft = 0;
        c.skew_fft = (uint32_t)chunk;
        return col(c, L, COL_ENC, s, err);
    }
    if (nch > 1 && L == (int)COLM_L && nch <= COLM_MAX_CHUNKS && col_ok(L, S, 1))
        return col_multi(k, m, S, S_user, d_orig, d_rec, nch, false, s, err);
    if (nch > 1 && col_chunks_ok(L, nch, S, false)) {
        // 256 / 512 / 1024-row chunks: one launch, one workgroup per (quad
        // column, recovery chunk), each running the originals' IFFT itself.
        // Every chunk's workgroups read the originals, and chunk 0's write
        // recovery rows [0, chunk): when the two arrays overlap (the Rate
        // API's work buffer, rate_low.rs:44-83) chunk 0 could overwrite
        // originals other chunks have not loaded yet, so the originals are
        // read from a copy in U then (U: next_pow2(k) rows, pitch S).
        const uint8_t* src = d_orig;
        size_t s_in = S_user;
        const uint8_t *o0 = d_orig, *o1 = d_orig + (k - 1) * S_user + S;
        const uint8_t *r0 = d_rec, *r1 = d_rec + (m - 1) * S_user + S;
        if (o0 < r1 && r0 < o1) {
            if (!U) return set_error(err, RS16_INVALID_ARGUMENT);
            RS16_HIP(hipMemcpy2DAsync(U, S, d_orig, S_user, S, k, hipMemcpyDeviceToDevice, s));
            src = U;
            s_in = S;
        }
        ColArgs c = col_args();
        c.in = src;
        c.out = d_rec;
        c.S_in = s_in;
        c.S_out = S_user;
        c.qrow = (uint32_t)(S / 8);
        c.in_rows = (uint32_t)k;
        c.out_rows = (uint32_t)m;
        c.skew_ifft = 0;
        c.skew_fft = (uint32_t)chunk;
        c.nch = nch;
        return col(c, L, COL_ENC, s, err);
    }
    // U belongs to the caller's stream (no engine-wide fallback: two calls
    // on concurrent streams sharing one buffer restored wrong data, round 3)
    if (!U) return set_error(err, RS16_INVALID_ARGUMENT);
    PassArgs a = base_args(this, S);
    a.seg_a = d_orig;
    a.S_seg = S_user;
    a.a_count = (uint32_t)k;
    a.skew_ifft = 0;
    a.out = U;
    a.lo = 0;
    RS16_PASS(ENC_FIRST, lo, a, 1u << hi, s);
    if (hi) {
        a.in = a.out = U;
        a.lo = lo;
        RS16_PASS(GEN_IFFT, hi, a, 1u << lo, s);
    }
    return fft_to_recovery(m, S, S_user, U, Z, d_rec, chunk, nch, (uint32_t)chunk, s, err);
}
