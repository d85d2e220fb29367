/*
 * rs16.h -- C ABI of the MI355X-native GF(2^16) Reed-Solomon codec.
 *
 * This is the drop-in boundary for the hot path of malaire/reed-solomon-16
 * v0.1.0 (a Rust crate).  Each entry point names the reference interface it
 * replaces (file:line in the reference tree).  A Rust `impl Engine` /
 * FFI stub binding these symbols is shown in INTEGRATION.md.
 *
 * Conventions
 *  - Every fallible call returns 0 (RS16_OK) or an error code and, if `err`
 *    is non-NULL, fills it with the code and the payload fields of the
 *    reference's `Error` variant (src/lib.rs:31-125) in declaration order.
 *  - Shard arrays are the reference's flat layout (ShardsRefMut,
 *    src/engine/shards.rs:60-66): shard i starts at byte i*shard_bytes;
 *    every 64-byte block holds 32 low bytes then 32 high bytes
 *    (src/algorithm.md:6-32).
 *  - `_device` / `d_` pointers are HIP device pointers on the engine's
 *    device; `stream` is a hipStream_t (NULL = the engine's own stream).
 *    Device-pointer calls are asynchronous on that stream.
 *  - One engine must not be used from two threads at once (it owns scratch
 *    workspace); create one engine per device/thread.  It may be used on
 *    several streams: a call that needs the engine's scratch on stream s
 *    first makes s wait (hipStreamWaitEvent) for the engine's previous such
 *    call when that was issued on another stream, so two streams never
 *    share the scratch concurrently (calls on one engine serialise; use one
 *    engine per stream for concurrent codecs).
 *  - rs16_engine_free waits for the engine's work (its own streams and the
 *    last caller stream it ran on, through an event), releases the work space of
 *    every encoder/decoder created on the engine and detaches them: a
 *    detached encoder/decoder fails every call with RS16_INVALID_ARGUMENT,
 *    and rs16_{en,de}coder_free of it only frees its host memory (safe in
 *    any order at process exit).
 */
#ifndef RS16_H
#define RS16_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Error -- reed_solomon_16::Error, src/lib.rs:31-125 ---------------- */
typedef enum rs16_error_code {
    RS16_OK = 0,
    RS16_DIFFERENT_SHARD_SIZE = 1,           /* v0 shard_bytes, v1 got */
    RS16_DUPLICATE_ORIGINAL_SHARD_INDEX = 2, /* v0 index */
    RS16_DUPLICATE_RECOVERY_SHARD_INDEX = 3, /* v0 index */
    RS16_INVALID_ORIGINAL_SHARD_INDEX = 4,   /* v0 original_count, v1 index */
    RS16_INVALID_RECOVERY_SHARD_INDEX = 5,   /* v0 recovery_count, v1 index */
    RS16_INVALID_SHARD_SIZE = 6,             /* v0 shard_bytes */
    RS16_NOT_ENOUGH_SHARDS = 7,              /* v0 original_count, v1 original_received_count,
                                                v2 recovery_received_count */
    RS16_TOO_FEW_ORIGINAL_SHARDS = 8,        /* v0 original_count, v1 original_received_count */
    RS16_TOO_MANY_ORIGINAL_SHARDS = 9,       /* v0 original_count */
    RS16_UNSUPPORTED_SHARD_COUNT = 10,       /* v0 original_count, v1 recovery_count */
    /* Not in the reference (it has no device and panics on misuse): */
    RS16_DEVICE_ERROR = 100,                 /* HIP runtime failure, v0 = hipError_t (RCCL: 1000 + ncclResult_t) */
    RS16_INVALID_ARGUMENT = 101              /* engine-op misuse the reference would panic on */
} rs16_error_code;

typedef struct rs16_error {
    int32_t code;
    uint64_t v0, v1, v2;
} rs16_error;

/* `impl Display for Error` (src/lib.rs:130-222): writes the exact message,
 * returns its length (excluding NUL); truncates to len-1 bytes. */
size_t rs16_error_message(const rs16_error* err, char* buf, size_t len);

/* ---- Engine -- trait Engine (src/engine.rs:140-260) ---------------------
 * rs16_engine_new plays NoSimd::new (src/engine/engine_nosimd.rs:27-35):
 * it builds the GF tables (src/engine/tables.rs) once per process and
 * uploads them to the device's HBM. */
typedef struct rs16_engine rs16_engine;
rs16_engine* rs16_engine_new(int device, rs16_error* err);
/* rs16_engine_new with creation flags (0 = rs16_engine_new).
 * RS16_ENGINE_OWN_QUEUE: the engine's stream gets a hardware queue of its
 * own (a stream with a CU mask enabling every CU; the HIP runtime shares its
 * GPU_MAX_HW_QUEUES queues among unmasked streams only).  Two engines whose
 * streams share a queue run one after the other; serving callers that keep
 * two stripes in flight on two engines create the second one this way so the
 * pair overlaps deterministically (profiles/r05_queues.txt).
 * Unknown flags: RS16_INVALID_ARGUMENT. */
enum { RS16_ENGINE_OWN_QUEUE = 1 };
rs16_engine* rs16_engine_new_ex(int device, int flags, rs16_error* err);
void rs16_engine_free(rs16_engine* eng);
int rs16_engine_device(const rs16_engine* eng);
void* rs16_engine_stream(const rs16_engine* eng);     /* hipStream_t owned by the engine */
int rs16_engine_synchronize(rs16_engine* eng, void* stream, rs16_error* err);

/* Engine::fft (src/engine.rs:158-165): in-place DIT FFT on shards
 * [pos, pos+size) of `data` (shard_count x shard_bytes, device).  Outputs
 * [pos, pos+truncated_size) are exact for any input.  */
int rs16_engine_fft(rs16_engine* eng, void* data, size_t shard_count, size_t shard_bytes, size_t pos, size_t size,
                    size_t truncated_size, size_t skew_delta, void* stream, rs16_error* err);
/* Engine::fft_skew_end (src/engine.rs:222-230): skew_delta = pos + size. */
int rs16_engine_fft_skew_end(rs16_engine* eng, void* data, size_t shard_count, size_t shard_bytes, size_t pos,
                             size_t size, size_t truncated_size, void* stream, rs16_error* err);
/* Engine::ifft (src/engine.rs:188-195).  As in the reference contract,
 * shards [pos+truncated_size, pos+size) must be zero on input. */
int rs16_engine_ifft(rs16_engine* eng, void* data, size_t shard_count, size_t shard_bytes, size_t pos, size_t size,
                     size_t truncated_size, size_t skew_delta, void* stream, rs16_error* err);
/* Engine::ifft_skew_end (src/engine.rs:242-250). */
int rs16_engine_ifft_skew_end(rs16_engine* eng, void* data, size_t shard_count, size_t shard_bytes, size_t pos,
                              size_t size, size_t truncated_size, void* stream, rs16_error* err);
/* Engine::fwht (src/engine.rs:175) on a device u16[65536]; data beyond
 * truncated_size must be zero (the only way eval_poly uses it).  Bit-exact
 * u16 outputs: the engine-level op runs the reference's layer order with its
 * add_mod / sub_mod (src/engine.rs:90-100), so 0 and 65535 come out where the
 * reference has them (tests/test_gpu_engine.py).  The decoders' internal
 * erasure-log kernels only need the residue mod 65535 and use a faster order
 * (both values mean the same log, exp[65535] == exp[0], src/engine/tables.rs:118). */
int rs16_engine_fwht(rs16_engine* eng, uint16_t* d_data, size_t truncated_size, void* stream, rs16_error* err);
/* Engine::eval_poly (src/engine.rs:207-218) on a device u16[65536]; bit-exact
 * as rs16_engine_fwht. */
int rs16_engine_eval_poly(rs16_engine* eng, uint16_t* d_erasures, size_t truncated_size, void* stream,
                          rs16_error* err);
/* Engine::mul (src/engine.rs:198): x[] *= log_m, bytes % 64 == 0. */
int rs16_engine_mul(rs16_engine* eng, void* d_x, size_t bytes, uint16_t log_m, void* stream, rs16_error* err);
/* Engine::xor (src/engine.rs:201): x[] ^= y[], bytes % 64 == 0. */
int rs16_engine_xor(rs16_engine* eng, void* d_x, const void* d_y, size_t bytes, void* stream, rs16_error* err);
/* Engine::xor_within (src/engine.rs:256-259), ranges must not overlap. */
int rs16_engine_xor_within(rs16_engine* eng, void* data, size_t shard_count, size_t shard_bytes, size_t x, size_t y,
                           size_t count, void* stream, rs16_error* err);
/* Engine::formal_derivative (src/engine.rs:233-238); shard_count must be a
 * power of two (the reference panics on slice bounds otherwise). */
int rs16_engine_formal_derivative(rs16_engine* eng, void* data, size_t shard_count, size_t shard_bytes, void* stream,
                                  rs16_error* err);

/* ---- Rates -- src/rate.rs:51-107, src/rate/rate_default.rs:15-64 --------- */
typedef enum rs16_rate { RS16_RATE_DEFAULT = 0, RS16_RATE_HIGH = 1, RS16_RATE_LOW = 2 } rs16_rate;
/* Rate::supports / ReedSolomonEncoder::supports (src/reed_solomon.rs:76-84). */
int rs16_supports(int rate, size_t original_count, size_t recovery_count);
/* Rate::validate (src/rate.rs:91-106). */
int rs16_validate(int rate, size_t original_count, size_t recovery_count, size_t shard_bytes, rs16_error* err);
/* use_high_rate (src/rate/rate_default.rs:15-64): 1 high, 0 low, -1 error. */
int rs16_use_high_rate(size_t original_count, size_t recovery_count, rs16_error* err);
/* {High,Low}Rate{Encoder,Decoder}::work_count (rate_high.rs:131-137,301-305; rate_low.rs:131-137,301-305). */
size_t rs16_encoder_work_count(int high, size_t original_count, size_t recovery_count);
size_t rs16_decoder_work_count(int high, size_t original_count, size_t recovery_count);

/* ---- Encoder -- RateEncoder (src/rate.rs:113-173) with the Rate chosen
 *      by `rate`; RS16_RATE_DEFAULT == ReedSolomonEncoder (src/reed_solomon.rs:13-85).
 *      Work space lives in HBM (EncoderWork, src/rate/encoder_work.rs). */
typedef struct rs16_encoder rs16_encoder;
rs16_encoder* rs16_encoder_new(rs16_engine* eng, int rate, size_t original_count, size_t recovery_count,
                               size_t shard_bytes, rs16_error* err);
void rs16_encoder_free(rs16_encoder* enc);
int rs16_encoder_reset(rs16_encoder* enc, size_t original_count, size_t recovery_count, size_t shard_bytes,
                       rs16_error* err);
/* add_original_shard (src/rate/encoder_work.rs:49-69); shard in host memory.
 * The shard is copied (host memcpy, no device call) into a page-locked image
 * of the work buffer; consecutive shards stream to HBM in 1 MiB DMA copies
 * while the caller keeps adding, so the caller may reuse its buffer at once. */
int rs16_encoder_add_original_shard(rs16_encoder* enc, const void* shard, size_t len, rs16_error* err);
/* same, shard in device memory (copied on the engine stream). */
int rs16_encoder_add_original_shard_device(rs16_encoder* enc, const void* d_shard, size_t len, rs16_error* err);
/* encode (rate_high.rs:44-83 / rate_low.rs:44-83); on success the
 * EncoderResult (src/encoder_result.rs) is valid until rs16_encoder_result_drop.
 * Returns once the work is enqueued on the engine stream: the last staged
 * rows go to HBM, the passes run, and when any original came from host
 * memory the recovery rows come back in one DMA copy to page-locked memory
 * (rs16_encoder_recovery waits for it).
 * The encode works in place: calling it again while the result is held
 * returns RS16_INVALID_ARGUMENT (the reference's &mut borrow makes that a
 * compile error, src/rate.rs:157-166); add_original_shard in that state
 * returns TooManyOriginalShards, as every original is in. */
int rs16_encoder_encode(rs16_encoder* enc, rs16_error* err);
/* EncoderResult::recovery (src/encoder_result.rs:16-19): host pointer to
 * recovery shard `index` (shard_bytes, page-locked, valid until the result is
 * dropped), NULL if index >= recovery_count (or on a device error, err set).
 * The first call waits for the recovery rows to be in host memory. */
const void* rs16_encoder_recovery(rs16_encoder* enc, size_t index, rs16_error* err);
/* The same shard in HBM: device pointer, NULL if index >= recovery_count. */
const void* rs16_encoder_recovery_device(rs16_encoder* enc, size_t index);
/* Copy recovery shard `index` to host memory; returns 1 if it exists, 0 if not, <0 on error. */
int rs16_encoder_recovery_copy(rs16_encoder* enc, size_t index, void* dst, size_t len, rs16_error* err);
/* Drop for EncoderResult (src/encoder_result.rs:48-52). */
void rs16_encoder_result_drop(rs16_encoder* enc);
int rs16_encoder_is_high_rate(const rs16_encoder* enc);

/* ---- Decoder -- RateDecoder (src/rate.rs:179-250); RS16_RATE_DEFAULT ==
 *      ReedSolomonDecoder (src/reed_solomon.rs:93-183). */
typedef struct rs16_decoder rs16_decoder;
rs16_decoder* rs16_decoder_new(rs16_engine* eng, int rate, size_t original_count, size_t recovery_count,
                               size_t shard_bytes, rs16_error* err);
void rs16_decoder_free(rs16_decoder* dec);
int rs16_decoder_reset(rs16_decoder* dec, size_t original_count, size_t recovery_count, size_t shard_bytes,
                       rs16_error* err);
/* add_original_shard / add_recovery_shard (src/rate/decoder_work.rs:62-116).
 * Host shards are staged like the encoder's (page-locked image of the work
 * layout, runs of consecutive positions streamed to HBM while adding). */
int rs16_decoder_add_original_shard(rs16_decoder* dec, size_t index, const void* shard, size_t len, rs16_error* err);
int rs16_decoder_add_recovery_shard(rs16_decoder* dec, size_t index, const void* shard, size_t len, rs16_error* err);
int rs16_decoder_add_original_shard_device(rs16_decoder* dec, size_t index, const void* d_shard, size_t len,
                                           rs16_error* err);
int rs16_decoder_add_recovery_shard_device(rs16_decoder* dec, size_t index, const void* d_shard, size_t len,
                                           rs16_error* err);
/* decode (rate_high.rs:168-247 / rate_low.rs:168-247); DecoderResult valid until drop.
 * The decode restores in place: decode or add_*_shard while the result is
 * held returns RS16_INVALID_ARGUMENT (a compile error in the reference). */
int rs16_decoder_decode(rs16_decoder* dec, rs16_error* err);
/* DecoderResult::restored_original (src/decoder_result.rs:16-19): host
 * pointer to restored original `index` (page-locked, valid until the result
 * is dropped), NULL if it was received or index >= original_count (or on a
 * device error, err set).  After a decode with host shards the restored rows
 * come back in one DMA copy; the first call waits for it. */
const void* rs16_decoder_restored_original(rs16_decoder* dec, size_t index, rs16_error* err);
/* The same shard in HBM: device pointer or NULL. */
const void* rs16_decoder_restored_original_device(rs16_decoder* dec, size_t index);
/* Copy restored original `index` to host; returns 1 if restored, 0 if None, <0 on error. */
int rs16_decoder_restored_original_copy(rs16_decoder* dec, size_t index, void* dst, size_t len, rs16_error* err);
/* Drop for DecoderResult (src/decoder_result.rs:44-48). */
void rs16_decoder_result_drop(rs16_decoder* dec);
int rs16_decoder_is_high_rate(const rs16_decoder* dec);

/* ---- Device-resident one-shot codec (the benchmark path) -----------------
 * reed_solomon_16::encode (src/lib.rs:242-279) with originals and recovery
 * already in HBM: d_original = original_count shards, d_recovery receives
 * recovery_count shards.  Default rate selection as ReedSolomonEncoder. */
int rs16_encode_device(rs16_engine* eng, size_t original_count, size_t recovery_count, size_t shard_bytes,
                       const void* d_original, void* d_recovery, void* stream, rs16_error* err);
/* rs16_encode_device for `nstripes` independent stripes of one geometry in
 * one call (many objects, each its own codeword set; SURVEY.md 8(f)3
 * "batched independent codewords"): stripe i's original_count shards at
 * d_original + i * original_stride bytes, its recovery_count shards written
 * at d_recovery + i * recovery_stride (strides >= count * shard_bytes and
 * multiples of 64, else RS16_INVALID_ARGUMENT).
 * Every stripe's result equals rs16_encode_device on it alone.  High-rate
 * stripes with original_count <= next_pow2(recovery_count) -- every stripe
 * with original_count <= recovery_count -- run batched, each pass launch
 * covering all stripes, so stripes far below the chip's size (100:100,
 * 1000:1000) still fill it; other shapes run stripe after stripe.  The
 * reference encodes one stripe per call (src/lib.rs:242-279). */
int rs16_encode_device_batch(rs16_engine* eng, size_t original_count, size_t recovery_count, size_t shard_bytes,
                             size_t nstripes, const void* d_original, size_t original_stride, void* d_recovery,
                             size_t recovery_stride, void* stream, rs16_error* err);
/* reed_solomon_16::decode (src/lib.rs:287-344), device-resident: d_original
 * holds original_count shard slots (received ones valid, flagged by the
 * device byte array d_original_received); d_recovery holds recovery_count
 * slots flagged by d_recovery_received.  The host passes the number of
 * received shards of each kind: they give the reference's NotEnoughShards /
 * nothing-to-do checks AND select the launch -- a count of 0 means "no
 * shard of this kind was received", and the first pass then launches no
 * tile of that segment.  The counts MUST equal the number of nonzero flags
 * (a 0 count with set flags drops those shards and restores wrong data
 * without an error; rs16_decode_check detects it after the fact).  Lost
 * originals are restored in place into d_original.  Default rate selection
 * as ReedSolomonDecoder. */
int rs16_decode_device(rs16_engine* eng, size_t original_count, size_t recovery_count, size_t shard_bytes,
                       void* d_original, const uint8_t* d_original_received, const void* d_recovery,
                       const uint8_t* d_recovery_received, size_t original_received_count,
                       size_t recovery_received_count, void* stream, rs16_error* err);
/* rs16_decode_device for `nstripes` independent stripes that lost the same
 * shards -- the case of a failed device, which holds the same shard index of
 * every stripe: the received flags and counts are shared, stripe i's
 * original slots at d_original + i * original_stride bytes (lost ones
 * restored in place), its recovery at d_recovery + i * recovery_stride
 * (strides as for rs16_encode_device_batch).
 * One eval_poly for all, every pass launch covering all stripes.  Every
 * stripe's result equals rs16_decode_device on it alone. */
int rs16_decode_device_batch(rs16_engine* eng, size_t original_count, size_t recovery_count, size_t shard_bytes,
                             size_t nstripes, void* d_original, size_t original_stride,
                             const uint8_t* d_original_received, const void* d_recovery, size_t recovery_stride,
                             const uint8_t* d_recovery_received, size_t original_received_count,
                             size_t recovery_received_count, void* stream, rs16_error* err);
/* rs16_decode_device for `nstripes` independent stripes, EACH WITH ITS OWN
 * received set (the reference decodes one stripe per call with that call's
 * received shards: src/lib.rs:287-344, src/rate/decoder_work.rs:62-139):
 * stripe i's flags at d_original_received + i * original_received_stride and
 * d_recovery_received + i * recovery_received_stride (strides >= the counts),
 * its received counts in the HOST arrays original_received_counts[i] /
 * recovery_received_counts[i] (which must equal its flags, as for
 * rs16_decode_device), its shards as for rs16_decode_device_batch.  Errors are
 * the per-stripe ones (NotEnoughShards with the first failing stripe's
 * numbers).  One eval_poly launch with a grid row per stripe, then pass
 * launches shared by all stripes.  Every stripe's result equals
 * rs16_decode_device on it alone.  (rs16_decode_check does not cover it.) */
int rs16_decode_device_batch_varied(rs16_engine* eng, size_t original_count, size_t recovery_count,
                                    size_t shard_bytes, size_t nstripes, void* d_original, size_t original_stride,
                                    const uint8_t* d_original_received, size_t original_received_stride,
                                    const void* d_recovery, size_t recovery_stride,
                                    const uint8_t* d_recovery_received, size_t recovery_received_stride,
                                    const size_t* original_received_counts, const size_t* recovery_received_counts,
                                    void* stream, rs16_error* err);
/* Checked mode of the engine's last decode: waits for `stream` and compares
 * the received counts that decode was given with the rows the device flags
 * mark received (the eval_poly kernels count them per 64-row chunk as they
 * scan the flags, off the host's path).  RS16_OK when they agree (or no
 * decode ran), else RS16_INVALID_ARGUMENT with v0 / v1 = the originals /
 * recovery shards the flags mark received. */
int rs16_decode_check(rs16_engine* eng, void* stream, rs16_error* err);
/* Concurrent column slices of rs16_encode_device / rs16_decode_device (1..4,
 * default 1): the shard columns are split into slices of multiples of 64
 * bytes (each 64-byte column block is an independent codeword, so results
 * are identical) that run on internal streams forked from and joined back
 * into the call's stream.  The calls stay asynchronous and ordered on
 * `stream`.  On MI355X / ROCm 7.2 the fork/join costs more than the overlap
 * gains; independent codecs belong on independent streams. */
int rs16_engine_set_slices(rs16_engine* eng, int slices, rs16_error* err);

/* ---- Host-resident one-shot codec ---------------------------------------
 * reed_solomon_16::encode / decode (src/lib.rs:242-344) with every shard in
 * host memory (page-locked, rs16_host_alloc, for DMA-rate copies; pageable
 * works too).  The shard columns are processed in slices of slice_bytes (a
 * multiple of 64; 0 = the whole shard) that alternate between two streams,
 * so that the host->device copy of one slice, the device codec of another
 * and the device->host copy of a third may overlap (on MI355X the pitched
 * copies of narrow slices cost more than the overlap gains; see
 * DESIGN.md).  Synchronous: returns when the
 * outputs are in host memory.  Decode: received flags are host byte arrays;
 * lost originals are restored in place into h_original. */
int rs16_encode_host(rs16_engine* eng, size_t original_count, size_t recovery_count, size_t shard_bytes,
                     const void* h_original, void* h_recovery, size_t slice_bytes, rs16_error* err);
int rs16_decode_host(rs16_engine* eng, size_t original_count, size_t recovery_count, size_t shard_bytes,
                     void* h_original, const uint8_t* original_received, const void* h_recovery,
                     const uint8_t* recovery_received, size_t slice_bytes, rs16_error* err);

/* ---- Split device decode -------------------------------------------------
 * rs16_decode_device in two halves on two streams.  rs16_decode_prepare
 * takes the received pattern only (the same flags / counts and checks as
 * rs16_decode_device: UnsupportedShardCount, InvalidArgument,
 * NotEnoughShards) and enqueues the erasure locator, eval_poly of the
 * erasure vector (src/rate/rate_high.rs:168-202, src/engine.rs:207-218), on
 * `stream`; rs16_decode_device_prepared then runs the rest of the decode
 * (src/rate/rate_high.rs:203-247) on its own stream, ordered after the
 * preparation.  The pattern of a decode is known before its shards are (a
 * storage system knows which devices failed), so the locator can be computed
 * while the shards are still being produced or copied in: work the caller
 * issues on the engine between the two calls that does not decode -- e.g.
 * the encode of the stripe whose recovery is about to be decoded -- runs
 * concurrently with the preparation.  One preparation per engine, consumed
 * by the next rs16_decode_device_prepared with the same (k, m, shard_bytes)
 * (else InvalidArgument); any other decode on the engine in between orders
 * itself after the preparation and discards it.  The flag arrays must keep
 * their contents until the prepared decode has run.  Results are those of
 * rs16_decode_device; rs16_decode_check covers the prepared decode. */
int rs16_decode_prepare(rs16_engine* eng, size_t original_count, size_t recovery_count, size_t shard_bytes,
                        const uint8_t* d_original_received, const uint8_t* d_recovery_received,
                        size_t original_received_count, size_t recovery_received_count, void* stream,
                        rs16_error* err);
int rs16_decode_device_prepared(rs16_engine* eng, size_t original_count, size_t recovery_count,
                                size_t shard_bytes, void* d_original, const void* d_recovery, void* stream,
                                rs16_error* err);

/* ---- Host-resident stripes, pipelined (full duplex) -----------------------
 * nstripes independent stripes in host memory (stripe i's originals at
 * h_original + i original_stride, its recovery at h_recovery + i
 * recovery_stride; page-locked memory for DMA-rate copies), each encoded /
 * decoded exactly as rs16_encode_host / rs16_decode_host would, with two
 * stripes in flight: the host->device copy of stripe i + 1 and the
 * device->host copy of stripe i - 1 run on two copy streams while stripe i
 * is on the device, so both directions of the link carry data at once (one
 * stripe alone cannot overlap: its outputs exist only after its inputs are
 * all in).  Copies are contiguous row runs, no pitched copies.  The
 * reference's EncoderWork / DecoderWork path (src/rate/encoder_work.rs:49-69,
 * src/encoder_result.rs:31-95) once per stripe.  Synchronous.  Decode: stripe
 * i's host flag bytes at original_received + i original_received_stride /
 * recovery_received + i recovery_received_stride; only received rows travel
 * to the device and only the lost originals come back (restored in place);
 * a stripe with too few shards fails the whole call before any copy
 * (NotEnoughShards, the first such stripe). */
int rs16_encode_host_batch(rs16_engine* eng, size_t original_count, size_t recovery_count, size_t shard_bytes,
                           size_t nstripes, const void* h_original, size_t original_stride, void* h_recovery,
                           size_t recovery_stride, rs16_error* err);
int rs16_decode_host_batch(rs16_engine* eng, size_t original_count, size_t recovery_count, size_t shard_bytes,
                           size_t nstripes, void* h_original, size_t original_stride,
                           const uint8_t* original_received, size_t original_received_stride,
                           const void* h_recovery, size_t recovery_stride, const uint8_t* recovery_received,
                           size_t recovery_received_stride, rs16_error* err);

/* ---- Several GPUs in one process ------------------------
 * reed_solomon_16::encode / decode of ONE stripe with host-resident shards,
 * its byte columns split over the n engines (one per GPU): engine j takes its
 * share of the B = shard_bytes / 64 column blocks (rs16_column_slice; every
 * column block is an independent codeword, src/algorithm.md:18-32), copies
 * them in with a pitched DMA copy, runs the device codec and copies them
 * back; the engines run concurrently, with no exchange between the GPUs.
 * Synchronous.  Results are identical to rs16_encode_host / rs16_decode_host
 * (n = 1 is that call with one whole-width slice).  Decode: host flag byte
 * arrays; lost originals restored in place into h_original. */
int rs16_encode_host_multi(rs16_engine* const* engines, int n, size_t original_count, size_t recovery_count,
                           size_t shard_bytes, const void* h_original, void* h_recovery, rs16_error* err);
int rs16_decode_host_multi(rs16_engine* const* engines, int n, size_t original_count, size_t recovery_count,
                           size_t shard_bytes, void* h_original, const uint8_t* original_received,
                           const void* h_recovery, const uint8_t* recovery_received, rs16_error* err);

/* ---- RCCL over xGMI: column-slice scatter / gather -----
 * For a stripe that lives in ONE GPU's HBM (BASELINE configs[4]): the root's
 * rows x shard_bytes array is split into byte-column slices, rank r getting
 * whole 64-byte column blocks, B / n of them and one more for the first
 * B mod n ranks (B = shard_bytes / 64; rs16_column_slice), as a contiguous
 * rows x width array -- itself a shard
 * array of shard_bytes = width, so every rank runs the device codec on its
 * slice with no further exchange -- and gathered back the same way.  The
 * root packs / unpacks with pitched device copies; the slices move with one
 * grouped ncclSend / ncclRecv per other rank (the root's own slice is one
 * pitched device copy, no RCCL).  Ranks are processes (one
 * rs16_comm_new each, with the root's rs16_comm_unique_id shared out of
 * band) or engines of one process (rs16_comm_init_all).  The collective
 * calls take this process's communicators (n of them, ranks in any order)
 * with one buffer per communicator: d_full is used on the root only,
 * d_slice on every rank.  Asynchronous on `stream` (n == 1) or on each
 * engine's stream. */
typedef struct rs16_comm rs16_comm;
int rs16_comm_unique_id(void* id128, rs16_error* err);
rs16_comm* rs16_comm_new(rs16_engine* eng, int nranks, int rank, const void* id128, rs16_error* err);
int rs16_comm_init_all(rs16_engine* const* engines, int n, rs16_comm** comms, rs16_error* err);
void rs16_comm_free(rs16_comm* comm);
int rs16_comm_rank(const rs16_comm* comm);
int rs16_comm_size(const rs16_comm* comm);
/* Column slice of `rank` among `nranks`: byte offset and width (multiples of 64; width may be 0). */
int rs16_column_slice(size_t shard_bytes, int nranks, int rank, size_t* offset, size_t* width);
int rs16_scatter_columns(rs16_comm* const* comms, int n, int root, size_t rows, size_t shard_bytes,
                         const void* const* d_full, void* const* d_slice, void* stream, rs16_error* err);
int rs16_gather_columns(rs16_comm* const* comms, int n, int root, size_t rows, size_t shard_bytes,
                        const void* const* d_slice, void* const* d_full, void* stream, rs16_error* err);
/* Diagnostics: the multi-rank data path of rs16_scatter_columns /
 * rs16_gather_columns on ONE rank.  `comm` is a one-rank communicator; the
 * array is split into `vslices` column slices (rs16_column_slice with nranks =
 * vslices) that are all owned by that rank: slice 0 is the root's own (one
 * pitched copy), every other slice goes through the staging pack, one grouped
 * ncclSend / ncclRecv per slice with the rank itself as the peer, and (gather)
 * the unpack, exactly as another rank's slice would.  d_slices[j] = slice j's
 * rows x width_j buffer.  No reference counterpart (the reference has no
 * multi-GPU path); lets a one-GPU machine run the code the driver's 8-GPU
 * run depends on (tests/test_gpu_rccl.py). */
int rs16_scatter_columns_virtual(rs16_comm* comm, int vslices, size_t rows, size_t shard_bytes, const void* d_full,
                                 void* const* d_slices, void* stream, rs16_error* err);
int rs16_gather_columns_virtual(rs16_comm* comm, int vslices, size_t rows, size_t shard_bytes,
                                const void* const* d_slices, void* d_full, void* stream, rs16_error* err);

/* ---- Device memory helpers (so FFI callers need no HIP headers) ------- */
void* rs16_device_alloc(rs16_engine* eng, size_t bytes, rs16_error* err);
void rs16_device_free(rs16_engine* eng, void* d_ptr);
int rs16_memcpy_htod(rs16_engine* eng, void* d_dst, const void* src, size_t bytes, void* stream, rs16_error* err);
int rs16_memcpy_dtoh(rs16_engine* eng, void* dst, const void* d_src, size_t bytes, void* stream, rs16_error* err);
int rs16_memset_device(rs16_engine* eng, void* d_dst, int value, size_t bytes, void* stream, rs16_error* err);
/* Streams (hipStream_t, non-blocking) on the engine's device, for callers
 * without HIP headers that run codecs on streams of their own. */
void* rs16_stream_create(rs16_engine* eng, rs16_error* err);
void rs16_stream_destroy(rs16_engine* eng, void* stream);
/* Page-locked host staging memory (hipHostMalloc, portable: usable by every
 * engine of a multi-GPU call): shards that start and end
 * in host memory move over PCIe at DMA rate from/to these buffers (the
 * host-resident path of EncoderWork / DecoderWork, src/rate/encoder_work.rs:49-69). */
void* rs16_host_alloc(rs16_engine* eng, size_t bytes, rs16_error* err);
void rs16_host_free(rs16_engine* eng, void* h_ptr);

/* Diagnostics: per-kernel timing.  When enabled, every HBM pass (and the
 * eval_poly kernel group) is bracketed by hipEvents on its launch stream.
 * rs16_engine_profile_read synchronizes and returns, for pass program
 * `prog` (0 .. rs16_prog_count()-1; the last id is eval_poly), the summed
 * milliseconds and the number of launches since the last reset. */
int rs16_engine_set_profiling(rs16_engine* eng, int enable, rs16_error* err);
int rs16_engine_profile_read(rs16_engine* eng, int prog, double* total_ms, uint64_t* launches, rs16_error* err);
void rs16_engine_profile_reset(rs16_engine* eng);
int rs16_prog_count(void);
/* Diagnostics: phase timeline.  Library builds made with -DRS16_STAMPS=1
 * (scripts/stamps.py; never the shipped one) make the passes launched under
 * profiling id `prog` write 16 u64 clock stamps per workgroup to d_buf
 * (workgroup b at d_buf[16 b]); prog = -1 or d_buf = NULL turns it off.  Other
 * builds accept the call and record nothing. */
int rs16_engine_set_stamps(rs16_engine* eng, void* d_buf, int prog, rs16_error* err);
const char* rs16_prog_name(int prog);

/* Diagnostics: switches of ONE engine to alternative code paths, for tests
 * and measurements only (results are identical; 0 = the shipped paths, the
 * state of every new engine).  Returns the engine's previous flags.  There is
 * no process-wide state: other engines keep their own flags.  Like every call
 * on an engine, not to be made while another thread issues work on it. */
enum {
    RS16_DIAG_FORCE_VOFF64 = 1,    /* 64-bit per-lane HBM offsets in every pass */
    RS16_DIAG_EVAL_TWO_KERNEL = 2, /* eval_poly: the two-kernel form everywhere */
    RS16_DIAG_EVAL_FULL = 4,       /* eval_poly: the full 65536-point form for n <= 2048 */
    RS16_DIAG_NO_COLUMN = 8,       /* 512 / 1024-row transforms through the pass codec instead of
                                      the one-launch column codec */
    RS16_DIAG_FORCE_COLUMN = 16,   /* ... through the column codec at any shard width / stripe count / chunk count */
    RS16_DIAG_TILE_LAST = 32,      /* the general decode's last pass (65536 work rows) one wave per quad
                                      column of a tile at any loss count (default: <= 2048 lost) */
    RS16_DIAG_NO_TILE_LAST = 64,   /* ... always as 8-wave items of 32 quad columns */
    RS16_DIAG_FD_LDS = 128,        /* the general decode's in-tile formal derivative always through LDS */
    RS16_DIAG_COL_RADIX4 = 256,    /* column codec: 4 rows per thread everywhere (no radix-2 form) */
    RS16_DIAG_NO_IDENTITY = 512,   /* a decode whose erased rows are exactly one half of the work rows (all
                                      originals lost, all recovery received, k = m = 2^j >= 2048): evaluate
                                      the erasure polynomial and multiply anyway (default: every erasure
                                      log is 0, the multipliers are identities and are skipped) */
    RS16_DIAG_NO_MID_DIRECT = 1024 /* the general decode's middle pass always as the 2^hi-point IFFT /
                                      derivative / FFT pass, also when the lost originals lie in at most
                                      4 of its output rows per column (default there: a direct product
                                      with the pass's matrix) */
};
int rs16_engine_set_diagnostics(rs16_engine* eng, int flags);
/* Deprecated (the round-4 process-wide form, kept for existing callers):
 * sets the flags every engine created AFTER the call starts with and returns
 * the previous default.  Engines that exist keep their own flags. */
int rs16_set_diagnostics(int flags);

/* Diagnostics: host-side evaluation of the device multiply (same v_perm
 * byte-table format and code path as the kernels, with v_perm emulated):
 * out[] = in[] * log_m for `bytes` (multiple of 64) bytes of shard data, with
 * Engine::mul semantics (log_m 65535 == x1).  Lets CPU-only tests check the
 * table format against the reference multiply (NoSimd::mul). */
void rs16_host_mul(const void* in, void* out, size_t bytes, uint16_t log_m);

/* Library/build identification, e.g. "rs16-mi355x gfx950". */
const char* rs16_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RS16_H */
