/*
 * rs16_oracle.c -- CPU ORACLE. TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle and the CPU baseline for the MI355X codec.
 * It is a plain-C restatement of the reference crate malaire/reed-solomon-16
 * v0.1.0 (Rust; no Rust toolchain exists in this image, so the reference
 * itself cannot be built -- see DESIGN.md "Oracle").  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / baseline.  Nothing in reed-solomon-16_amd/ links it.
 *
 * Parity pinning: tests/test_oracle_golden.py checks every SHA-256 recovery
 * hash of /root/reference/src/test_util.rs:583-837 (DEFAULT_TINY, HIGH_TINY,
 * LOW_TINY and the named large constants) against BOTH engines restated
 * here (Naive and NoSimd), exactly as the reference's roundtrip_single!
 * macro does (src/test_util.rs:173-205).  The vectors are committed as data
 * in tests/golden/reference_hashes.json.
 *
 * Every function cites the reference file:line it follows.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* GF constants -- src/engine.rs:59-74                                 */
/* ------------------------------------------------------------------ */
#define GF_BITS 16
#define GF_ORDER 65536u
#define GF_MODULUS 65535u
#define GF_POLYNOMIAL 0x1002Du

static const uint16_t CANTOR_BASIS[GF_BITS] = {
    0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
    0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E,
};

/* add_mod / sub_mod -- src/engine.rs:90-100 */
static inline uint16_t add_mod(uint16_t x, uint16_t y) {
    uint64_t sum = (uint64_t)x + (uint64_t)y;
    return (uint16_t)(sum + (sum >> GF_BITS));
}
static inline uint16_t sub_mod(uint16_t x, uint16_t y) {
    uint64_t dif = (uint64_t)x - (uint64_t)y; /* wrapping_sub on usize */
    return (uint16_t)(dif + (dif >> GF_BITS));
}

static size_t next_pow2(size_t x) { /* usize::next_power_of_two */
    size_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

/* ------------------------------------------------------------------ */
/* Tables -- src/engine/tables.rs                                      */
/* ------------------------------------------------------------------ */
static uint16_t *g_exp, *g_log, *g_skew, *g_log_walsh;
static uint16_t (*g_mul16)[4][16];
static int g_init_done;

/* tables::mul -- src/engine/tables.rs:70-76 */
static inline uint16_t tmul(uint16_t x, uint16_t log_m) {
    return x == 0 ? 0 : g_exp[add_mod(g_log[x], log_m)];
}

/* initialize_exp_log -- src/engine/tables.rs:83-124 */
static void init_exp_log(void) {
    g_exp = calloc(GF_ORDER, 2);
    g_log = calloc(GF_ORDER, 2);
    size_t state = 1;
    for (uint32_t i = 0; i < GF_MODULUS; i++) {
        g_exp[state] = (uint16_t)i;
        state <<= 1;
        if (state >= GF_ORDER) state ^= GF_POLYNOMIAL;
    }
    g_exp[0] = GF_MODULUS;
    g_log[0] = 0;
    for (int i = 0; i < GF_BITS; i++) {
        size_t width = (size_t)1 << i;
        for (size_t j = 0; j < width; j++) g_log[j + width] = g_log[j] ^ CANTOR_BASIS[i];
    }
    for (size_t i = 0; i < GF_ORDER; i++) g_log[i] = g_exp[g_log[i]];
    for (size_t i = 0; i < GF_ORDER; i++) g_exp[g_log[i]] = (uint16_t)i;
    g_exp[GF_MODULUS] = g_exp[0];
}

/* initialize_mul16 -- src/engine/tables.rs:142-160 */
static void init_mul16(void) {
    g_mul16 = calloc(GF_ORDER, sizeof *g_mul16);
    for (uint32_t log_m = 0; log_m <= GF_MODULUS; log_m++) {
        for (uint32_t i = 0; i < 16; i++) {
            g_mul16[log_m][0][i] = tmul((uint16_t)i, (uint16_t)log_m);
            g_mul16[log_m][1][i] = tmul((uint16_t)(i << 4), (uint16_t)log_m);
            g_mul16[log_m][2][i] = tmul((uint16_t)(i << 8), (uint16_t)log_m);
            g_mul16[log_m][3][i] = tmul((uint16_t)(i << 12), (uint16_t)log_m);
        }
    }
}

/* initialize_skew -- src/engine/tables.rs:164-205 */
static void init_skew(void) {
    g_skew = calloc(GF_MODULUS, 2);
    uint16_t temp[GF_BITS - 1];
    for (int i = 1; i < GF_BITS; i++) temp[i - 1] = (uint16_t)(1u << i);
    for (int m = 0; m < GF_BITS - 1; m++) {
        size_t step = (size_t)1 << (m + 1);
        g_skew[((size_t)1 << m) - 1] = 0;
        for (int i = m; i < GF_BITS - 1; i++) {
            size_t s = (size_t)1 << (i + 1);
            for (size_t j = ((size_t)1 << m) - 1; j < s; j += step) g_skew[j + s] = g_skew[j] ^ temp[i];
        }
        temp[m] = (uint16_t)(GF_MODULUS - g_log[tmul(temp[m], g_log[temp[m] ^ 1])]);
        for (int i = m + 1; i < GF_BITS - 1; i++) {
            uint16_t sum = add_mod(g_log[temp[i] ^ 1], temp[m]);
            temp[i] = tmul(temp[i], sum);
        }
    }
    for (size_t i = 0; i < GF_MODULUS; i++) g_skew[i] = g_log[g_skew[i]];
}

/* ------------------------------------------------------------------ */
/* Engines: Naive (src/engine/engine_naive.rs) and NoSimd              */
/* (src/engine/engine_nosimd.rs).                                       */
/* Data view = ShardsRefMut (src/engine/shards.rs:60-66): flat bytes,   */
/* shard i at data + i*shard_bytes.                                     */
/* ------------------------------------------------------------------ */
enum { ENGINE_NAIVE = 0, ENGINE_NOSIMD = 1 };

#define SHARD(data, sb, i) ((data) + (size_t)(i) * (sb))

/* Naive::xor -- src/engine/engine_naive.rs:143-152 */
static void naive_xor(uint8_t *x, const uint8_t *y, size_t n) {
    for (size_t i = 0; i < n; i++) x[i] ^= y[i];
}
/* NoSimd::xor -- src/engine/engine_nosimd.rs:81-88 (u64 words) */
static void nosimd_xor(uint8_t *x, const uint8_t *y, size_t n) {
    for (size_t i = 0; i < n; i += 8) {
        uint64_t a, b;
        memcpy(&a, x + i, 8);
        memcpy(&b, y + i, 8);
        a ^= b;
        memcpy(x + i, &a, 8);
    }
}
static void eng_xor(int eng, uint8_t *x, const uint8_t *y, size_t n) {
    if (eng == ENGINE_NAIVE) naive_xor(x, y, n); else nosimd_xor(x, y, n);
}

/* Naive::mul -- src/engine/engine_naive.rs:126-141 */
static void naive_mul(uint8_t *x, size_t n, uint16_t log_m) {
    for (size_t pos = 0; pos < n; pos += 64)
        for (int i = 0; i < 32; i++) {
            uint16_t v = (uint16_t)(x[pos + i] | (x[pos + i + 32] << 8));
            uint16_t prod = tmul(v, log_m);
            x[pos + i] = (uint8_t)prod;
            x[pos + i + 32] = (uint8_t)(prod >> 8);
        }
}
/* Naive::mul_add -- src/engine/engine_naive.rs:168-184 */
static void naive_mul_add(uint8_t *x, const uint8_t *y, size_t n, uint16_t log_m) {
    for (size_t pos = 0; pos < n; pos += 64)
        for (int i = 0; i < 32; i++) {
            uint16_t v = (uint16_t)(y[pos + i] | (y[pos + i + 32] << 8));
            uint16_t prod = tmul(v, log_m);
            x[pos + i] ^= (uint8_t)prod;
            x[pos + i + 32] ^= (uint8_t)(prod >> 8);
        }
}
/* NoSimd::mul -- src/engine/engine_nosimd.rs:65-79 */
static void nosimd_mul(uint8_t *x, size_t n, uint16_t log_m) {
    const uint16_t (*lut)[16] = g_mul16[log_m];
    for (size_t pos = 0; pos < n; pos += 64)
        for (int i = 0; i < 32; i++) {
            unsigned lo = x[pos + i], hi = x[pos + i + 32];
            uint16_t prod = lut[0][lo & 15] ^ lut[1][lo >> 4] ^ lut[2][hi & 15] ^ lut[3][hi >> 4];
            x[pos + i] = (uint8_t)prod;
            x[pos + i + 32] = (uint8_t)(prod >> 8);
        }
}
/* NoSimd::mul_add -- src/engine/engine_nosimd.rs:105-119 */
static void nosimd_mul_add(uint8_t *x, const uint8_t *y, size_t n, uint16_t log_m) {
    const uint16_t (*lut)[16] = g_mul16[log_m];
    for (size_t pos = 0; pos < n; pos += 64)
        for (int i = 0; i < 32; i++) {
            unsigned lo = y[pos + i], hi = y[pos + i + 32];
            uint16_t prod = lut[0][lo & 15] ^ lut[1][lo >> 4] ^ lut[2][hi & 15] ^ lut[3][hi >> 4];
            x[pos + i] ^= (uint8_t)prod;
            x[pos + i + 32] ^= (uint8_t)(prod >> 8);
        }
}
static void eng_mul(int eng, uint8_t *x, size_t n, uint16_t log_m) {
    if (eng == ENGINE_NAIVE) naive_mul(x, n, log_m); else nosimd_mul(x, n, log_m);
}

/* Naive::fft -- src/engine/engine_naive.rs:43-73 */
static void naive_fft(uint8_t *d, size_t sb, size_t pos, size_t size, size_t trunc, size_t skew_delta) {
    for (size_t dist = size / 2; dist > 0; dist /= 2)
        for (size_t r = 0; r < trunc; r += dist * 2) {
            uint16_t log_m = g_skew[r + dist + skew_delta - 1];
            for (size_t i = r; i < r + dist; i++) {
                uint8_t *a = SHARD(d, sb, pos + i), *b = SHARD(d, sb, pos + i + dist);
                if (log_m != GF_MODULUS) naive_mul_add(a, b, sb, log_m);
                naive_xor(b, a, sb);
            }
        }
}
/* Naive::ifft -- src/engine/engine_naive.rs:94-124 */
static void naive_ifft(uint8_t *d, size_t sb, size_t pos, size_t size, size_t trunc, size_t skew_delta) {
    for (size_t dist = 1; dist < size; dist *= 2)
        for (size_t r = 0; r < trunc; r += dist * 2) {
            uint16_t log_m = g_skew[r + dist + skew_delta - 1];
            for (size_t i = r; i < r + dist; i++) {
                uint8_t *a = SHARD(d, sb, pos + i), *b = SHARD(d, sb, pos + i + dist);
                naive_xor(b, a, sb);
                if (log_m != GF_MODULUS) naive_mul_add(a, b, sb, log_m);
            }
        }
}
/* Naive::fwht -- src/engine/engine_naive.rs:75-92 */
static void naive_fwht(uint16_t *data, size_t trunc) {
    for (size_t dist = 1; dist < GF_ORDER; dist *= 2)
        for (size_t r = 0; r < trunc; r += dist * 2)
            for (size_t i = r; i < r + dist; i++) {
                uint16_t sum = add_mod(data[i], data[i + dist]);
                uint16_t dif = sub_mod(data[i], data[i + dist]);
                data[i] = sum;
                data[i + dist] = dif;
            }
}

/* NoSimd fft_butterfly_partial / two_layers / fft_private --
 * src/engine/engine_nosimd.rs:190-284 */
static void nosimd_fft_bfly(uint8_t *x, uint8_t *y, size_t sb, uint16_t log_m) {
    nosimd_mul_add(x, y, sb, log_m);
    nosimd_xor(y, x, sb);
}
static void nosimd_fft(uint8_t *d, size_t sb, size_t pos, size_t size, size_t trunc, size_t skew_delta) {
    size_t dist4 = size, dist = size >> 2;
    while (dist != 0) {
        for (size_t r = 0; r < trunc; r += dist4) {
            size_t base = r + dist + skew_delta - 1;
            uint16_t log_m01 = g_skew[base];
            uint16_t log_m02 = g_skew[base + dist];
            uint16_t log_m23 = g_skew[base + dist * 2];
            for (size_t i = r; i < r + dist; i++) {
                uint8_t *s0 = SHARD(d, sb, pos + i), *s1 = SHARD(d, sb, pos + i + dist);
                uint8_t *s2 = SHARD(d, sb, pos + i + 2 * dist), *s3 = SHARD(d, sb, pos + i + 3 * dist);
                if (log_m02 == GF_MODULUS) {
                    nosimd_xor(s2, s0, sb);
                    nosimd_xor(s3, s1, sb);
                } else {
                    nosimd_fft_bfly(s0, s2, sb, log_m02);
                    nosimd_fft_bfly(s1, s3, sb, log_m02);
                }
                if (log_m01 == GF_MODULUS) nosimd_xor(s1, s0, sb); else nosimd_fft_bfly(s0, s1, sb, log_m01);
                if (log_m23 == GF_MODULUS) nosimd_xor(s3, s2, sb); else nosimd_fft_bfly(s2, s3, sb, log_m23);
            }
        }
        dist4 = dist;
        dist >>= 2;
    }
    if (dist4 == 2) {
        for (size_t r = 0; r < trunc; r += 2) {
            uint16_t log_m = g_skew[r + skew_delta];
            uint8_t *x = SHARD(d, sb, pos + r), *y = SHARD(d, sb, pos + r + 1);
            if (log_m == GF_MODULUS) nosimd_xor(y, x, sb); else nosimd_fft_bfly(x, y, sb, log_m);
        }
    }
}
/* NoSimd ifft_butterfly_partial / two_layers / ifft_private --
 * src/engine/engine_nosimd.rs:291-384 */
static void nosimd_ifft_bfly(uint8_t *x, uint8_t *y, size_t sb, uint16_t log_m) {
    nosimd_xor(y, x, sb);
    nosimd_mul_add(x, y, sb, log_m);
}
static void nosimd_ifft(uint8_t *d, size_t sb, size_t pos, size_t size, size_t trunc, size_t skew_delta) {
    size_t dist = 1, dist4 = 4;
    while (dist4 <= size) {
        for (size_t r = 0; r < trunc; r += dist4) {
            size_t base = r + dist + skew_delta - 1;
            uint16_t log_m01 = g_skew[base];
            uint16_t log_m02 = g_skew[base + dist];
            uint16_t log_m23 = g_skew[base + dist * 2];
            for (size_t i = r; i < r + dist; i++) {
                uint8_t *s0 = SHARD(d, sb, pos + i), *s1 = SHARD(d, sb, pos + i + dist);
                uint8_t *s2 = SHARD(d, sb, pos + i + 2 * dist), *s3 = SHARD(d, sb, pos + i + 3 * dist);
                if (log_m01 == GF_MODULUS) nosimd_xor(s1, s0, sb); else nosimd_ifft_bfly(s0, s1, sb, log_m01);
                if (log_m23 == GF_MODULUS) nosimd_xor(s3, s2, sb); else nosimd_ifft_bfly(s2, s3, sb, log_m23);
                if (log_m02 == GF_MODULUS) {
                    nosimd_xor(s2, s0, sb);
                    nosimd_xor(s3, s1, sb);
                } else {
                    nosimd_ifft_bfly(s0, s2, sb, log_m02);
                    nosimd_ifft_bfly(s1, s3, sb, log_m02);
                }
            }
        }
        dist = dist4;
        dist4 <<= 2;
    }
    if (dist < size) {
        uint16_t log_m = g_skew[dist + skew_delta - 1];
        if (log_m == GF_MODULUS) {
            nosimd_xor(SHARD(d, sb, pos + dist), SHARD(d, sb, pos), dist * sb); /* xor_within */
        } else {
            for (size_t i = 0; i < dist; i++)
                nosimd_ifft_bfly(SHARD(d, sb, pos + i), SHARD(d, sb, pos + i + dist), sb, log_m);
        }
    }
}
/* NoSimd::fwht_private -- src/engine/engine_nosimd.rs:121-183 */
static void nosimd_fwht(uint16_t *data, size_t trunc) {
    size_t dist = 1, dist4 = 4;
    while (dist4 <= GF_ORDER) {
        for (size_t r = 0; r < trunc; r += dist4)
            for (size_t i = r; i < r + dist; i++) {
                uint16_t t0 = data[i], t1 = data[i + dist], t2 = data[i + dist * 2], t3 = data[i + dist * 3];
                uint16_t s, f;
                s = add_mod(t0, t1); f = sub_mod(t0, t1); t0 = s; t1 = f;
                s = add_mod(t2, t3); f = sub_mod(t2, t3); t2 = s; t3 = f;
                s = add_mod(t0, t2); f = sub_mod(t0, t2); t0 = s; t2 = f;
                s = add_mod(t1, t3); f = sub_mod(t1, t3); t1 = s; t3 = f;
                data[i] = t0; data[i + dist] = t1; data[i + dist * 2] = t2; data[i + dist * 3] = t3;
            }
        dist = dist4;
        dist4 <<= 2;
    }
    if (dist < GF_ORDER)
        for (size_t i = 0; i < dist; i++) {
            uint16_t sum = add_mod(data[i], data[i + dist]);
            uint16_t dif = sub_mod(data[i], data[i + dist]);
            data[i] = sum;
            data[i + dist] = dif;
        }
}

static void eng_fft(int eng, uint8_t *d, size_t sb, size_t pos, size_t size, size_t trunc, size_t sd) {
    if (eng == ENGINE_NAIVE) naive_fft(d, sb, pos, size, trunc, sd); else nosimd_fft(d, sb, pos, size, trunc, sd);
}
static void eng_ifft(int eng, uint8_t *d, size_t sb, size_t pos, size_t size, size_t trunc, size_t sd) {
    if (eng == ENGINE_NAIVE) naive_ifft(d, sb, pos, size, trunc, sd); else nosimd_ifft(d, sb, pos, size, trunc, sd);
}
static void eng_fwht(int eng, uint16_t *data, size_t trunc) {
    if (eng == ENGINE_NAIVE) naive_fwht(data, trunc); else nosimd_fwht(data, trunc);
}

/* initialize_log_walsh::<E> -- src/engine/tables.rs:127-139.  Both
 * engines' fwht give the same table; built with NoSimd once. */
static void init_log_walsh(void) {
    g_log_walsh = calloc(GF_ORDER, 2);
    memcpy(g_log_walsh, g_log, GF_ORDER * 2);
    g_log_walsh[0] = 0;
    nosimd_fwht(g_log_walsh, GF_ORDER);
}

/* Engine::eval_poly -- src/engine.rs:207-218 */
static void eng_eval_poly(int eng, uint16_t *e, size_t trunc) {
    eng_fwht(eng, e, trunc);
    for (size_t i = 0; i < GF_ORDER; i++)
        e[i] = (uint16_t)(((uint64_t)e[i] * (uint64_t)g_log_walsh[i]) % GF_MODULUS);
    eng_fwht(eng, e, GF_ORDER);
}
/* Engine::xor_within -- src/engine.rs:256-259 (non-overlapping ranges) */
static void eng_xor_within(int eng, uint8_t *d, size_t sb, size_t x, size_t y, size_t count) {
    eng_xor(eng, SHARD(d, sb, x), SHARD(d, sb, y), count * sb);
}
/* Engine::formal_derivative -- src/engine.rs:233-238 */
static void eng_formal_derivative(int eng, uint8_t *d, size_t sb, size_t len) {
    for (size_t i = 1; i < len; i++) {
        size_t width = ((i ^ (i - 1)) + 1) >> 1;
        eng_xor_within(eng, d, sb, i - width, i, width);
    }
}

void oracle_init(void) {
    if (g_init_done) return;
    init_exp_log();
    init_mul16();
    init_skew();
    init_log_walsh();
    g_init_done = 1;
}

/* ------------------------------------------------------------------ */
/* Errors -- src/lib.rs:31-125 (same variants, same payload fields)   */
/* ------------------------------------------------------------------ */
typedef struct {
    int32_t code;
    uint64_t a, b, c;
} oracle_error;
enum {
    E_OK = 0,
    E_DIFFERENT_SHARD_SIZE = 1,          /* shard_bytes, got */
    E_DUPLICATE_ORIGINAL_SHARD_INDEX = 2, /* index */
    E_DUPLICATE_RECOVERY_SHARD_INDEX = 3, /* index */
    E_INVALID_ORIGINAL_SHARD_INDEX = 4,   /* original_count, index */
    E_INVALID_RECOVERY_SHARD_INDEX = 5,   /* recovery_count, index */
    E_INVALID_SHARD_SIZE = 6,             /* shard_bytes */
    E_NOT_ENOUGH_SHARDS = 7,              /* original_count, orig_recv, rec_recv */
    E_TOO_FEW_ORIGINAL_SHARDS = 8,        /* original_count, orig_recv */
    E_TOO_MANY_ORIGINAL_SHARDS = 9,       /* original_count */
    E_UNSUPPORTED_SHARD_COUNT = 10,       /* original_count, recovery_count */
};
static int set_err(oracle_error *e, int code, uint64_t a, uint64_t b, uint64_t c) {
    if (e) { e->code = code; e->a = a; e->b = b; e->c = c; }
    return code;
}

/* ------------------------------------------------------------------ */
/* Rates -- src/rate.rs, src/rate/rate_{high,low,default}.rs          */
/* ------------------------------------------------------------------ */
enum { RATE_DEFAULT = 0, RATE_HIGH = 1, RATE_LOW = 2 };

/* HighRate::supports -- src/rate/rate_high.rs:19-25 */
static int high_supports(size_t k, size_t m) {
    return k > 0 && m > 0 && k < GF_ORDER && m < GF_ORDER && next_pow2(m) + k <= GF_ORDER;
}
/* LowRate::supports -- src/rate/rate_low.rs:19-25 */
static int low_supports(size_t k, size_t m) {
    return k > 0 && m > 0 && k < GF_ORDER && m < GF_ORDER && next_pow2(k) + m <= GF_ORDER;
}
/* use_high_rate -- src/rate/rate_default.rs:15-64.  Returns 1/0 or -1 (error). */
int oracle_use_high_rate(size_t k, size_t m, oracle_error *err) {
    if (k > GF_ORDER || m > GF_ORDER) { set_err(err, E_UNSUPPORTED_SHARD_COUNT, k, m, 0); return -1; }
    size_t kp = next_pow2(k), mp = next_pow2(m);
    size_t smaller = kp < mp ? kp : mp;
    size_t larger = k > m ? k : m;
    if (k == 0 || m == 0 || smaller + larger > GF_ORDER) { set_err(err, E_UNSUPPORTED_SHARD_COUNT, k, m, 0); return -1; }
    if (kp < mp) return 0;
    if (kp > mp) return 1;
    return k <= m ? 1 : 0;
}
int oracle_supports(int rate, size_t k, size_t m) {
    if (rate == RATE_HIGH) return high_supports(k, m);
    if (rate == RATE_LOW) return low_supports(k, m);
    return oracle_use_high_rate(k, m, NULL) >= 0;
}
/* Rate::validate -- src/rate.rs:91-106 */
int oracle_validate(int rate, size_t k, size_t m, size_t sb, oracle_error *err) {
    if (!oracle_supports(rate, k, m)) return set_err(err, E_UNSUPPORTED_SHARD_COUNT, k, m, 0);
    if (sb == 0 || (sb & 63) != 0) return set_err(err, E_INVALID_SHARD_SIZE, sb, 0, 0);
    return set_err(err, E_OK, 0, 0, 0);
}
/* work_count -- src/rate/rate_high.rs:131-137, 301-305; src/rate/rate_low.rs:131-137, 301-305 */
size_t oracle_encoder_work_count(int high, size_t k, size_t m) {
    size_t chunk = high ? next_pow2(m) : next_pow2(k);
    size_t n = high ? k : m;
    return (n + chunk - 1) / chunk * chunk;
}
size_t oracle_decoder_work_count(int high, size_t k, size_t m) {
    return high ? next_pow2(next_pow2(m) + k) : next_pow2(next_pow2(k) + m);
}

/* --- Encoder (EncoderWork src/rate/encoder_work.rs + HighRateEncoder /
 *     LowRateEncoder / DefaultRateEncoder) --- */
typedef struct {
    int rate_kind; /* RATE_DEFAULT / RATE_HIGH / RATE_LOW as requested */
    int high;      /* resolved rate */
    int engine;
    size_t k, m, sb;
    size_t received;
    size_t work_count;
    uint8_t *work;
    size_t work_cap;
} oracle_encoder;

static int encoder_reset_impl(oracle_encoder *e, size_t k, size_t m, size_t sb, oracle_error *err) {
    int high;
    if (e->rate_kind == RATE_DEFAULT) {
        high = oracle_use_high_rate(k, m, err);
        if (high < 0) return err ? err->code : E_UNSUPPORTED_SHARD_COUNT;
    } else {
        high = e->rate_kind == RATE_HIGH;
    }
    int rc = oracle_validate(high ? RATE_HIGH : RATE_LOW, k, m, sb, err);
    if (rc) return rc;
    /* EncoderWork::reset -- src/rate/encoder_work.rs:95-108 */
    e->high = high;
    e->k = k; e->m = m; e->sb = sb;
    e->received = 0;
    e->work_count = oracle_encoder_work_count(high, k, m);
    size_t need = e->work_count * sb;
    if (need > e->work_cap) {
        e->work = realloc(e->work, need);
        memset(e->work + e->work_cap, 0, need - e->work_cap);
        e->work_cap = need;
    }
    return set_err(err, E_OK, 0, 0, 0);
}

oracle_encoder *oracle_encoder_new(int rate, int engine, size_t k, size_t m, size_t sb, oracle_error *err) {
    oracle_init();
    oracle_encoder *e = calloc(1, sizeof *e);
    e->rate_kind = rate;
    e->engine = engine;
    if (encoder_reset_impl(e, k, m, sb, err)) { free(e->work); free(e); return NULL; }
    return e;
}
int oracle_encoder_reset(oracle_encoder *e, size_t k, size_t m, size_t sb, oracle_error *err) {
    return encoder_reset_impl(e, k, m, sb, err);
}
void oracle_encoder_free(oracle_encoder *e) { if (e) { free(e->work); free(e); } }

/* EncoderWork::add_original_shard -- src/rate/encoder_work.rs:49-69 */
int oracle_encoder_add_original_shard(oracle_encoder *e, const uint8_t *shard, size_t len, oracle_error *err) {
    if (e->received == e->k) return set_err(err, E_TOO_MANY_ORIGINAL_SHARDS, e->k, 0, 0);
    if (len != e->sb) return set_err(err, E_DIFFERENT_SHARD_SIZE, e->sb, len, 0);
    memcpy(SHARD(e->work, e->sb, e->received), shard, len);
    e->received++;
    return set_err(err, E_OK, 0, 0, 0);
}

/* HighRateEncoder::encode -- src/rate/rate_high.rs:44-83 */
static void high_encode(oracle_encoder *e) {
    uint8_t *w = e->work;
    size_t sb = e->sb, k = e->k, m = e->m, chunk = next_pow2(m);
    int eng = e->engine;
    size_t first = k < chunk ? k : chunk;
    memset(SHARD(w, sb, first), 0, (chunk - first) * sb);
    eng_ifft(eng, w, sb, 0, chunk, first, chunk); /* ifft_skew_end */
    if (k > chunk) {
        size_t cs = chunk;
        while (cs + chunk <= k) {
            eng_ifft(eng, w, sb, cs, chunk, chunk, cs + chunk);
            eng_xor_within(eng, w, sb, 0, cs, chunk);
            cs += chunk;
        }
        size_t last = k % chunk;
        if (last > 0) {
            memset(SHARD(w, sb, cs + last), 0, (e->work_count - cs - last) * sb);
            eng_ifft(eng, w, sb, cs, chunk, last, cs + chunk);
            eng_xor_within(eng, w, sb, 0, cs, chunk);
        }
    }
    eng_fft(eng, w, sb, 0, chunk, m, 0);
}
/* LowRateEncoder::encode -- src/rate/rate_low.rs:44-83 */
static void low_encode(oracle_encoder *e) {
    uint8_t *w = e->work;
    size_t sb = e->sb, k = e->k, m = e->m, chunk = next_pow2(k);
    int eng = e->engine;
    memset(SHARD(w, sb, k), 0, (chunk - k) * sb);
    eng_ifft(eng, w, sb, 0, chunk, k, 0);
    for (size_t cs = chunk; cs < m; cs += chunk) memmove(SHARD(w, sb, cs), w, chunk * sb); /* copy_within */
    size_t cs = 0;
    while (cs + chunk <= m) {
        eng_fft(eng, w, sb, cs, chunk, chunk, cs + chunk); /* fft_skew_end */
        cs += chunk;
    }
    size_t last = m % chunk;
    if (last > 0) eng_fft(eng, w, sb, cs, chunk, last, cs + chunk);
}
/* encode_begin -- src/rate/encoder_work.rs:71-84 */
int oracle_encoder_encode(oracle_encoder *e, oracle_error *err) {
    if (e->received != e->k) return set_err(err, E_TOO_FEW_ORIGINAL_SHARDS, e->k, e->received, 0);
    if (e->high) high_encode(e); else low_encode(e);
    return set_err(err, E_OK, 0, 0, 0);
}
/* EncoderWork::recovery -- src/rate/encoder_work.rs:87-93 */
const uint8_t *oracle_encoder_recovery(oracle_encoder *e, size_t index) {
    return index < e->m ? SHARD(e->work, e->sb, index) : NULL;
}
/* EncoderWork::reset_received (EncoderResult Drop) -- src/rate/encoder_work.rs:110-112 */
void oracle_encoder_reset_received(oracle_encoder *e) { e->received = 0; }
int oracle_encoder_is_high(oracle_encoder *e) { return e->high; }

/* --- Decoder (DecoderWork src/rate/decoder_work.rs + High/Low/Default
 *     rate decoders) --- */
typedef struct {
    int rate_kind, high, engine;
    size_t k, m, sb;
    size_t orig_base, rec_base;
    size_t orig_recv, rec_recv;
    size_t work_count;
    uint8_t *received; /* byte per position, len work_count */
    size_t recv_cap;
    uint8_t *work;
    size_t work_cap;
} oracle_decoder;

static int decoder_reset_impl(oracle_decoder *d, size_t k, size_t m, size_t sb, oracle_error *err) {
    int high;
    if (d->rate_kind == RATE_DEFAULT) {
        high = oracle_use_high_rate(k, m, err);
        if (high < 0) return err ? err->code : E_UNSUPPORTED_SHARD_COUNT;
    } else {
        high = d->rate_kind == RATE_HIGH;
    }
    int rc = oracle_validate(high ? RATE_HIGH : RATE_LOW, k, m, sb, err);
    if (rc) return rc;
    /* DecoderWork::reset -- src/rate/decoder_work.rs:145-176;
     * layouts: src/rate/rate_high.rs:279-299, src/rate/rate_low.rs:279-299 */
    d->high = high;
    d->k = k; d->m = m; d->sb = sb;
    d->orig_base = high ? next_pow2(m) : 0;
    d->rec_base = high ? 0 : next_pow2(k);
    d->orig_recv = d->rec_recv = 0;
    d->work_count = oracle_decoder_work_count(high, k, m);
    if (d->work_count > d->recv_cap) {
        d->received = realloc(d->received, d->work_count);
        d->recv_cap = d->work_count;
    }
    memset(d->received, 0, d->recv_cap);
    size_t need = d->work_count * sb;
    if (need > d->work_cap) {
        d->work = realloc(d->work, need);
        memset(d->work + d->work_cap, 0, need - d->work_cap);
        d->work_cap = need;
    }
    return set_err(err, E_OK, 0, 0, 0);
}
oracle_decoder *oracle_decoder_new(int rate, int engine, size_t k, size_t m, size_t sb, oracle_error *err) {
    oracle_init();
    oracle_decoder *d = calloc(1, sizeof *d);
    d->rate_kind = rate;
    d->engine = engine;
    if (decoder_reset_impl(d, k, m, sb, err)) { free(d->work); free(d->received); free(d); return NULL; }
    return d;
}
int oracle_decoder_reset(oracle_decoder *d, size_t k, size_t m, size_t sb, oracle_error *err) {
    return decoder_reset_impl(d, k, m, sb, err);
}
void oracle_decoder_free(oracle_decoder *d) { if (d) { free(d->work); free(d->received); free(d); } }

/* DecoderWork::add_original_shard -- src/rate/decoder_work.rs:62-88 */
int oracle_decoder_add_original_shard(oracle_decoder *d, size_t index, const uint8_t *shard, size_t len, oracle_error *err) {
    size_t pos = d->orig_base + index;
    if (index >= d->k) return set_err(err, E_INVALID_ORIGINAL_SHARD_INDEX, d->k, index, 0);
    if (d->received[pos]) return set_err(err, E_DUPLICATE_ORIGINAL_SHARD_INDEX, index, 0, 0);
    if (len != d->sb) return set_err(err, E_DIFFERENT_SHARD_SIZE, d->sb, len, 0);
    memcpy(SHARD(d->work, d->sb, pos), shard, len);
    d->orig_recv++;
    d->received[pos] = 1;
    return set_err(err, E_OK, 0, 0, 0);
}
/* DecoderWork::add_recovery_shard -- src/rate/decoder_work.rs:90-116 */
int oracle_decoder_add_recovery_shard(oracle_decoder *d, size_t index, const uint8_t *shard, size_t len, oracle_error *err) {
    size_t pos = d->rec_base + index;
    if (index >= d->m) return set_err(err, E_INVALID_RECOVERY_SHARD_INDEX, d->m, index, 0);
    if (d->received[pos]) return set_err(err, E_DUPLICATE_RECOVERY_SHARD_INDEX, index, 0, 0);
    if (len != d->sb) return set_err(err, E_DIFFERENT_SHARD_SIZE, d->sb, len, 0);
    memcpy(SHARD(d->work, d->sb, pos), shard, len);
    d->rec_recv++;
    d->received[pos] = 1;
    return set_err(err, E_OK, 0, 0, 0);
}

/* HighRateDecoder::decode -- src/rate/rate_high.rs:168-247 and
 * LowRateDecoder::decode -- src/rate/rate_low.rs:168-247.
 * Layout: [a_base, a_base + a_count) = first block (recovery for high,
 * original for low), [chunk, chunk + b_count) = second block. */
static void rate_decode(oracle_decoder *d) {
    size_t sb = d->sb, n = d->work_count;
    size_t a_count = d->high ? d->m : d->k;
    size_t b_count = d->high ? d->k : d->m;
    size_t chunk = next_pow2(a_count);
    size_t end = chunk + b_count;
    uint8_t *w = d->work;
    int eng = d->engine;
    uint16_t *er = calloc(GF_ORDER, 2);
    for (size_t i = 0; i < a_count; i++) if (!d->received[i]) er[i] = 1;
    if (d->high) for (size_t i = a_count; i < chunk; i++) er[i] = 1;
    for (size_t i = chunk; i < end; i++) if (!d->received[i]) er[i] = 1;
    if (!d->high) for (size_t i = end; i < GF_ORDER; i++) er[i] = 1;
    eng_eval_poly(eng, er, d->high ? end : GF_ORDER);
    for (size_t i = 0; i < a_count; i++) {
        if (d->received[i]) eng_mul(eng, SHARD(w, sb, i), sb, er[i]);
        else memset(SHARD(w, sb, i), 0, sb);
    }
    memset(SHARD(w, sb, a_count), 0, (chunk - a_count) * sb);
    for (size_t i = chunk; i < end; i++) {
        if (d->received[i]) eng_mul(eng, SHARD(w, sb, i), sb, er[i]);
        else memset(SHARD(w, sb, i), 0, sb);
    }
    memset(SHARD(w, sb, end), 0, (n - end) * sb);
    eng_ifft(eng, w, sb, 0, n, end, 0);
    eng_formal_derivative(eng, w, sb, n);
    eng_fft(eng, w, sb, 0, n, end, 0);
    /* reveal erasures: lost originals */
    size_t ob = d->orig_base;
    for (size_t i = ob; i < ob + d->k; i++)
        if (!d->received[i]) eng_mul(eng, SHARD(w, sb, i), sb, (uint16_t)(GF_MODULUS - er[i]));
    free(er);
}
/* decode_begin -- src/rate/decoder_work.rs:120-139 */
int oracle_decoder_decode(oracle_decoder *d, oracle_error *err) {
    if (d->orig_recv + d->rec_recv < d->k)
        return set_err(err, E_NOT_ENOUGH_SHARDS, d->k, d->orig_recv, d->rec_recv);
    if (d->orig_recv == d->k) return set_err(err, E_OK, 0, 0, 0); /* nothing to do */
    rate_decode(d);
    return set_err(err, E_OK, 0, 0, 0);
}
/* DecoderWork::restored_original -- src/rate/decoder_work.rs:185-193 */
const uint8_t *oracle_decoder_restored_original(oracle_decoder *d, size_t index) {
    size_t pos = d->orig_base + index;
    if (index < d->k && !d->received[pos]) return SHARD(d->work, d->sb, pos);
    return NULL;
}
/* DecoderWork::reset_received (DecoderResult Drop) -- src/rate/decoder_work.rs:178-183 */
void oracle_decoder_reset_received(oracle_decoder *d) {
    d->orig_recv = d->rec_recv = 0;
    memset(d->received, 0, d->recv_cap);
}
int oracle_decoder_is_high(oracle_decoder *d) { return d->high; }

/* ------------------------------------------------------------------ */
/* Engine-level entry points (for engine parity tests)                 */
/* ------------------------------------------------------------------ */
void oracle_fft(int eng, uint8_t *d, size_t sb, size_t pos, size_t size, size_t trunc, size_t sd) {
    oracle_init(); eng_fft(eng, d, sb, pos, size, trunc, sd);
}
void oracle_ifft(int eng, uint8_t *d, size_t sb, size_t pos, size_t size, size_t trunc, size_t sd) {
    oracle_init(); eng_ifft(eng, d, sb, pos, size, trunc, sd);
}
void oracle_fwht(int eng, uint16_t *data, size_t trunc) { oracle_init(); eng_fwht(eng, data, trunc); }
void oracle_eval_poly(int eng, uint16_t *e, size_t trunc) { oracle_init(); eng_eval_poly(eng, e, trunc); }
void oracle_mul(int eng, uint8_t *x, size_t n, uint16_t log_m) { oracle_init(); eng_mul(eng, x, n, log_m); }
void oracle_xor(int eng, uint8_t *x, const uint8_t *y, size_t n) { eng_xor(eng, x, y, n); }
void oracle_formal_derivative(int eng, uint8_t *d, size_t sb, size_t len) { eng_formal_derivative(eng, d, sb, len); }
const uint16_t *oracle_table(int which) {
    oracle_init();
    switch (which) {
    case 0: return g_exp;
    case 1: return g_log;
    case 2: return g_skew;
    case 3: return g_log_walsh;
    default: return NULL;
    }
}

/* ------------------------------------------------------------------ */
/* CPU baseline loop -- benches/benchmarks.rs:60-109 (benchmarks_main) */
/* ------------------------------------------------------------------ */
/* One benchmark row of the reference's `main` group, timed the way its
 * b.iter closures run, with the restated engine `engine` behind the
 * DefaultRate encoder/decoder (ReedSolomonEncoder / ReedSolomonDecoder):
 *   loss_percent < 0: add_original_shard x k + encode          (:71-76)
 *   else: L = min(k, m) * loss_percent / 100; add_original_shard(i) for
 *         i < k - L, add_recovery_shard(i) for i < L, decode     (:84-107)
 * `original` holds k shards, `recovery` m shards (S bytes each, contiguous).
 * Iterations run until min_seconds have passed (at least one); returns the
 * iteration count and the elapsed seconds.  Used only by bench.py's
 * cpu_baseline leg. */
#include <time.h>
static double oracle_now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
int oracle_bench_main(int engine, size_t k, size_t m, size_t S, const uint8_t *original, const uint8_t *recovery,
                      int loss_percent, double min_seconds, size_t *iters, double *seconds) {
    oracle_error err;
    size_t n = 0;
    double t0 = oracle_now(), t = 0.0;
    if (loss_percent < 0) {
        oracle_encoder *e = oracle_encoder_new(0, engine, k, m, S, &err);
        if (!e) return err.code ? err.code : -1;
        do {
            for (size_t i = 0; i < k; i++)
                if (oracle_encoder_add_original_shard(e, original + i * S, S, &err)) return err.code;
            if (oracle_encoder_encode(e, &err)) return err.code;
            oracle_encoder_reset_received(e); /* EncoderResult dropped */
            n++;
            t = oracle_now() - t0;
        } while (t < min_seconds);
        oracle_encoder_free(e);
    } else {
        const size_t loss = (k < m ? k : m) * (size_t)loss_percent / 100;
        oracle_decoder *d = oracle_decoder_new(0, engine, k, m, S, &err);
        if (!d) return err.code ? err.code : -1;
        do {
            for (size_t i = 0; i < k - loss; i++)
                if (oracle_decoder_add_original_shard(d, i, original + i * S, S, &err)) return err.code;
            for (size_t i = 0; i < loss; i++)
                if (oracle_decoder_add_recovery_shard(d, i, recovery + i * S, S, &err)) return err.code;
            if (oracle_decoder_decode(d, &err)) return err.code;
            oracle_decoder_reset_received(d); /* DecoderResult dropped */
            n++;
            t = oracle_now() - t0;
        } while (t < min_seconds);
        oracle_decoder_free(d);
    }
    *iters = n;
    *seconds = t;
    return 0;
}
