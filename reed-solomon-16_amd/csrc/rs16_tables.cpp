// rs16_tables.cpp -- GF(2^16) constant tables, built once per process on the
// host and uploaded to HBM by each engine (rs16_engine.cpp).
//
// Field definition (must match the reference bit for bit):
//   GF_POLYNOMIAL 0x1002D, elements in the Cantor basis
//   (src/engine.rs:59-74; construction src/engine/tables.rs:83-124),
//   FFT twiddle logs "skew" (src/engine/tables.rs:164-205),
//   LogWalsh = FWHT(log) with log[0] = 0 (src/engine/tables.rs:127-139).
// The device-side multiply tables are a GPU-specific format (v_perm byte
// tables, rs16_gf.hpp), not the reference's Mul16 nibble tables.
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "rs16_internal.hpp"

namespace rs16 {

namespace {
const uint16_t kCantorBasis[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                   0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
HostTables g_tables;
std::once_flag g_once;

inline uint16_t gf_mul(const HostTables& t, uint16_t x, uint32_t log_m) {
    return x == 0 ? 0 : t.exp[add_mod(t.log[x], log_m)];
}

void fwht_full(std::vector<uint16_t>& v) {
    for (uint32_t d = 1; d < GF_ORDER; d <<= 1)
        for (uint32_t r = 0; r < GF_ORDER; r += 2 * d)
            for (uint32_t i = r; i < r + d; i++) {
                uint32_t a = v[i], b = v[i + d];
                v[i] = (uint16_t)add_mod(a, b);
                v[i + d] = (uint16_t)sub_mod(a, b);
            }
}

void build(HostTables& t) {
    t.exp.assign(GF_ORDER, 0);
    t.log.assign(GF_ORDER, 0);
    // Exponent table of the LFSR over 0x1002D: position -> exponent.
    {
        uint32_t state = 1;
        for (uint32_t i = 0; i < GF_MODULUS; i++) {
            t.exp[state] = (uint16_t)i;
            state <<= 1;
            if (state >= GF_ORDER) state ^= 0x1002Du;
        }
        t.exp[0] = (uint16_t)GF_MODULUS;
    }
    // Cantor-basis element i (as XOR of basis vectors by the bits of i),
    // then log[i] = exponent of that element and exp = its inverse map.
    {
        std::vector<uint16_t> cb(GF_ORDER, 0);
        for (int b = 0; b < 16; b++) {
            uint32_t w = 1u << b;
            for (uint32_t j = 0; j < w; j++) cb[j + w] = cb[j] ^ kCantorBasis[b];
        }
        for (uint32_t i = 0; i < GF_ORDER; i++) t.log[i] = t.exp[cb[i]];
        for (uint32_t i = 0; i < GF_ORDER; i++) t.exp[t.log[i]] = (uint16_t)i;
        t.exp[GF_MODULUS] = t.exp[0];
    }
    // FFT twiddle logs.
    {
        std::vector<uint16_t> sk(GF_MODULUS, 0);
        uint16_t temp[15];
        for (int i = 1; i < 16; i++) temp[i - 1] = (uint16_t)(1u << i);
        for (int m = 0; m < 15; m++) {
            const uint32_t step = 1u << (m + 1);
            sk[(1u << m) - 1] = 0;
            for (int i = m; i < 15; i++) {
                const uint32_t s = 1u << (i + 1);
                for (uint32_t j = (1u << m) - 1; j < s; j += step) sk[j + s] = sk[j] ^ temp[i];
            }
            temp[m] = (uint16_t)(GF_MODULUS - t.log[gf_mul(t, temp[m], t.log[temp[m] ^ 1])]);
            for (int i = m + 1; i < 15; i++) temp[i] = gf_mul(t, temp[i], add_mod(t.log[temp[i] ^ 1], temp[m]));
        }
        t.skew.resize(GF_MODULUS);
        for (uint32_t i = 0; i < GF_MODULUS; i++) t.skew[i] = t.log[sk[i]];
    }
    // LogWalsh.
    t.log_walsh = t.log;
    t.log_walsh[0] = 0;
    fwht_full(t.log_walsh);

    // The pass kernels skip the multiply of uniform groups whose twiddle is
    // the sentinel and recognise those by index: the sentinel entries are
    // exactly the indices 2^i - 1 (rs16_pass.hip, GroupLoop).  A table that
    // broke this would give wrong results, so it is checked here, once.
    for (uint32_t i = 0; i < GF_MODULUS; i++)
        if ((t.skew[i] == GF_MODULUS) != ((i & (i + 1)) == 0)) {
            fprintf(stderr, "rs16: skew table sentinel at unexpected index %u\n", i);
            abort();
        }
    // FFT/IFFT twiddle table *entries*: sentinel GF_MODULUS -> ZERO_ENTRY.
    t.skew_entry.assign(GF_ORDER, ZERO_ENTRY);
    for (uint32_t i = 0; i < GF_MODULUS; i++) t.skew_entry[i] = t.skew[i] == GF_MODULUS ? ZERO_ENTRY : t.skew[i];

    // v_perm multiply tables (layout in rs16_gf.hpp).
    t.mul_tab.assign((size_t)TAB_ENTRIES * TAB_DWORDS, 0);
    static const int kOff3[4] = {0, 3, 8, 11};
    static const int kOff2[2] = {6, 14};
    for (uint32_t lm = 0; lm < GF_ORDER; lm++) {
        uint32_t* e = &t.mul_tab[(size_t)lm * TAB_DWORDS];
        for (int g = 0; g < 4; g++)
            for (uint32_t v = 0; v < 8; v++) {
                uint16_t p = gf_mul(t, (uint16_t)(v << kOff3[g]), lm);
                for (int ob = 0; ob < 2; ob++) {
                    uint32_t byte = (p >> (8 * ob)) & 0xFF;
                    e[(g * 2 + ob) * 2 + (v >> 2)] |= byte << (8 * (v & 3));
                }
            }
        for (int gg = 0; gg < 2; gg++)
            for (uint32_t v = 0; v < 4; v++) {
                uint16_t p = gf_mul(t, (uint16_t)(v << kOff2[gg]), lm);
                for (int ob = 0; ob < 2; ob++) e[16 + gg * 2 + ob] |= ((p >> (8 * ob)) & 0xFFu) << (8 * v);
            }
    }
    // entry ZERO_ENTRY stays all zero.

    // The table of every twiddle index, so that a pass stages a twiddle's
    // table with one load instead of skew_entry -> mul_tab.
    t.skew_tab.resize((size_t)GF_ORDER * TAB_DWORDS);
    for (uint32_t i = 0; i < GF_ORDER; i++)
        std::copy_n(&t.mul_tab[(size_t)t.skew_entry[i] * TAB_DWORDS], TAB_DWORDS, &t.skew_tab[(size_t)i * TAB_DWORDS]);

    // Column codec images: table g of layer kb (g = 2^L - 2^(L-kb) + j, group
    // j covering rows [j 2^(kb+1), (j+1) 2^(kb+1))) is the twiddle of skew
    // index j 2^(kb+1) + 2^kb + delta - 1 (engine_naive.rs:43-124).
    t.col_img.assign(COL_IMG_DWORDS, 0);
    for (uint32_t L = COL_LMIN; L <= COL_LGEN; L++)
        for (uint32_t d = 0; d < col_img_count(L); d++) {
            const uint32_t N = 1u << L, delta = d * N;
            uint32_t* img = &t.col_img[col_img_offset(L, d)];
            for (uint32_t g = 0; g + 1 < N; g++) {
                uint32_t kb = 0;
                while (g >= N - (N >> (kb + 1))) kb++;
                const uint32_t j = g - (N - (N >> kb));
                const uint32_t idx = (j << (kb + 1)) + (1u << kb) + delta - 1;
                std::copy_n(&t.skew_tab[(size_t)idx * TAB_DWORDS], 20, img + (size_t)g * 20);
            }
        }

    // eval_poly (src/engine.rs:207-218) = H(log_walsh . H(e)) over 65536
    // points; for e supported on [0, n) and outputs on [0, n) it is the XOR
    // convolution out[i] = sum_j e[j] W[i ^ j], W = H(log_walsh), i.e.
    // H_n(H_n(e) . V) with V = n^-1 H_n(W[0, n)) (n^-1 = 2^(16 - log2 n)
    // mod 65535).  Exact integers, reduced mod 65535.
    {
        std::vector<int64_t> w(GF_ORDER);
        for (uint32_t i = 0; i < GF_ORDER; i++) w[i] = t.log_walsh[i];
        auto fwht = [](int64_t* x, uint32_t n) {
            for (uint32_t d = 1; d < n; d <<= 1)
                for (uint32_t i = 0; i < n; i += 2 * d)
                    for (uint32_t j = i; j < i + d; j++) {
                        const int64_t a = x[j], b = x[j + d];
                        x[j] = a + b;
                        x[j + d] = a - b;
                    }
        };
        auto mod = [](int64_t v) { return (uint32_t)(((v % 65535) + 65535) % 65535); };
        fwht(w.data(), GF_ORDER);
        t.col_k.assign(COL_LGEN + 2, 0);
        {
            int64_t pre = 0;
            for (uint32_t n = 1, j = 0; n <= (2u << COL_LMAX); n <<= 1) {
                for (; j < n; j++) pre += mod(w[j]);
                uint32_t lg = 0;
                while ((1u << lg) < n) lg++;
                if (lg < t.col_k.size()) t.col_k[lg] = mod((int64_t)t.log_walsh[0] - pre);
            }
        }
        t.col_v.assign(COL_V_DWORDS, 0);
        for (uint32_t n = 1u << COL_LMIN; n <= (2u << COL_LMAX); n <<= 1) {
            std::vector<int64_t> v(n);
            for (uint32_t i = 0; i < n; i++) v[i] = mod(w[i]);
            fwht(v.data(), n);
            uint32_t lg = 0;
            while ((1u << lg) < n) lg++;
            const int64_t inv = (int64_t)1 << (16 - lg);  // n^-1 = 2^(16 - log2 n) mod 65535 (2^16 = 1)
            for (uint32_t k = 0; k < n; k++) t.col_v[col_v_offset(n) + k] = mod(mod(v[k]) * inv);
        }
    }
}
}  // namespace

// The general decode's middle pass as a matrix (rs16_engine::mid_matrix):
// DEC_MID maps the 2^hi rows t << lo | j of every tile column j (lo = L / 2,
// hi = L - lo, skew 0) by u = FFT_hi (I + H) IFFT_hi z -- the IFFT / FFT
// layers lo .. L-1 (src/engine/engine_nosimd.rs fft / ifft: twiddle
// skew[r + dist - 1] of the block at global row r, butterflies x ^= y m, y ^= x
// and y ^= x, x ^= y m) around the high-bit half of the formal derivative
// (src/engine.rs formal_derivative: row t takes row t | 2^c for every tile
// bit c clear in t).  The twiddle indices do not involve j, so one 2^hi x
// 2^hi matrix serves every column; entry [o][t] = the log of M[o][t]
// (ZERO_ENTRY for 0), column t computed as the image of the unit vector at t.
std::vector<uint32_t> mid_matrix_entries(const HostTables& t, int L) {
    const int lo = L / 2, hi = L - lo;
    const uint32_t N = 1u << hi;
    const uint16_t one = t.exp[0];  // the element whose log is 0
    std::vector<uint32_t> ent((size_t)N * N, ZERO_ENTRY);
    std::vector<uint16_t> v(N), w(N);
    auto tw = [&](uint32_t r_tile, int kb) {  // twiddle log of the block at tile row r_tile, layer kb
        const uint32_t m = (uint32_t)(lo + kb);
        return (uint32_t)t.skew[((size_t)r_tile << lo) + (1u << m) - 1];
    };
    for (uint32_t c = 0; c < N; c++) {
        std::fill(v.begin(), v.end(), 0);
        v[c] = one;
        for (int kb = 0; kb < hi; kb++) {  // IFFT, low layers first
            const uint32_t d = 1u << kb;
            for (uint32_t r = 0; r < N; r += 2 * d) {
                const uint32_t lm = tw(r, kb);
                for (uint32_t i = r; i < r + d; i++) {
                    v[i + d] ^= v[i];
                    if (lm != GF_MODULUS) v[i] ^= gf_mul(t, v[i + d], lm);
                }
            }
        }
        for (uint32_t i = 0; i < N; i++) {  // (I + H): the formal derivative's tile bits
            uint16_t x = v[i];
            for (uint32_t b = 1; b < N; b <<= 1)
                if (!(i & b)) x ^= v[i | b];
            w[i] = x;
        }
        for (int kb = hi - 1; kb >= 0; kb--) {  // FFT, high layers first
            const uint32_t d = 1u << kb;
            for (uint32_t r = 0; r < N; r += 2 * d) {
                const uint32_t lm = tw(r, kb);
                for (uint32_t i = r; i < r + d; i++) {
                    if (lm != GF_MODULUS) w[i] ^= gf_mul(t, w[i + d], lm);
                    w[i + d] ^= w[i];
                }
            }
        }
        for (uint32_t o = 0; o < N; o++) ent[(size_t)o * N + c] = w[o] ? t.log[w[o]] : ZERO_ENTRY;
    }
    return ent;
}

const HostTables& host_tables() {
    std::call_once(g_once, [] { build(g_tables); });
    return g_tables;
}

}  // namespace rs16
