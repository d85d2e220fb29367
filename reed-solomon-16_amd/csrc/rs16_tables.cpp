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
}
}  // namespace

const HostTables& host_tables() {
    std::call_once(g_once, [] { build(g_tables); });
    return g_tables;
}

}  // namespace rs16
