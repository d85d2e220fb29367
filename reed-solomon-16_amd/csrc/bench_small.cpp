// bench_small.cpp -- latency of small device-resident stripes (BASELINE
// configs[1] / [2], 1000:1000 x 1 KiB) through the C ABI from a compiled
// caller: rs16_encode_device / rs16_decode_device (100 % original loss) back
// to back on the engine stream, timed by the host around N calls + one sync,
// and the host's enqueue time alone (no sync).  Separates the library's
// launch path from a Python caller's (scripts/probe_small.py).
//
// usage: rs16_bench_small K M S    -> one JSON object
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/rs16.h"

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    if (argc != 4) return fprintf(stderr, "usage: %s K M S\n", argv[0]), 2;
    const size_t k = strtoull(argv[1], 0, 10), m = strtoull(argv[2], 0, 10), S = strtoull(argv[3], 0, 10);
    rs16_error err;
    rs16_engine* eng = rs16_engine_new(0, &err);
    if (!eng) return fprintf(stderr, "engine: %d\n", err.code), 1;
    std::vector<uint8_t> h(k * S);
    for (size_t i = 0; i < h.size(); i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
    std::vector<uint8_t> fo(k, 0), fr(m, 1);
    void* d_o = rs16_device_alloc(eng, k * S, &err);
    void* d_r = rs16_device_alloc(eng, m * S, &err);
    void* d_x = rs16_device_alloc(eng, k * S, &err);
    uint8_t* d_fo = (uint8_t*)rs16_device_alloc(eng, k, &err);
    uint8_t* d_fr = (uint8_t*)rs16_device_alloc(eng, m, &err);
    if (!d_o || !d_r || !d_x || !d_fo || !d_fr) return fprintf(stderr, "alloc\n"), 1;
    rs16_memcpy_htod(eng, d_o, h.data(), k * S, nullptr, &err);
    rs16_memcpy_htod(eng, d_fo, fo.data(), k, nullptr, &err);
    rs16_memcpy_htod(eng, d_fr, fr.data(), m, nullptr, &err);
    auto enc = [&]() { return rs16_encode_device(eng, k, m, S, d_o, d_r, nullptr, &err); };
    auto dec = [&]() { return rs16_decode_device(eng, k, m, S, d_x, d_fo, d_r, d_fr, 0, m, nullptr, &err); };
    if (enc() || dec() || rs16_engine_synchronize(eng, nullptr, &err)) return fprintf(stderr, "codec: %d\n", err.code), 1;
    std::vector<uint8_t> back(k * S);
    rs16_memcpy_dtoh(eng, back.data(), d_x, k * S, nullptr, &err);
    if (back != h) return fprintf(stderr, "decode did not restore\n"), 1;
    printf("{");
    const char* names[2] = {"encode", "decode"};
    for (int which = 0; which < 2; which++) {
        auto fn = [&]() { return which ? dec() : enc(); };
        for (int i = 0; i < 200; i++) fn();
        rs16_engine_synchronize(eng, nullptr, &err);
        const int n = 5000;
        const double t0 = now();
        for (int i = 0; i < n; i++)
            if (fn()) return fprintf(stderr, "codec: %d\n", err.code), 1;
        const double t1 = now();
        rs16_engine_synchronize(eng, nullptr, &err);
        const double t2 = now();
        printf("%s\"%s\": {\"enqueue_us_per_call\": %.2f, \"host_timed_us_per_call\": %.2f}", which ? ", " : "",
               names[which], (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6);
    }
    printf("}\n");
    rs16_engine_free(eng);
    return 0;
}
