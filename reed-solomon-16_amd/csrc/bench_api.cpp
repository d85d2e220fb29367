// bench_api.cpp -- the reference's own benchmark loop (benches/benchmarks.rs:
// 33-113, group "main") run against the MI355X engine through the C ABI only
// (include/rs16.h), the way a compiled FFI caller drives it: per iteration
//   ReedSolomonEncoder: add_original_shard x k, encode            (:71-76)
//   ReedSolomonDecoder: add_original_shard x (k - L), add_recovery_shard x L,
//                       decode, L = min(k, m) * loss% / 100         (:98-106)
// with shards in ordinary (pageable) host memory, one heap allocation per
// shard like the reference's Vec<Vec<u8>>.  The result of each iteration is
// dropped unread, as in the reference bench; a second encoder row also reads
// every recovery shard back through EncoderResult::recovery, and the timer
// stops only after the engine's stream has drained.
//
// usage: rs16_bench_api K M S ORIGINAL.bin RECOVERY_OUT.bin MIN_SECONDS
//   ORIGINAL.bin: K x S bytes.  RECOVERY_OUT.bin receives the recovery shards
//   of the first round (the caller checks them against the oracle).
// Prints one JSON object.  Exit status != 0 on any error or mismatch.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/rs16.h"

using Clock = std::chrono::steady_clock;
typedef std::vector<std::vector<uint8_t>> Shards;

static void die(const char* what, const rs16_error& e) {
    char msg[256];
    rs16_error_message(&e, msg, sizeof msg);
    fprintf(stderr, "rs16_bench_api: %s: %s\n", what, msg);
    exit(1);
}
#define CK(call, what)                       \
    do {                                     \
        if ((call) != 0) die(what, err);     \
    } while (0)

static double now() { return std::chrono::duration<double>(Clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    if (argc != 7) {
        fprintf(stderr, "usage: %s K M S ORIGINAL.bin RECOVERY_OUT.bin MIN_SECONDS\n", argv[0]);
        return 2;
    }
    const size_t k = strtoull(argv[1], 0, 10), m = strtoull(argv[2], 0, 10), S = strtoull(argv[3], 0, 10);
    const double min_s = atof(argv[6]);
    Shards original(k, std::vector<uint8_t>(S));
    {
        FILE* f = fopen(argv[4], "rb");
        if (!f) return perror(argv[4]), 1;
        for (auto& s : original)
            if (fread(s.data(), 1, S, f) != S) return fprintf(stderr, "short read\n"), 1;
        fclose(f);
    }
    rs16_error err;
    rs16_engine* eng = rs16_engine_new(0, &err);
    if (!eng) die("engine", err);
    rs16_encoder* enc = rs16_encoder_new(eng, RS16_RATE_DEFAULT, k, m, S, &err);
    if (!enc) die("encoder", err);
    rs16_decoder* dec = rs16_decoder_new(eng, RS16_RATE_DEFAULT, k, m, S, &err);
    if (!dec) die("decoder", err);

    // First round: the recovery shards (reed_solomon_16::encode, src/lib.rs:242-279).
    Shards recovery(m, std::vector<uint8_t>(S));
    for (auto& s : original) CK(rs16_encoder_add_original_shard(enc, s.data(), S, &err), "add_original_shard");
    CK(rs16_encoder_encode(enc, &err), "encode");
    for (size_t i = 0; i < m; i++) {
        const void* p = rs16_encoder_recovery(enc, i, &err);
        if (!p) die("recovery", err);
        memcpy(recovery[i].data(), p, S);
    }
    if (rs16_encoder_recovery(enc, m, &err) != nullptr) return fprintf(stderr, "recovery(m) not None\n"), 1;
    rs16_encoder_result_drop(enc);
    {
        FILE* f = fopen(argv[5], "wb");
        if (!f) return perror(argv[5]), 1;
        for (auto& s : recovery) fwrite(s.data(), 1, S, f);
        fclose(f);
    }

    auto encode_round = [&](bool read_back) {
        for (auto& s : original) CK(rs16_encoder_add_original_shard(enc, s.data(), S, &err), "add_original_shard");
        CK(rs16_encoder_encode(enc, &err), "encode");
        if (read_back) {
            volatile uint8_t sink = 0;
            for (size_t i = 0; i < m; i++) {
                const uint8_t* p = (const uint8_t*)rs16_encoder_recovery(enc, i, &err);
                if (!p) die("recovery", err);
                sink ^= p[0];
            }
            (void)sink;
        }
        rs16_encoder_result_drop(enc);  // EncoderResult dropped (src/encoder_result.rs:48-52)
    };
    const size_t max_loss = k < m ? k : m;
    auto decode_round = [&](size_t loss) {
        for (size_t i = 0; i < k - loss; i++)
            CK(rs16_decoder_add_original_shard(dec, i, original[i].data(), S, &err), "add_original_shard");
        for (size_t i = 0; i < loss; i++)
            CK(rs16_decoder_add_recovery_shard(dec, i, recovery[i].data(), S, &err), "add_recovery_shard");
        CK(rs16_decoder_decode(dec, &err), "decode");
        rs16_decoder_result_drop(dec);
    };
    // Timed like criterion's b.iter: warm-up, then iterations until
    // min_seconds; the stream is drained inside the timed span.
    auto timed = [&](auto&& round) {
        round();
        round();
        CK(rs16_engine_synchronize(eng, nullptr, &err), "synchronize");
        size_t n = 0;
        const double t0 = now();
        double t = 0;
        do {
            round();
            n++;
            if (n % 4 == 0 || now() - t0 >= min_s) {
                CK(rs16_engine_synchronize(eng, nullptr, &err), "synchronize");
                t = now() - t0;
            }
        } while (t < min_s || n < 3);
        return t / (double)n;
    };
    const double gib = (double)(k + m) * (double)S / (double)(1ull << 30);
    printf("{\"k\": %zu, \"m\": %zu, \"shard_bytes\": %zu", k, m, S);
    const double te = timed([&] { encode_round(false); });
    printf(", \"encoder_us\": %.2f, \"encoder_gib_s\": %.3f", te * 1e6, gib / te);
    const double tr = timed([&] { encode_round(true); });
    printf(", \"encoder_read_back_us\": %.2f, \"encoder_read_back_gib_s\": %.3f", tr * 1e6, gib / tr);
    for (int pct : {1, 100}) {
        const size_t loss = max_loss * (size_t)pct / 100;
        // correctness of this loss pattern: every lost original restored
        for (size_t i = 0; i < k - loss; i++)
            CK(rs16_decoder_add_original_shard(dec, i, original[i].data(), S, &err), "add_original_shard");
        for (size_t i = 0; i < loss; i++)
            CK(rs16_decoder_add_recovery_shard(dec, i, recovery[i].data(), S, &err), "add_recovery_shard");
        CK(rs16_decoder_decode(dec, &err), "decode");
        for (size_t i = 0; i < k; i++) {
            const void* p = rs16_decoder_restored_original(dec, i, &err);
            if ((p != nullptr) != (i >= k - loss)) return fprintf(stderr, "restored set differs at %zu\n", i), 1;
            if (p && memcmp(p, original[i].data(), S) != 0)
                return fprintf(stderr, "restored original %zu differs (loss %d%%)\n", i, pct), 1;
        }
        rs16_decoder_result_drop(dec);
        const double td = timed([&] { decode_round(loss); });
        printf(", \"decoder_%dpct_us\": %.2f, \"decoder_%dpct_gib_s\": %.3f", pct, td * 1e6, pct, gib / td);
    }
    printf(", \"verified\": true}\n");
    rs16_decoder_free(dec);
    rs16_encoder_free(enc);
    rs16_engine_free(eng);
    return 0;
}
