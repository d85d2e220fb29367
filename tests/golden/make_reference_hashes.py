"""Generate tests/golden/reference_hashes.json from the reference's own golden
vectors (run once in the build container; /root/reference is not needed at
test time).

Source of the data:
  * hash tables DEFAULT_TINY / HIGH_TINY / LOW_TINY and the named constants:
    /root/reference/src/test_util.rs:583-837
  * roundtrip parameters (decoder_original / decoder_recovery index sets) from
    the call sites:
      roundtrips_tiny             src/rate/rate_high.rs:339-352, rate_low.rs:339-352,
                                  rate_default.rs:372-385
      roundtrip_*_originals_missing / no_originals_missing
                                  src/rate/rate_high.rs:319-336, rate_low.rs:319-336
      large (#[ignore]) cases     src/rate/rate_high.rs:354-397, rate_low.rs:354-397
      two-round cases             src/rate/rate_high.rs:402-420, rate_low.rs:402-420,
                                  rate_default.rs:390-439, src/reed_solomon.rs:244-271
Only data (k, m, seed, shard_bytes, index ranges, SHA-256 hex) is written.
"""
import json
import re
import sys
from pathlib import Path

REF = Path("/root/reference/src/test_util.rs")
OUT = Path(__file__).with_name("reference_hashes.json")


def main():
    text = REF.read_text()
    consts = dict(re.findall(r'pub\(crate\) const ([A-Z0-9_]+): &str =\s*"([0-9a-f]{64})"', text))

    def table(name):
        body = re.search(name + r": &\[\(usize, usize, u8, &str\)\] = &\[(.*?)\];", text, re.S).group(1)
        rows = []
        for m in re.finditer(r'\((\d+),\s*(\d+),\s*(\d+),\s*(?:"([0-9a-f]{64})"|([A-Z0-9_]+))\)', body):
            k, mm, seed = int(m.group(1)), int(m.group(2)), int(m.group(3))
            h = m.group(4) or consts[m.group(5)]
            rows.append({"k": k, "m": mm, "seed": seed, "hash": h})
        return rows

    tiny = {"default": table("DEFAULT_TINY"), "high": table("HIGH_TINY"), "low": table("LOW_TINY")}
    for rate, rows in tiny.items():
        for r in rows:
            # roundtrips_tiny: decoder gets originals [m..k) and recovery [0..min(k,m))
            r.update(shard_bytes=1024, rate=rate,
                     dec_original=[[r["m"], max(r["k"], r["m"])]] if r["k"] > r["m"] else [],
                     dec_recovery=[[0, min(r["k"], r["m"])]])

    R = lambda a, b: [[a, b]]
    single = [
        # rate_high.rs:319-336 / rate_low.rs:319-336
        dict(rate="high", k=3, m=3, shard_bytes=1024, seed=133, hash=consts["EITHER_3_3"], dec_original=[], dec_recovery=R(0, 3)),
        dict(rate="high", k=3, m=2, shard_bytes=1024, seed=132, hash=consts["HIGH_3_2"], dec_original=R(0, 3), dec_recovery=[]),
        dict(rate="low", k=3, m=3, shard_bytes=1024, seed=133, hash=consts["EITHER_3_3"], dec_original=[], dec_recovery=R(0, 3)),
        dict(rate="low", k=2, m=3, shard_bytes=1024, seed=123, hash=consts["LOW_2_3"], dec_original=[[0, 1], [1, 2]], dec_recovery=[]),
        # lib.rs:356-369 roundtrip (one-shot encode/decode, default rate)
        dict(rate="default", k=2, m=3, shard_bytes=1024, seed=123, hash=consts["LOW_2_3"], dec_original=[], dec_recovery=R(0, 2)),
    ]
    large = [
        # rate_high.rs:354-397 (#[ignore])
        dict(rate="high", k=3000, m=30000, shard_bytes=64, seed=14, hash=consts["HIGH_3000_30000_14"], dec_original=[], dec_recovery=R(0, 3000)),
        dict(rate="high", k=32768, m=32768, shard_bytes=64, seed=11, hash=consts["EITHER_32768_32768_11"], dec_original=[], dec_recovery=R(0, 32768)),
        dict(rate="high", k=60000, m=3000, shard_bytes=64, seed=12, hash=consts["HIGH_60000_3000_12"], dec_original=R(3000, 60000), dec_recovery=R(0, 3000)),
        # rate_low.rs:354-397 (#[ignore])
        dict(rate="low", k=3000, m=60000, shard_bytes=64, seed=13, hash=consts["LOW_3000_60000_13"], dec_original=[], dec_recovery=R(0, 3000)),
        dict(rate="low", k=30000, m=3000, shard_bytes=64, seed=15, hash=consts["LOW_30000_3000_15"], dec_original=R(3000, 30000), dec_recovery=R(0, 3000)),
        dict(rate="low", k=32768, m=32768, shard_bytes=64, seed=11, hash=consts["EITHER_32768_32768_11"], dec_original=[], dec_recovery=R(0, 32768)),
    ]

    def rr(k, m, h, o, r, seed, sb=1024):
        return dict(k=k, m=m, shard_bytes=sb, hash=consts[h], dec_original=o, dec_recovery=r, seed=seed)

    L = lambda *xs: [[x, x + 1] for x in xs]
    two_rounds = [
        # rate_high.rs:402-420
        dict(rate="high", explicit_reset=False, a=rr(3, 2, "HIGH_3_2", L(1), L(0, 1), 132), b=rr(3, 2, "HIGH_3_2_232", L(0), L(0, 1), 232)),
        dict(rate="high", explicit_reset=True, a=rr(3, 2, "HIGH_3_2", L(1), L(0, 1), 132), b=rr(5, 2, "HIGH_5_2", L(0, 2, 4), L(0, 1), 152)),
        # rate_low.rs:402-420
        dict(rate="low", explicit_reset=False, a=rr(2, 3, "LOW_2_3", [], L(0, 2), 123), b=rr(2, 3, "LOW_2_3_223", [], L(1, 2), 223)),
        dict(rate="low", explicit_reset=True, a=rr(2, 3, "LOW_2_3", [], L(0, 2), 123), b=rr(2, 5, "LOW_2_5", [], L(0, 4), 125)),
        # rate_default.rs:390-439
        dict(rate="default", explicit_reset=False, a=rr(2, 3, "LOW_2_3", [], L(0, 2), 123), b=rr(2, 3, "LOW_2_3_223", L(0), L(1), 223)),
        dict(rate="default", explicit_reset=True, a=rr(3, 2, "HIGH_3_2", L(1), L(0, 1), 132), b=rr(5, 3, "HIGH_5_3", L(1, 3), L(0, 1, 2), 153)),
        dict(rate="default", explicit_reset=True, a=rr(3, 2, "HIGH_3_2", L(1), L(0, 1), 132), b=rr(2, 3, "LOW_2_3", [], L(0, 2), 123)),
        dict(rate="default", explicit_reset=True, a=rr(2, 3, "LOW_2_3", [], L(0, 1), 123), b=rr(3, 2, "HIGH_3_2", L(1), L(0, 1), 132)),
        dict(rate="default", explicit_reset=True, a=rr(2, 3, "LOW_2_3", [], L(0, 2), 123), b=rr(3, 5, "LOW_3_5", [], L(0, 2, 4), 135)),
        # reed_solomon.rs:244-271 (ReedSolomonEncoder/Decoder, default rate)
        dict(rate="default", explicit_reset=True, a=rr(2, 3, "LOW_2_3", [], L(0, 1), 123), b=rr(3, 2, "HIGH_3_2", L(1), L(0, 1), 132)),
    ]
    OUT.write_text(json.dumps({"source": "malaire/reed-solomon-16 v0.1.0 src/test_util.rs:583-837",
                               "tiny": tiny, "single": single, "large": large,
                               "two_rounds": two_rounds}, indent=1))
    print("wrote", OUT, sum(len(v) for v in tiny.values()), "tiny rows")


if __name__ == "__main__":
    sys.exit(main())
