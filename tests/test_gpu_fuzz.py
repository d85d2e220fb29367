"""Random round trips on the GPU, after examples/test-random-roundtrips.rs:72-256:
random original/recovery counts (log-uniform up to the GF_ORDER limit,
:101-116), shard sizes up to 64 B (MAX_SHARD_BYTES_LOG = 6, :18, :96-97),
loss count = recovery_count half the time, else uniform in 1..=recovery_count
(:118-123), loss positions sampled over originals + recovery (:125-128); each
case runs DefaultRate and, where supported, HighRate and LowRate (:137-174)
with one encoder and one decoder per rate reused across cases (the work-buffer
reuse of :144-145, via reset).  Recovery shards must equal the oracle's
(the reference checks Naive == NoSimd), restored originals the inputs.
"""
import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.util import generate_original

pytestmark = pytest.mark.gpu
GF_ORDER = 65536
CASES = 24


def next_pow2(x):
    return 1 << (x - 1).bit_length()


def random_case(rng):
    sb = 64  # MIN = MAX_SHARD_BYTES_LOG = 6 (:17-18)
    while True:
        k = int(2.0 ** rng.uniform(0.0, 16.0))
        m = int(2.0 ** rng.uniform(0.0, 16.0))
        if next_pow2(min(k, m)) + max(k, m) <= GF_ORDER:
            return k, m, sb


def roundtrip(enc, dec, rate, k, m, sb, original, lost):
    enc.reset(k, m, sb)
    for s in original:
        enc.add_original_shard(s)
    with enc.encode() as res:
        recovery = list(res.recovery_iter())
    want = O.encode(k, m, original, rate=rate)
    assert b"".join(recovery) == want.tobytes(), (rate, k, m)
    dec.reset(k, m, sb)
    for i in range(k):
        if not lost[i]:
            dec.add_original_shard(i, original[i])
    for i in range(m):
        if not lost[k + i]:
            dec.add_recovery_shard(i, recovery[i])
    with dec.decode() as res:
        restored = dict(res.restored_original_iter())
    assert set(restored) == {i for i in range(k) if lost[i]}, (rate, k, m)
    for i, v in restored.items():
        assert v == original[i].tobytes(), (rate, k, m, i)


def test_random_roundtrips():
    rng = np.random.default_rng(20240611)
    coders = {}
    for case in range(CASES):
        k, m, sb = random_case(rng)
        original = generate_original(k, sb, case & 0xFF)
        loss = m if rng.random() < 0.5 else int(rng.integers(1, m + 1))
        lost = np.zeros(k + m, bool)
        lost[rng.choice(k + m, size=loss, replace=False)] = True
        for rate in ("default", "high", "low"):
            if rate != "default" and not rs16.supports(k, m, rate):
                continue
            if rate not in coders:
                coders[rate] = (rs16.RateEncoder(1, 1, 64, rate), rs16.RateDecoder(1, 1, 64, rate))
            enc, dec = coders[rate]
            roundtrip(enc, dec, rate, k, m, sb, original, lost)
