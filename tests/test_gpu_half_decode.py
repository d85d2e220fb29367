"""GPU parity of the half-transform decode (every original lost; see
rs16_engine.cpp half_decode and tests/test_half_decode.py for the identity):
the restored originals must equal the originals bit for bit, and the decoder
must agree with the oracle's decode, for high and low rate, one-pass
(n/2 <= 256 rows) and three-pass sizes, padding rows (m < chunk) and
recovery subsets with missing rows (m > k)."""
import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu

CASES = [
    # (k, m, rate, recovery rows given: "all" | "first-k" | "random-k")
    (1, 1, "high", "all"), (1, 2, "high", "first-k"), (2, 2, "high", "all"), (3, 4, "high", "random-k"),
    (5, 7, "high", "random-k"), (100, 100, "high", "all"), (128, 128, "high", "all"), (200, 256, "high", "random-k"),
    (256, 300, "high", "random-k"), (300, 300, "high", "all"), (1000, 1000, "high", "all"),
    (1000, 1024, "high", "random-k"), (3000, 4000, "high", "random-k"), (8192, 8192, "high", "all"),
    (1, 1, "low", "all"), (3, 3, "low", "all"), (100, 100, "low", "all"), (100, 128, "low", "random-k"),
    (1000, 1000, "low", "all"), (3000, 4096, "low", "random-k"), (8000, 8192, "low", "all"),
    (16000, 16384, "default", "random-k"),
]


def received(m, k, how, seed):
    if how == "all":
        return np.arange(m)
    if how == "first-k":
        return np.arange(k)
    return np.sort(np.random.default_rng(seed).choice(m, k, replace=False))


@pytest.mark.parametrize("k,m,rate,how", CASES, ids=lambda v: str(v))
def test_half_decode_rate_decoder(k, m, rate, how):
    sb = 128
    original = generate_original(k, sb, k + m)
    recovery = O.encode(k, m, original, rate=rate)
    dec = rs16.RateDecoder(k, m, sb, rate)
    for i in received(m, k, how, k):
        dec.add_recovery_shard(int(i), recovery[i])
    with dec.decode() as res:
        got = dict(res.restored_original_iter())
    assert sorted(got) == list(range(k))
    for i in range(k):
        assert got[i] == original[i].tobytes(), i


@pytest.mark.parametrize("k,m", [(1000, 1000), (32768, 32768), (20000, 32768)])
def test_half_decode_device(k, m):
    eng = rs16.default_engine()
    sb = 1024 if k <= 1000 else 256
    original = generate_original(k, sb, 3)
    d_orig = DeviceArray.from_numpy(eng, original)
    d_rec = DeviceArray(eng, m * sb)
    rs16.encode_device(k, m, sb, d_orig.ptr, d_rec.ptr, engine=eng)
    d_orig.upload(np.full_like(original, 0x5A))
    rm = np.zeros(m, np.uint8)
    rm[received(m, k, "random-k", 7)] = 1
    d_of = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    d_rf = DeviceArray.from_numpy(eng, rm)
    rs16.decode_device(k, m, sb, d_orig.ptr, d_of.ptr, d_rec.ptr, d_rf.ptr, 0, k, engine=eng)
    assert np.array_equal(d_orig.download(shape=(k, sb)), original)
