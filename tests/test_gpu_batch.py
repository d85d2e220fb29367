"""rs16_encode_device_batch (include/rs16.h): many independent stripes of one
geometry per call.  Every stripe's recovery must equal the oracle's encode of
that stripe alone (src/lib.rs:242-279); the batched launches (high rate,
k <= chunk) and the stripe-by-stripe fallback (multi-chunk high rate, low
rate) are both covered, with strides wider than a stripe (the gap bytes must
stay untouched) and the 1000:1000 x 1 KiB stripe of BASELINE configs[1]."""
import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,m,sb,n,pad", [
    (100, 100, 1024, 8, 0), (1000, 1000, 1024, 6, 0), (1, 1, 64, 7, 64), (3, 5, 128, 9, 192),
    (200, 300, 192, 5, 0), (4096, 4096, 128, 3, 64), (513, 1024, 64, 4, 0), (2000, 2000, 64, 3, 128),
    (3000, 1000, 64, 3, 64), (100, 3000, 64, 2, 0),
])
def test_batch_matches_oracle(k, m, sb, n, pad):
    eng = rs16.default_engine()
    so, sr = k * sb + pad, m * sb + pad
    stripes = [generate_original(k, sb, 31 * i + k) for i in range(n)]
    host_o = np.full(n * so, 0xEE, np.uint8)
    for i, o in enumerate(stripes):
        host_o[i * so:i * so + k * sb] = o.reshape(-1)
    d_o = DeviceArray.from_numpy(eng, host_o)
    d_r = DeviceArray.from_numpy(eng, np.full(n * sr, 0x77, np.uint8))
    rs16.encode_device_batch(k, m, sb, n, d_o.ptr, so, d_r.ptr, sr, engine=eng)
    got = d_r.download(shape=(n * sr,))
    for i, o in enumerate(stripes):
        want = O.encode(k, m, o)
        assert np.array_equal(got[i * sr:i * sr + m * sb].reshape(m, sb), want), i
        assert (got[i * sr + m * sb:(i + 1) * sr] == 0x77).all(), i  # gap bytes untouched


def test_batch_errors_and_empty():
    eng = rs16.default_engine()
    d = DeviceArray(eng, 64 * 8)
    rs16.encode_device_batch(2, 2, 64, 0, d.ptr, 128, d.ptr, 128, engine=eng)  # nothing to do
    with pytest.raises(rs16.Error) as e:
        rs16.encode_device_batch(2, 2, 64, 2, d.ptr, 64, d.ptr, 128, engine=eng)  # stride < k * S
    assert e.value.kind == "InvalidArgument"
    with pytest.raises(rs16.Error) as e:
        rs16.encode_device_batch(2, 2, 64, 2, d.ptr, 160, d.ptr, 128, engine=eng)  # stride not in 64 B blocks
    assert e.value.kind == "InvalidArgument"
    with pytest.raises(rs16.Error) as e:
        rs16.encode_device_batch(2, 2, 100, 2, d.ptr, 256, d.ptr, 256, engine=eng)
    assert e.value.kind == "InvalidShardSize"
    f = DeviceArray(eng, 64)
    with pytest.raises(rs16.Error) as e:  # (decode: the reference's NotEnoughShards first)
        rs16.decode_device_batch(2, 2, 64, 2, d.ptr, 128, f.ptr, d.ptr, 128, f.ptr, 0, 1, engine=eng)
    assert e.value.kind == "NotEnoughShards"
    with pytest.raises(rs16.Error) as e:
        rs16.decode_device_batch(2, 2, 64, 2, d.ptr, 96, f.ptr, d.ptr, 128, f.ptr, 0, 2, engine=eng)
    assert e.value.kind == "InvalidArgument"


@pytest.mark.parametrize("k,m,sb,n,pattern", [
    (1000, 1000, 1024, 6, "all"), (1000, 1000, 1024, 5, "tail"), (100, 100, 1024, 9, "all"),
    (100, 300, 192, 4, "scatter"), (4096, 4096, 128, 3, "tail"), (4096, 4096, 128, 3, "all"),
    (2000, 3000, 64, 4, "scatter"), (3, 5, 64, 7, "all"), (3000, 1000, 64, 3, "scatter"),
    (300, 3000, 64, 3, "all"),
])
def test_decode_batch_shared_pattern(k, m, sb, n, pattern):
    # every stripe lost the same originals (a failed device); the restored
    # originals of every stripe must be the originals, and the recovery rows
    # and the received originals must stay untouched
    eng = rs16.default_engine()
    pad = 64
    so, sr = k * sb + pad, m * sb + pad
    stripes = [generate_original(k, sb, 17 * i + k) for i in range(n)]
    recs = [O.encode(k, m, o) for o in stripes]
    lost = min(k, m)
    om = np.ones(k, bool)
    if pattern == "all":
        om[:lost] = False
    elif pattern == "tail":
        om[k - max(1, lost // 100):] = False
    else:
        om[np.random.default_rng(k + m).choice(k, lost // 2 + 1, replace=False)] = False
    nlost = int((~om).sum())
    rm = np.zeros(m, bool)
    rm[np.random.default_rng(m).choice(m, nlost, replace=False)] = True
    host_o = np.full(n * so, 0x3C, np.uint8)
    host_r = np.full(n * sr, 0x3C, np.uint8)
    for i in range(n):
        held = stripes[i].copy()
        held[~om] = 0xA5  # garbage in the lost slots
        host_o[i * so:i * so + k * sb] = held.reshape(-1)
        host_r[i * sr:i * sr + m * sb] = recs[i].reshape(-1)
    d_o, d_r = DeviceArray.from_numpy(eng, host_o), DeviceArray.from_numpy(eng, host_r)
    d_of = DeviceArray.from_numpy(eng, om.astype(np.uint8))
    d_rf = DeviceArray.from_numpy(eng, rm.astype(np.uint8))
    rs16.decode_device_batch(k, m, sb, n, d_o.ptr, so, d_of.ptr, d_r.ptr, sr, d_rf.ptr, int(om.sum()), nlost,
                             engine=eng)
    got = d_o.download(shape=(n * so,))
    for i in range(n):
        assert np.array_equal(got[i * so:i * so + k * sb].reshape(k, sb), stripes[i]), i
        assert (got[i * so + k * sb:(i + 1) * so] == 0x3C).all(), i
    assert np.array_equal(d_r.download(shape=(n * sr,)), host_r)


@pytest.mark.parametrize("k,m,n", [(2, 3, 2048), (4, 4, 1000), (16, 16, 777)])
def test_batch_many_small_stripes(k, m, n):
    # thousands of tiny stripes in one call (large grids, stripe counts that
    # are not multiples of 8): encode, then decode with every original lost
    eng = rs16.default_engine()
    sb = 64
    rng = np.random.default_rng(n)
    orig = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    d_o = DeviceArray.from_numpy(eng, orig.reshape(-1))
    d_r = DeviceArray(eng, n * m * sb)
    rs16.encode_device_batch(k, m, sb, n, d_o.ptr, k * sb, d_r.ptr, m * sb, engine=eng)
    rec = d_r.download(shape=(n, m, sb))
    for i in (0, 1, n // 2, n - 1):
        assert np.array_equal(rec[i], O.encode(k, m, orig[i])), i
    d_x = DeviceArray.from_numpy(eng, np.zeros(n * k * sb, np.uint8))
    fo = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    rm = np.zeros(m, np.uint8)
    rm[:k] = 1
    fr = DeviceArray.from_numpy(eng, rm)
    rs16.decode_device_batch(k, m, sb, n, d_x.ptr, k * sb, fo.ptr, d_r.ptr, m * sb, fr.ptr, 0, k, engine=eng)
    assert np.array_equal(d_x.download(shape=(n, k, sb)), orig)
