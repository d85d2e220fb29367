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
        rs16.encode_device_batch(2, 2, 100, 2, d.ptr, 256, d.ptr, 256, engine=eng)
    assert e.value.kind == "InvalidShardSize"
