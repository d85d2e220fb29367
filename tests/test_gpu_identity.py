"""The identity-multiplier decode (rs16_engine::identity_logs, DESIGN.md
3.13): a decode whose erased rows are exactly one half of the work rows
(every original lost, every recovery shard received, k = m = 2^j >= 2048)
skips eval_poly and both per-row multiplies (every erasure log is 0,
tests/test_eval_identity.py), and its passes count the received rows for
rs16_decode_check.  Every entry point that reaches it must restore the
originals bit for bit (src/rate/rate_high.rs:168-247, rate_low.rs:168-247),
with RS16_DIAG_NO_IDENTITY (the evaluated path) as the control, and the
checked mode must still catch flags that disagree with the counts."""
import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = rs16.Engine(0)
    yield e
    e.close()


def stripe(eng, k, sb, seed):
    original = generate_original(k, sb, seed)
    d_o = DeviceArray.from_numpy(eng, original)
    d_r = DeviceArray(eng, k * sb)
    rs16.encode_device(k, k, sb, d_o.ptr, d_r.ptr, engine=eng)
    return original, d_o, d_r


@pytest.mark.parametrize("diag", [0, rs16.DIAG_NO_IDENTITY], ids=["identity", "evaluated"])
@pytest.mark.parametrize("k,sb,slices", [(2048, 64, 1), (4096, 192, 1), (8192, 128, 3), (32768, 1024, 1),
                                         (32768, 128, 2)])
def test_device_decode(eng, k, sb, slices, diag):
    old = eng.set_diagnostics(diag)
    eng.set_slices(slices)
    try:
        original, d_o, d_r = stripe(eng, k, sb, k + sb)
        assert np.array_equal(d_r.download(shape=(k, sb))[:4], O.encode(k, k, original)[:4])
        d_x = DeviceArray.from_numpy(eng, np.full_like(original, 0xA5))  # lost rows hold garbage
        d_fo = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
        d_fr = DeviceArray.from_numpy(eng, np.ones(k, np.uint8))
        for _ in range(2):
            rs16.decode_device(k, k, sb, d_x.ptr, d_fo.ptr, d_r.ptr, d_fr.ptr, 0, k, engine=eng, check=True)
            assert np.array_equal(d_x.download(shape=(k, sb)), original)
            d_x.upload(np.full_like(original, 0x3C))
    finally:
        eng.set_slices(1)
        eng.set_diagnostics(old)


@pytest.mark.parametrize("k", [2048, 32768])
def test_checked_mode_catches_a_missing_recovery_flag(eng, k):
    # the counts claim every recovery shard, the flags miss one: the passes'
    # own counts (no eval_poly ran) expose it
    sb = 64
    original, d_o, d_r = stripe(eng, k, sb, 5)
    rf = np.ones(k, np.uint8)
    rf[k // 3] = 0
    d_x = DeviceArray(eng, k * sb)
    d_fo = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    d_fr = DeviceArray.from_numpy(eng, rf)
    with pytest.raises(rs16.Error) as e:
        rs16.decode_device(k, k, sb, d_x.ptr, d_fo.ptr, d_r.ptr, d_fr.ptr, 0, k, engine=eng, check=True)
    assert e.value.kind == "InvalidArgument"
    # and a received original the counts deny
    of = np.zeros(k, np.uint8)
    of[7] = 1
    d_fo.upload(of)
    d_fr.upload(np.ones(k, np.uint8))
    with pytest.raises(rs16.Error) as e:
        rs16.decode_device(k, k, sb, d_x.ptr, d_fo.ptr, d_r.ptr, d_fr.ptr, 0, k, engine=eng, check=True)
    assert e.value.kind == "InvalidArgument"
    # consistent flags pass the check
    d_fo.upload(np.zeros(k, np.uint8))
    rs16.decode_device(k, k, sb, d_x.ptr, d_fo.ptr, d_r.ptr, d_fr.ptr, 0, k, engine=eng, check=True)
    assert np.array_equal(d_x.download(shape=(k, sb)), original)


@pytest.mark.parametrize("k,n", [(2048, 3), (4096, 2)])
def test_batched_stripes(eng, k, n):
    sb = 128
    stripes = [generate_original(k, sb, 40 + i) for i in range(n)]
    host_o = np.concatenate([s.reshape(-1) for s in stripes])
    d_o = DeviceArray.from_numpy(eng, host_o)
    d_r = DeviceArray(eng, n * k * sb)
    rs16.encode_device_batch(k, k, sb, n, d_o.ptr, k * sb, d_r.ptr, k * sb, engine=eng)
    d_x = DeviceArray.from_numpy(eng, np.full_like(host_o, 0x77))
    d_fo = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    d_fr = DeviceArray.from_numpy(eng, np.ones(k, np.uint8))
    rs16.decode_device_batch(k, k, sb, n, d_x.ptr, k * sb, d_fo.ptr, d_r.ptr, k * sb, d_fr.ptr, 0, k, engine=eng)
    assert np.array_equal(d_x.download(shape=(n * k * sb,)), host_o)


@pytest.mark.parametrize("rate", ["high", "low"])
@pytest.mark.parametrize("k", [2048, 8192])
def test_rate_decoder(k, rate):
    # the Rate API (its counts come from its own received set); the low rate
    # erases the tail [n, 65536) as well (rate_low.rs:183-197)
    sb = 64
    original = generate_original(k, sb, k)
    recovery = O.encode(k, k, original, rate=rate)
    dec = rs16.RateDecoder(k, k, sb, rate)
    for i in range(k):
        dec.add_recovery_shard(i, recovery[i])
    with dec.decode() as res:
        got = dict(res.restored_original_iter())
    assert sorted(got) == list(range(k))
    assert all(got[i] == original[i].tobytes() for i in range(k))


def test_prepared(eng):
    k, sb = 4096, 64
    original, d_o, d_r = stripe(eng, k, sb, 11)
    d_x = DeviceArray(eng, k * sb)
    d_fo = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    d_fr = DeviceArray.from_numpy(eng, np.ones(k, np.uint8))
    side = eng.create_stream()
    try:
        rs16.decode_prepare(k, k, sb, d_fo.ptr, d_fr.ptr, 0, k, stream=side, engine=eng)
        rs16.encode_device(k, k, sb, d_o.ptr, d_r.ptr, engine=eng)
        rs16.decode_device_prepared(k, k, sb, d_x.ptr, d_r.ptr, engine=eng, check=True)
        assert np.array_equal(d_x.download(shape=(k, sb)), original)
    finally:
        eng.synchronize()
        eng.destroy_stream(side)
