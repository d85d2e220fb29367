"""The split device decode (rs16_decode_prepare + rs16_decode_device_prepared,
include/rs16.h): the erasure locator of the received pattern on a side
stream (src/rate/rate_high.rs:168-202, src/engine.rs:207-218) while the
engine stream encodes the stripe whose recovery the decode then reads
(src/rate/rate_high.rs:203-247).  Every result must equal the oracle's
originals bit for bit, exactly as rs16_decode_device's; the error and
ordering rules of the split are checked too."""
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


def masks(k, m, pattern, seed):
    rng = np.random.default_rng(seed)
    om, rm = np.ones(k, bool), np.zeros(m, bool)
    lost = min(k, m)
    if pattern == "all":
        om[:lost] = False
        rm[:lost] = True
    elif pattern == "1pct":  # benches/benchmarks.rs:81-105
        L = max(1, lost // 100)
        om[k - L:] = False
        rm[:L] = True
    elif pattern == "none":
        rm[:3] = True
    else:
        nl = int(rng.integers(1, lost + 1))
        om[rng.choice(k, nl, replace=False)] = False
        rm[rng.choice(m, min(m, nl + 2), replace=False)] = True
    return om, rm


@pytest.mark.parametrize("k,m,sb,pattern", [
    (32768, 32768, 64, "all"),      # half-transform decode, 3 passes
    (32768, 32768, 128, "1pct"),    # general decode, tile_last, lost-range pruning
    (4096, 4096, 256, "scatter"),   # general decode
    (1000, 1000, 1024, "all"),      # column codec: the kernel evaluates the polynomial (nothing to prepare)
    (1000, 1000, 64, "1pct"),       # column general decode over 2^11 work rows
    (300, 3000, 64, "scatter"),     # low rate
    (100, 100, 64, "none"),         # nothing to restore
])
def test_prepare_then_encode_then_decode(eng, k, m, sb, pattern):
    side = eng.create_stream()
    try:
        original = generate_original(k, sb, k % 251)
        om, rm = masks(k, m, pattern, k + m)
        d_o = DeviceArray.from_numpy(eng, original)
        d_r = DeviceArray(eng, m * sb)
        held = original.copy()
        held[~om] = 0xA5
        d_x = DeviceArray.from_numpy(eng, held)
        d_fo = DeviceArray.from_numpy(eng, om.astype(np.uint8))
        d_fr = DeviceArray.from_numpy(eng, rm.astype(np.uint8))
        for rnd in range(3):  # (repeated: each preparation waits for the previous decode)
            d_x.upload(held)
            rs16.decode_prepare(k, m, sb, d_fo.ptr, d_fr.ptr, int(om.sum()), int(rm.sum()), stream=side, engine=eng)
            rs16.encode_device(k, m, sb, d_o.ptr, d_r.ptr, engine=eng)  # the recovery the decode reads
            rs16.decode_device_prepared(k, m, sb, d_x.ptr, d_r.ptr, engine=eng, check=True)
            assert np.array_equal(d_x.download(shape=(k, sb)), original), rnd
        assert np.array_equal(d_r.download(shape=(m, sb)), O.encode(k, m, original))
    finally:
        eng.synchronize()
        eng.destroy_stream(side)


def test_prepared_rules(eng):
    k, m, sb = 2000, 2000, 64
    original = generate_original(k, sb, 3)
    recovery = O.encode(k, m, original)
    d_r = DeviceArray.from_numpy(eng, recovery)
    d_x = DeviceArray.from_numpy(eng, np.zeros_like(original))
    d_fo = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    d_fr = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    # no preparation
    with pytest.raises(rs16.Error) as e:
        rs16.decode_device_prepared(k, m, sb, d_x.ptr, d_r.ptr, engine=eng)
    assert e.value.kind == "InvalidArgument"
    # the preparation's own checks (src/rate/decoder_work.rs:120-139)
    with pytest.raises(rs16.Error) as e:
        rs16.decode_prepare(k, m, sb, d_fo.ptr, d_fr.ptr, 0, 10, engine=eng)
    assert e.value == rs16.Error("NotEnoughShards", original_count=k, original_received_count=0,
                                 recovery_received_count=10)
    # another geometry than prepared
    rs16.decode_prepare(k, m, sb, d_fo.ptr, d_fr.ptr, 0, m, engine=eng)
    with pytest.raises(rs16.Error) as e:
        rs16.decode_device_prepared(k, m, 128, d_x.ptr, d_r.ptr, engine=eng)
    assert e.value.kind == "InvalidArgument"
    # (the failed call consumed nothing: the preparation is still there)
    rs16.decode_device_prepared(k, m, sb, d_x.ptr, d_r.ptr, engine=eng)
    assert np.array_equal(d_x.download(shape=(k, sb)), original)
    # consumed once
    with pytest.raises(rs16.Error) as e:
        rs16.decode_device_prepared(k, m, sb, d_x.ptr, d_r.ptr, engine=eng)
    assert e.value.kind == "InvalidArgument"
    # a plain decode in between discards the preparation (and orders after it)
    side = eng.create_stream()
    try:
        rs16.decode_prepare(k, m, sb, d_fo.ptr, d_fr.ptr, 0, m, stream=side, engine=eng)
        d_x.upload(np.zeros_like(original))
        rs16.decode_device(k, m, sb, d_x.ptr, d_fo.ptr, d_r.ptr, d_fr.ptr, 0, m, engine=eng)
        assert np.array_equal(d_x.download(shape=(k, sb)), original)
        with pytest.raises(rs16.Error) as e:
            rs16.decode_device_prepared(k, m, sb, d_x.ptr, d_r.ptr, engine=eng)
        assert e.value.kind == "InvalidArgument"
        # a second preparation replaces the first
        om, rm = masks(k, m, "scatter", 9)
        d_fo2 = DeviceArray.from_numpy(eng, om.astype(np.uint8))
        d_fr2 = DeviceArray.from_numpy(eng, rm.astype(np.uint8))
        rs16.decode_prepare(k, m, sb, d_fo.ptr, d_fr.ptr, 0, m, stream=side, engine=eng)
        rs16.decode_prepare(k, m, sb, d_fo2.ptr, d_fr2.ptr, int(om.sum()), int(rm.sum()), stream=side, engine=eng)
        held = original.copy()
        held[~om] = 0x5A
        d_x.upload(held)
        rs16.decode_device_prepared(k, m, sb, d_x.ptr, d_r.ptr, engine=eng, check=True)
        assert np.array_equal(d_x.download(shape=(k, sb)), original)
    finally:
        eng.synchronize()
        eng.destroy_stream(side)


def test_prepared_discarded_by_host_batch(eng):
    """a pipelined host batch decode evaluates on its lanes' own
    eval sets, but still rewrites the engine's path state (identity logs,
    fused eval, column eval) a prepared decode reads.  A preparation followed
    by a host batch decode is therefore discarded: the prepared call refuses
    (InvalidArgument) instead of running the batch's path on logs that were
    never written, and a fresh preparation restores bit for bit."""
    k = m = 32768
    sb = 64
    original = generate_original(k, sb, 21)
    recovery = O.encode(k, m, original)
    d_r = DeviceArray.from_numpy(eng, recovery)
    d_x = DeviceArray.from_numpy(eng, np.zeros_like(original))
    # the preparation: every original lost (identity logs, no eval kernel)
    d_fo = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    d_fr = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    # the host batch: the reference bench's 1 % loss (general decode)
    om, rm = masks(k, m, "1pct", 0)
    h_o = np.stack([original, original])
    h_o[:, ~om] = 0x3C
    h_r = np.stack([recovery, recovery])
    fo = np.ascontiguousarray(np.stack([om, om]).astype(np.uint8))
    fr = np.ascontiguousarray(np.stack([rm, rm]).astype(np.uint8))
    rs16.decode_prepare(k, m, sb, d_fo.ptr, d_fr.ptr, 0, m, engine=eng)
    rs16.decode_host_batch(k, m, sb, 2, h_o, k * sb, fo, k, h_r, m * sb, fr, m, engine=eng)
    for i in range(2):
        assert np.array_equal(h_o[i], original), i
    with pytest.raises(rs16.Error) as e:
        rs16.decode_device_prepared(k, m, sb, d_x.ptr, d_r.ptr, engine=eng)
    assert e.value.kind == "InvalidArgument"
    rs16.decode_prepare(k, m, sb, d_fo.ptr, d_fr.ptr, 0, m, engine=eng)
    rs16.decode_device_prepared(k, m, sb, d_x.ptr, d_r.ptr, engine=eng, check=True)
    assert np.array_equal(d_x.download(shape=(k, sb)), original)


def test_prepared_with_slices():
    e = rs16.Engine(0)
    try:
        e.set_slices(3)
        k, m, sb = 4096, 4096, 192 * 2
        original = generate_original(k, sb, 4)
        d_o = DeviceArray.from_numpy(e, original)
        d_r = DeviceArray(e, m * sb)
        om, rm = masks(k, m, "all", 1)
        d_x = DeviceArray.from_numpy(e, np.zeros_like(original))
        d_fo = DeviceArray.from_numpy(e, om.astype(np.uint8))
        d_fr = DeviceArray.from_numpy(e, rm.astype(np.uint8))
        side = e.create_stream()
        rs16.decode_prepare(k, m, sb, d_fo.ptr, d_fr.ptr, 0, m, stream=side, engine=e)
        rs16.encode_device(k, m, sb, d_o.ptr, d_r.ptr, engine=e)
        rs16.decode_device_prepared(k, m, sb, d_x.ptr, d_r.ptr, engine=e, check=True)
        assert np.array_equal(d_x.download(shape=(k, sb)), original)
        e.synchronize()
        e.destroy_stream(side)
    finally:
        e.close()
