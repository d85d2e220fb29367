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


def _varied_masks(k, m, n, seed, mode):
    """Per-stripe received masks: each stripe its own random loss set (mode
    "mixed": some stripes lose every original, some lose a few, some none),
    the recovery shards received chosen at random to cover the losses."""
    rng = np.random.default_rng(seed)
    oms, rms = [], []
    for i in range(n):
        om = np.ones(k, bool)
        kind = mode if mode != "mixed" else ("all", "few", "none", "scatter")[i % 4]
        lost = min(k, m)
        if kind == "all":
            om[:lost] = False
        elif kind == "few":
            om[rng.choice(k, max(1, lost // 50), replace=False)] = False
        elif kind == "scatter":
            om[rng.choice(k, int(rng.integers(1, lost + 1)), replace=False)] = False
        nlost = int((~om).sum())
        rm = np.zeros(m, bool)
        extra = int(rng.integers(0, m - nlost + 1)) if m > nlost else 0
        rm[rng.choice(m, nlost + extra, replace=False)] = True
        oms.append(om)
        rms.append(rm)
    return oms, rms


@pytest.mark.parametrize("k,m,sb,n,mode", [
    (1000, 1000, 1024, 8, "scatter"),   # column general decode (n = 2^11 work rows), per-stripe flags
    (1000, 1000, 1024, 5, "all"),       # every stripe loses every original (half decode), own recovery sets
    (1000, 1000, 64, 6, "mixed"),
    (100, 100, 1024, 9, "mixed"),
    (4096, 4096, 128, 4, "mixed"),      # pass codec, per-stripe eval grid rows (aligned one-kernel form)
    (4000, 3000, 64, 3, "scatter"),     # unaligned segments: two-kernel eval form, lost-range pruning
    (32768, 32768, 64, 2, "mixed"),     # the 65536-row decode, T = 8 passes finishing eval's last H_lo
    (300, 3000, 64, 3, "mixed"),        # low rate
    (3, 5, 64, 7, "mixed"),
    (100, 100, 64, 300, "mixed"),       # more stripes than one group (256): two groups of eval + passes
    (3, 5, 64, 513, "mixed"),           # three groups, the last of one stripe
])
def test_decode_batch_varied(k, m, sb, n, mode):
    # stripes with losses of their own, one call; every
    # stripe restored bit for bit (the oracle's encode gives the recovery),
    # garbage in the lost slots, gap bytes and recovery untouched
    eng = rs16.default_engine()
    pad = 64
    so, sr = k * sb + pad, m * sb + pad
    stripes = [generate_original(k, sb, 13 * i + k + m) for i in range(n)]
    recs = [O.encode(k, m, o) for o in stripes]
    oms, rms = _varied_masks(k, m, n, k * 7 + n, mode)
    fso, fsr = k + 3, m + 5  # flag strides wider than a stripe's flags
    host_o = np.full(n * so, 0x3C, np.uint8)
    host_r = np.full(n * sr, 0x3C, np.uint8)
    fo = np.full(n * fso, 0xFF, np.uint8)
    fr = np.full(n * fsr, 0xFF, np.uint8)
    for i in range(n):
        held = stripes[i].copy()
        held[~oms[i]] = 0xA5
        host_o[i * so:i * so + k * sb] = held.reshape(-1)
        rec = recs[i].copy()
        rec[~rms[i]] = 0x5A  # recovery shards not received hold garbage too
        host_r[i * sr:i * sr + m * sb] = rec.reshape(-1)
        fo[i * fso:i * fso + k] = oms[i]
        fr[i * fsr:i * fsr + m] = rms[i]
    d_o, d_r = DeviceArray.from_numpy(eng, host_o), DeviceArray.from_numpy(eng, host_r)
    d_fo, d_fr = DeviceArray.from_numpy(eng, fo), DeviceArray.from_numpy(eng, fr)
    rs16.decode_device_batch_varied(k, m, sb, n, d_o.ptr, so, d_fo.ptr, fso, d_r.ptr, sr, d_fr.ptr, fsr,
                                    [int(x.sum()) for x in oms], [int(x.sum()) for x in rms], engine=eng)
    got = d_o.download(shape=(n * so,))
    for i in range(n):
        assert np.array_equal(got[i * so:i * so + k * sb].reshape(k, sb), stripes[i]), i
        assert (got[i * so + k * sb:(i + 1) * so] == 0x3C).all(), i
    assert np.array_equal(d_r.download(shape=(n * sr,)), host_r)


def test_decode_batch_varied_errors():
    eng = rs16.default_engine()
    d = DeviceArray(eng, 64 * 8)
    f = DeviceArray(eng, 64)
    # nothing to restore anywhere / no stripes: OK without a launch
    rs16.decode_device_batch_varied(2, 2, 64, 2, d.ptr, 128, f.ptr, 2, d.ptr, 128, f.ptr, 2, [2, 2], [0, 1], engine=eng)
    rs16.decode_device_batch_varied(2, 2, 64, 0, d.ptr, 128, f.ptr, 2, d.ptr, 128, f.ptr, 2, [], [], engine=eng)
    with pytest.raises(rs16.Error) as e:  # the second stripe has too few shards
        rs16.decode_device_batch_varied(2, 2, 64, 2, d.ptr, 128, f.ptr, 2, d.ptr, 128, f.ptr, 2, [2, 0], [0, 1],
                                        engine=eng)
    assert e.value == rs16.Error("NotEnoughShards", original_count=2, original_received_count=0,
                                 recovery_received_count=1)
    with pytest.raises(rs16.Error) as e:  # flag stride below the count
        rs16.decode_device_batch_varied(2, 2, 64, 2, d.ptr, 128, f.ptr, 1, d.ptr, 128, f.ptr, 2, [1, 1], [1, 1],
                                        engine=eng)
    assert e.value.kind == "InvalidArgument"


@pytest.mark.parametrize("diag", ["DIAG_TILE_LAST", "DIAG_NO_TILE_LAST"])
@pytest.mark.parametrize("mode", ["mixed", "scatter"])
def test_decode_batch_varied_last_pass_paths(diag, mode):
    # the 65536-row varied decode with its last pass forced to each form
    # (tile_last_kernel with per-stripe lost ranges / zero tiles, and the
    # 8-wave items)
    old = rs16.set_diagnostics(getattr(rs16, diag))
    try:
        test_decode_batch_varied(32768, 32768, 64, 3, mode)
    finally:
        rs16.set_diagnostics(old)
