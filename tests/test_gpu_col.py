"""GPU parity of the one-launch column codec (rs16_col.hip): every encode whose
transform has 512 or 1024 rows and every half-transform decode (all originals
lost) over 512 / 1024-row halves runs as one kernel per call.  Its results
must equal the oracle's (the NoSimd restatement, src/rate/rate_high.rs:44-83,
src/rate/rate_low.rs:44-83) and the pass codec's (rs16.DIAG_NO_COLUMN) bit for
bit: high and low rate, partial chunks, every shard width class, column
slices of wider arrays, batched stripes, the in-place work buffer of the Rate
API, and decodes with lost recovery shards and garbage in the lost slots.
"""
import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return rs16.default_engine()


@pytest.fixture
def force_column():
    old = rs16.set_diagnostics(rs16.DIAG_FORCE_COLUMN)
    yield
    rs16.set_diagnostics(old)


@pytest.fixture
def no_column():
    old = rs16.set_diagnostics(rs16.DIAG_NO_COLUMN)
    yield
    rs16.set_diagnostics(old)


@pytest.fixture(params=["radix2", "radix4"])
def form(request):
    # the encode / half decode of 2^8 .. 2^10 rows run the radix-2 kernel
    # (col2_kernel, 2 rows per thread) by default; RS16_DIAG_COL_RADIX4 keeps
    # the 4-rows-per-thread kernel (col_kernel) for them
    old = rs16.set_diagnostics(0)  # (keeps the flags other fixtures set)
    rs16.set_diagnostics(old | (rs16.DIAG_COL_RADIX4 if request.param == "radix4" else 0))
    yield request.param
    rs16.set_diagnostics(old)


def dev_encode(eng, original, m):
    k, sb = original.shape
    d_orig = DeviceArray.from_numpy(eng, original)
    d_rec = DeviceArray.from_numpy(eng, np.full((m, sb), 0x5A, np.uint8))
    rs16.encode_device(k, m, sb, d_orig.ptr, d_rec.ptr, engine=eng)
    return d_rec.download(shape=(m, sb))


def dev_decode(eng, original, recovery, orig_mask, rec_mask):
    k, sb = original.shape
    m = recovery.shape[0]
    holes = original.copy()
    holes[~orig_mask] = 0xA5
    d_orig = DeviceArray.from_numpy(eng, holes)
    d_rec = DeviceArray.from_numpy(eng, recovery)
    d_of = DeviceArray.from_numpy(eng, orig_mask.astype(np.uint8))
    d_rf = DeviceArray.from_numpy(eng, rec_mask.astype(np.uint8))
    rs16.decode_device(k, m, sb, d_orig.ptr, d_of.ptr, d_rec.ptr, d_rf.ptr, int(orig_mask.sum()),
                       int(rec_mask.sum()), engine=eng, check=True)
    return d_orig.download(shape=(k, sb))


# (k, m): chunk = 512 / 1024 rows on the high-rate side, and low-rate cases
# whose one recovery chunk is 512 / 1024 rows
CASES = [(1, 257), (100, 300), (257, 512), (512, 512), (300, 1000), (1000, 1000), (1024, 1024), (511, 513),
         (700, 600), (1000, 520), (1024, 600), (600, 1024),
         # 64 / 128 / 256-row transforms (one wave or less per workgroup)
         (50, 60), (100, 100), (30, 100), (200, 256), (256, 129), (100, 40), (64, 33), (1, 64)]


@pytest.mark.parametrize("k,m", CASES)
@pytest.mark.parametrize("sb", [64, 1024])
def test_col_encode_vs_oracle(eng, k, m, sb, form):
    original = generate_original(k, sb, k + 7 * m + sb)
    assert np.array_equal(dev_encode(eng, original, m), O.encode(k, m, original))


@pytest.mark.parametrize("sb", [192, 4096, 65536])
def test_col_encode_widths(eng, sb, force_column):
    # (wider than the codec's default limit: forced, rs16.DIAG_FORCE_COLUMN)
    k, m = 1000, 1000
    original = generate_original(k, sb, sb)
    recovery = dev_encode(eng, original, m)
    assert np.array_equal(recovery, O.encode(k, m, original))
    om, rm = np.zeros(k, bool), np.ones(m, bool)
    assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


@pytest.mark.parametrize("k,m", [(1000, 1000), (300, 1000), (512, 512), (1024, 600)])
def test_col_matches_pass_codec(eng, k, m, no_column):
    # (the fixture sets DIAG_NO_COLUMN for the reference run; the column run
    # switches it off around its own call)
    sb = 256
    original = generate_original(k, sb, 3 * k + m)
    want = dev_encode(eng, original, m)
    old = rs16.set_diagnostics(0)
    try:
        got = dev_encode(eng, original, m)
    finally:
        rs16.set_diagnostics(old)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("k,m", [(1000, 1000), (512, 512), (257, 300), (100, 1000), (1024, 1024), (600, 1024),
                                 (1000, 520), (100, 100), (60, 64), (200, 256), (33, 64), (128, 200)])
@pytest.mark.parametrize("lost_rec", [0, 5])
def test_col_half_decode(eng, k, m, lost_rec, form):
    """Every original lost, recovery shards given (some of them lost too):
    the half-transform decode; restored bit for bit."""
    if m - lost_rec < k:
        pytest.skip("not enough recovery shards")
    sb = 128
    original = generate_original(k, sb, k + m)
    recovery = O.encode(k, m, original)
    om = np.zeros(k, bool)
    rm = np.ones(m, bool)
    rng = np.random.default_rng(k * m)
    if lost_rec:
        rm[rng.choice(m, lost_rec, replace=False)] = False
    assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


@pytest.mark.parametrize("rate", ["high", "low"])
@pytest.mark.parametrize("k,m", [(1000, 1000), (512, 300), (300, 512), (100, 100), (200, 60)])
def test_col_rate_api_in_place(eng, rate, k, m):
    """The Rate API's work buffer: originals, recovery and restored rows
    share one array (in == out for the column encode)."""
    sb = 64
    if not rs16.supports(k, m, rate):
        pytest.skip("unsupported")
    original = generate_original(k, sb, k ^ m)
    enc = rs16.RateEncoder(k, m, sb, rate, engine=eng)
    for o in original:
        enc.add_original_shard(o)
    with enc.encode() as res:
        rec = np.stack([np.frombuffer(r, np.uint8) for r in res.recovery_iter()])
    assert np.array_equal(rec, O.encode(k, m, original, rate=rate))
    # lose the first min(k, m) originals (all of them when k <= m: the half decode)
    lost = min(k, m)
    dec = rs16.RateDecoder(k, m, sb, rate, engine=eng)
    for i in range(lost, k):
        dec.add_original_shard(i, original[i])
    for i in range(lost):
        dec.add_recovery_shard(i, rec[i])
    with dec.decode() as res:
        got = dict(res.restored_original_iter())
    assert sorted(got) == list(range(lost))
    assert all(np.array_equal(np.frombuffer(got[i], np.uint8), original[i]) for i in range(lost))


@pytest.mark.parametrize("k,m", [
    # low rate, 128-row chunks (colm_kernel: one wave per recovery chunk)
    (100, 1000), (65, 300), (128, 2048),
    # low rate, 256-1024-row chunks (a workgroup per quad column and recovery chunk)
    (300, 2000), (200, 1500), (1000, 3000), (1000, 6000), (512, 2100),
    # high rate multi-chunk (chunk IFFTs, then the FFT of their XOR)
    (1000, 100), (3000, 1000), (2000, 300)])
@pytest.mark.parametrize("sb", [64, 1024])
def test_col_multi_chunk_rate_api_in_place(eng, k, m, sb):
    """Multi-chunk encodes through the Rate API, whose work buffer holds the
    originals and receives the recovery in place (rate_low.rs:44-83,
    rate_high.rs:44-83): no workgroup may overwrite originals another one
    has not read yet (chunk 0's recovery rows overlay them)."""
    original = generate_original(k, sb, 13 * k + m + sb)
    want = O.encode(k, m, original)
    for rnd in range(2):  # (a second round on the same encoder: stale rows in the buffer)
        enc = rs16.ReedSolomonEncoder(k, m, sb, engine=eng)
        for o in original:
            enc.add_original_shard(o)
        with enc.encode() as res:
            rec = np.stack([np.frombuffer(r, np.uint8) for r in res.recovery_iter()])
        assert np.array_equal(rec, want), rnd


@pytest.mark.parametrize("k,m,n,sb", [(1000, 1000, 5, 128), (512, 512, 3, 128), (300, 1000, 4, 128),
                                      (1000, 1000, 6, 1024), (100, 100, 7, 192)])
def test_col_batched_stripes(eng, k, m, n, sb, force_column, form):
    pad = 64
    so, sr = k * sb + pad, m * sb + pad
    stripes = [generate_original(k, sb, 11 * i + k) for i in range(n)]
    host_o = np.full(n * so, 0xEE, np.uint8)
    for i, o in enumerate(stripes):
        host_o[i * so:i * so + k * sb] = o.reshape(-1)
    d_o = DeviceArray.from_numpy(eng, host_o)
    d_r = DeviceArray.from_numpy(eng, np.full(n * sr, 0x77, np.uint8))
    rs16.encode_device_batch(k, m, sb, n, d_o.ptr, so, d_r.ptr, sr, engine=eng)
    got = d_r.download(shape=(n * sr,))
    recs = []
    for i, o in enumerate(stripes):
        want = O.encode(k, m, o)
        recs.append(want)
        assert np.array_equal(got[i * sr:i * sr + m * sb].reshape(m, sb), want), i
        assert (got[i * sr + m * sb:(i + 1) * sr] == 0x77).all(), i
    # batched half decode: every original of every stripe lost
    d_o2 = DeviceArray.from_numpy(eng, np.full(n * so, 0xA5, np.uint8))
    d_of = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    d_rf = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    rs16.decode_device_batch(k, m, sb, n, d_o2.ptr, so, d_of.ptr, d_r.ptr, sr, d_rf.ptr, 0, m, engine=eng)
    back = d_o2.download(shape=(n * so,))
    for i, o in enumerate(stripes):
        assert np.array_equal(back[i * so:i * so + k * sb].reshape(k, sb), o), i
        assert (back[i * so + k * sb:(i + 1) * so] == 0xA5).all(), i


@pytest.mark.parametrize("slices", [2, 3])
def test_col_column_slices(slices):
    """Column slices of wider arrays (row stride > slice width; rs16_engine_set_slices):
    every slice is its own column launch, encode and half decode."""
    eng = rs16.Engine(0)
    eng.set_slices(slices)
    k, m, sb = 1000, 1000, 1024 + 64 * slices
    original = generate_original(k, sb, 99 + slices)
    recovery = dev_encode(eng, original, m)
    assert np.array_equal(recovery, O.encode(k, m, original))
    om, rm = np.zeros(k, bool), np.ones(m, bool)
    assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


def test_col_host_multi(eng):
    k, m, sb = 1000, 1000, 1024
    original = generate_original(k, sb, 98)
    rec = np.zeros((m, sb), np.uint8)
    rs16.encode_host_multi(k, m, sb, original, rec, [eng, rs16.Engine(0)])
    assert np.array_equal(rec, O.encode(k, m, original))


@pytest.mark.parametrize("k,m", [(900, 1000), (100, 120)])
def test_col_decode_check_counts(eng, k, m):
    """The column decoder evaluates the polynomial itself (no eval kernel) and
    writes the per-chunk received counts rs16_decode_check reads: a caller
    whose counts disagree with its flags gets InvalidArgument."""
    sb = 64
    original = generate_original(k, sb, 5)
    recovery = O.encode(k, m, original)
    d_orig = DeviceArray.from_numpy(eng, np.zeros_like(original))
    d_rec = DeviceArray.from_numpy(eng, recovery)
    d_of = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    d_rf = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    rs16.decode_device(k, m, sb, d_orig.ptr, d_of.ptr, d_rec.ptr, d_rf.ptr, 0, m, engine=eng, check=True)
    assert np.array_equal(d_orig.download(shape=(k, sb)), original)
    with pytest.raises(rs16.Error) as e:
        rs16.decode_device(k, m, sb, d_orig.ptr, d_of.ptr, d_rec.ptr, d_rf.ptr, 0, m - 1, engine=eng, check=True)
    assert e.value.kind == "InvalidArgument"


@pytest.mark.parametrize("k,m", [(100, 100), (300, 300), (200, 256), (50, 60), (512, 512), (33, 64), (700, 300),
                                 # 2^11 work rows (8-wave workgroups)
                                 (1000, 1000), (1000, 100), (1024, 1024), (600, 1000), (1500, 500),
                                 # low rate (originals = segment A, erasure tail of ones)
                                 (100, 1000), (60, 1000), (200, 700)])
@pytest.mark.parametrize("pattern", ["1pct", "random", "mixed", "tail_rec", "two_blocks"])
def test_col_general_decode(eng, k, m, pattern, form):
    """The general decode (any loss pattern) of up to 2048 work rows in one
    launch: polynomial, gather of both segments, IFFT, formal derivative, FFT,
    reveal (rate_high.rs:168-247); every lost original restored bit for bit,
    received originals untouched.  tail_rec / two_blocks: the radix-2
    kernel's per-wave skips (128-row blocks with no received row, with no
    lost original) at other blocks than the reference pattern's."""
    sb = 64
    original = generate_original(k, sb, 3 * k + m)
    recovery = O.encode(k, m, original)
    rng = np.random.default_rng(k + 5 * m)
    om, rm = np.ones(k, bool), np.zeros(m, bool)
    if pattern == "1pct":  # benches/benchmarks.rs:81-105
        loss = max(1, min(k, m) // 100)
        om[k - loss:] = False
        rm[:loss] = True
    elif pattern == "tail_rec":  # the last recovery shards, lost originals at the front
        loss = max(1, min(k, m) // 50)
        om[:loss] = False
        rm[m - loss:] = True
    elif pattern == "two_blocks":  # lost originals in two distant 128-row blocks
        loss = max(2, min(k, m) // 40)
        half = loss // 2
        om[:half] = False
        om[k - (loss - half):] = False
        rm[rng.choice(m, min(m, loss + 1), replace=False)] = True
    else:
        loss = int(rng.integers(1, min(k, m) + 1)) if pattern == "random" else min(k, m) // 2
        om[rng.choice(k, loss, replace=False)] = False
        rm[rng.choice(m, min(m, loss + (3 if m > loss + 3 else 0)), replace=False)] = True
    if rm.sum() + om.sum() < k:
        pytest.skip("not enough shards")
    assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


def test_col_general_decode_matches_pass_codec(eng, no_column):
    k, m, sb = 300, 300, 128
    original = generate_original(k, sb, 17)
    recovery = O.encode(k, m, original)
    om, rm = np.ones(k, bool), np.zeros(m, bool)
    om[::7] = False
    rm[:60] = True
    want = dev_decode(eng, original, recovery, om, rm)
    old = rs16.set_diagnostics(0)
    try:
        got = dev_decode(eng, original, recovery, om, rm)
    finally:
        rs16.set_diagnostics(old)
    assert np.array_equal(got, want) and np.array_equal(got, original)


@pytest.mark.parametrize("rate", ["high", "low"])
@pytest.mark.parametrize("k,m", [(300, 300), (100, 1000), (1000, 100)])
def test_col_general_decode_rate_api(eng, rate, k, m):
    """General decodes through the Rate API's work buffer, both rates forced."""
    sb = 64
    if not rs16.supports(k, m, rate):
        pytest.skip("unsupported")
    original = generate_original(k, sb, 7 * k + m)
    recovery = O.encode(k, m, original, rate=rate)
    rng = np.random.default_rng(k * m + len(rate))
    lost = sorted(rng.choice(k, min(k, m) // 3 + 1, replace=False).tolist())
    dec = rs16.RateDecoder(k, m, sb, rate, engine=eng)
    for i in range(k):
        if i not in lost:
            dec.add_original_shard(i, original[i])
    for i in rng.choice(m, len(lost), replace=False).tolist():
        dec.add_recovery_shard(int(i), recovery[i])
    with dec.decode() as res:
        got = dict(res.restored_original_iter())
    assert sorted(got) == lost
    assert all(np.array_equal(np.frombuffer(got[i], np.uint8), original[i]) for i in lost)


@pytest.mark.parametrize("k,m", [(1000, 100), (129, 100), (2048, 128), (300, 65), (2049, 100),
                                 (100, 1000), (100, 129), (128, 2048), (65, 300), (100, 2100), (1, 200)])
@pytest.mark.parametrize("sb", [64, 192, 1024])
def test_col_multi_chunk_encode(eng, k, m, sb):
    # multi-chunk encodes of 128-row chunks in one launch (colm_kernel, one
    # wave per chunk; rate_high.rs:44-83 / rate_low.rs:44-83): 2..16 chunks of
    # either rate, partial last chunks; 17 chunks take the pass form.  Equal
    # to the oracle and to the pass codec (RS16_DIAG_NO_COLUMN).
    original = generate_original(k, sb, 5 * k + m + sb)
    got = dev_encode(eng, original, m)
    assert np.array_equal(got, O.encode(k, m, original))
    old = rs16.set_diagnostics(rs16.DIAG_NO_COLUMN)
    try:
        assert np.array_equal(dev_encode(eng, original, m), got)
    finally:
        rs16.set_diagnostics(old)


@pytest.mark.parametrize("k,m", [(3000, 1000), (1025, 1000), (2000, 300), (1500, 200), (10000, 1000), (40000, 1000),
                                 (1000, 3000), (1000, 1025), (300, 2000), (200, 1500), (1000, 10000), (1000, 40000)])
@pytest.mark.parametrize("sb", [64, 1024])
def test_col_chunks_encode(eng, k, m, sb):
    # multi-chunk encodes of 256 / 512 / 1024-row chunks in the radix-2
    # column codec (rate_high.rs:44-83: every chunk's IFFT, then the FFT of
    # their XOR -- two launches; rate_low.rs:44-83: one launch, a workgroup
    # per quad column and recovery chunk); partial last chunks, and up to 40
    # chunks (beyond the codec's default chunk-row limit: forced,
    # RS16_DIAG_FORCE_COLUMN).  Equal to the oracle and to the pass codec
    # (RS16_DIAG_NO_COLUMN).
    original = generate_original(k, sb, 7 * k + m + sb)
    old = rs16.set_diagnostics(rs16.DIAG_FORCE_COLUMN)
    try:
        got = dev_encode(eng, original, m)
    finally:
        rs16.set_diagnostics(old)
    assert np.array_equal(got, O.encode(k, m, original))
    old = rs16.set_diagnostics(rs16.DIAG_NO_COLUMN)
    try:
        assert np.array_equal(dev_encode(eng, original, m), got)
    finally:
        rs16.set_diagnostics(old)
