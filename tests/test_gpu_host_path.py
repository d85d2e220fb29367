"""GPU parity of the host-resident one-shot codec (rs16_encode_host /
rs16_decode_host, include/rs16.h): shards in host memory, column slices
pipelined over two streams.  Results must equal the oracle's recovery shards
and the originals bit for bit for any slice width (multiples of 64, with a
last partial slice), both rates, pinned and pageable host buffers."""
import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import PinnedArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return rs16.default_engine()


@pytest.mark.parametrize("k,m,sb,slice_bytes,pinned", [
    (1000, 1000, 1024, 0, True),     # default slices (S/8)
    (1000, 1000, 1024, 192, False),  # pageable buffers, partial last slice
    (3000, 30000, 320, 128, True),   # low rate
    (32768, 32768, 256, 64, True),   # max shard count, 64-byte slices
    (100, 3, 64 * 5, 64, False),     # multi-chunk high rate
])
def test_host_encode_decode(eng, k, m, sb, slice_bytes, pinned):
    original = generate_original(k, sb, 3)
    if pinned:
        ho, hr = PinnedArray(eng, k * sb), PinnedArray(eng, m * sb)
        ho.array[:] = original.reshape(-1)
        horig, hrec = ho.array.reshape(k, sb), hr.array.reshape(m, sb)
    else:
        horig, hrec = original.copy(), np.zeros((m, sb), np.uint8)
    rs16.encode_host(k, m, sb, horig, hrec, slice_bytes, engine=eng)
    assert np.array_equal(hrec, O.encode(k, m, original))
    loss = min(k, m)  # as benches/benchmarks.rs:82-87 at 100 %
    of = np.ones(k, np.uint8)
    of[:loss] = 0
    rf = np.zeros(m, np.uint8)
    rf[:loss] = 1
    horig[:loss] = 0xA5  # lost slots hold garbage
    rs16.decode_host(k, m, sb, horig, of, hrec, rf, slice_bytes, engine=eng)
    assert np.array_equal(horig, original)


def test_host_decode_errors(eng):
    original = generate_original(4, 64, 1)
    rec = np.zeros((2, 64), np.uint8)
    rs16.encode_host(4, 2, 64, original, rec, engine=eng)
    with pytest.raises(rs16.Error) as e:
        rs16.decode_host(4, 2, 64, original.copy(), np.array([1, 0, 0, 1], np.uint8), rec,
                         np.array([1, 0], np.uint8), engine=eng)
    assert e.value == rs16.Error("NotEnoughShards", original_count=4, original_received_count=2,
                                 recovery_received_count=1)


# Scratch ownership of the two host slots: every slot
# runs its slices on its own stream with its own work buffers -- the low-rate
# multi-chunk encoder's transformed originals (U) and the column decoder's
# received counts included; nothing falls back to engine-wide scratch.  Many
# narrow slices (>= 4 per slot) make the two slots overlap for most of the
# call; results must equal the oracle's bit for bit, every time.
@pytest.mark.parametrize("k,m,sb,slice_bytes,loss", [
    (300, 3000, 1024, 128, "all"),    # low rate, 6 recovery chunks of 512 (encode_low_multi per slot)
    (1000, 1000, 1024, 128, "1pct"),  # general decode of 2^11 work rows: column codec, polynomial in the kernel
    (100, 1000, 512, 64, "1pct"),     # low-rate column general decode (n = 2^11 rows)
    (1000, 1000, 1024, 64, "all"),    # half-transform column decode, 16 slices
])
def test_host_slots_own_scratch(eng, k, m, sb, slice_bytes, loss):
    original = generate_original(k, sb, 11)
    want = O.encode(k, m, original)
    for rep in range(3):
        hrec = np.zeros((m, sb), np.uint8)
        rs16.encode_host(k, m, sb, original, hrec, slice_bytes, engine=eng)
        assert np.array_equal(hrec, want), f"encode, repetition {rep}"
        L = min(k, m) if loss == "all" else max(1, min(k, m) // 100)
        of = np.ones(k, np.uint8)
        of[k - L:] = 0
        rf = np.zeros(m, np.uint8)
        rf[:L] = 1
        horig = original.copy()
        horig[k - L:] = 0x5A
        rs16.decode_host(k, m, sb, horig, of, hrec, rf, slice_bytes, engine=eng)
        assert np.array_equal(horig, original), f"decode, repetition {rep}"


@pytest.mark.parametrize("k,m,sb,n,pinned,pattern", [
    (1000, 1000, 1024, 5, True, "all"),       # column codec, half decode, odd stripe count
    (1000, 1000, 1024, 4, False, "mixed"),    # pageable buffers
    (4096, 4096, 256, 6, True, "mixed"),      # pass codec, per-stripe losses (some stripes lose nothing)
    (3000, 30000, 128, 3, True, "mixed"),     # low rate
    (100, 3, 64 * 5, 7, True, "scatter"),     # multi-chunk high rate
    (32768, 32768, 64, 3, True, "all"),       # max shard count
    (50, 60, 64, 1, True, "scatter"),         # one stripe
])
def test_host_batch_pipelined(eng, k, m, sb, n, pinned, pattern):
    """rs16_encode_host_batch / rs16_decode_host_batch:
    stripes with gaps between them, two in flight on two copy streams; every
    stripe's recovery equals the oracle's, every lost original comes back,
    received originals and the gaps are untouched."""
    pad = 64
    so, sr = k * sb + pad, m * sb + pad
    stripes = [generate_original(k, sb, 40 + i) for i in range(n)]

    def buf(nbytes, fill):
        if pinned:
            p = PinnedArray(eng, nbytes)
            p.array[:] = fill
            return p, p.array
        return None, np.full(nbytes, fill, np.uint8)

    keep_o, ho = buf(n * so, 0xEE)
    keep_r, hr = buf(n * sr, 0x77)
    for i, o in enumerate(stripes):
        ho[i * so:i * so + k * sb] = o.reshape(-1)
    rs16.encode_host_batch(k, m, sb, n, ho, so, hr, sr, engine=eng)
    recs = []
    for i, o in enumerate(stripes):
        rec = hr[i * sr:i * sr + m * sb].reshape(m, sb)
        assert np.array_equal(rec, O.encode(k, m, o)), i
        assert (hr[i * sr + m * sb:(i + 1) * sr] == 0x77).all(), i
        recs.append(rec.copy())
    # per-stripe loss patterns
    rng = np.random.default_rng(k + n)
    fso, fsr = k + 1, m + 3
    fo = np.zeros(n * fso, np.uint8)
    fr = np.zeros(n * fsr, np.uint8)
    for i in range(n):
        kind = pattern if pattern != "mixed" else ("all", "scatter", "none")[i % 3]
        om, rm = np.ones(k, bool), np.zeros(m, bool)
        lost = min(k, m)
        if kind == "all":
            om[:lost] = False
        elif kind == "scatter":
            om[rng.choice(k, int(rng.integers(1, lost + 1)), replace=False)] = False
        rm[rng.choice(m, min(m, int((~om).sum()) + 1), replace=False)] = True
        fo[i * fso:i * fso + k] = om
        fr[i * fsr:i * fsr + m] = rm
        seg = ho[i * so:i * so + k * sb].reshape(k, sb)
        seg[~om] = 0xA5
        hr[i * sr:i * sr + m * sb].reshape(m, sb)[~rm] = 0x3C  # not-received recovery holds garbage
    rs16.decode_host_batch(k, m, sb, n, ho, so, fo, fso, hr, sr, fr, fsr, engine=eng)
    for i, o in enumerate(stripes):
        assert np.array_equal(ho[i * so:i * so + k * sb].reshape(k, sb), o), i
        assert (ho[i * so + k * sb:(i + 1) * so] == 0xEE).all(), i


def test_host_batch_errors(eng):
    k, m, sb = 10, 5, 64
    ho, hr = np.zeros(3 * k * sb, np.uint8), np.zeros(3 * m * sb, np.uint8)
    fo, fr = np.ones(3 * k, np.uint8), np.zeros(3 * m, np.uint8)
    fo[k:k + 7] = 0  # stripe 1 lost 7 originals with no recovery shard
    with pytest.raises(rs16.Error) as e:
        rs16.decode_host_batch(k, m, sb, 3, ho, k * sb, fo, k, hr, m * sb, fr, m, engine=eng)
    assert e.value == rs16.Error("NotEnoughShards", original_count=k, original_received_count=3,
                                 recovery_received_count=0)
    with pytest.raises(rs16.Error) as e:  # stride below a stripe
        rs16.encode_host_batch(k, m, sb, 2, ho, k * sb - 64, hr, m * sb, engine=eng)
    assert e.value.kind == "InvalidArgument"
    rs16.encode_host_batch(k, m, sb, 0, ho, k * sb, hr, m * sb, engine=eng)  # no stripes: OK
