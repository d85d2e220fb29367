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
