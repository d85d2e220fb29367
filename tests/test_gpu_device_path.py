"""GPU parity of the device-resident one-shot path (the benchmark path) at
BASELINE.json's configurations, against the oracle (same ChaCha8 inputs as
benches/benchmarks.rs:21-28, seed 0) and the oracle-generated SHA-256
fixtures in tests/golden/kib_hashes.json; full-size properties: decode after
erasure restores every lost original bit-exactly, for 100 %, 1 % and random
loss patterns, both rates, single- and multi-chunk.
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu
KIB = {(c["k"], c["m"]): c for c in json.loads((Path(__file__).parent / "golden" / "kib_hashes.json").read_text())["cases"]}


@pytest.fixture(scope="module")
def eng():
    return rs16.default_engine()


def dev_encode(eng, original, m):
    k, sb = original.shape
    d_orig = DeviceArray.from_numpy(eng, original)
    d_rec = DeviceArray(eng, m * sb)
    rs16.encode_device(k, m, sb, d_orig.ptr, d_rec.ptr, engine=eng)
    return d_rec.download(shape=(m, sb))


def dev_decode(eng, original, recovery, orig_mask, rec_mask):
    k, sb = original.shape
    m = recovery.shape[0]
    holes = original.copy()
    holes[~orig_mask] = 0xA5  # garbage in lost slots must not matter
    d_orig = DeviceArray.from_numpy(eng, holes)
    d_rec = DeviceArray.from_numpy(eng, recovery)
    d_of = DeviceArray.from_numpy(eng, orig_mask.astype(np.uint8))
    d_rf = DeviceArray.from_numpy(eng, rec_mask.astype(np.uint8))
    rs16.decode_device(k, m, sb, d_orig.ptr, d_of.ptr, d_rec.ptr, d_rf.ptr, int(orig_mask.sum()),
                       int(rec_mask.sum()), engine=eng)
    return d_orig.download(shape=(k, sb))


@pytest.mark.parametrize("k,m", [(100, 100), (1000, 1000), (32768, 32768)])
def test_baseline_configs_encode_decode(eng, k, m):
    original = generate_original(k, 1024, 0)
    recovery = dev_encode(eng, original, m)
    assert hashlib.sha256(recovery.tobytes()).hexdigest() == KIB[(k, m)]["recovery_sha256"]
    # 100 % original loss: recovery 0..k given (benches/benchmarks.rs:82-87 with loss = min(k, m))
    loss = min(k, m)
    om = np.ones(k, bool)
    om[:loss] = False
    rm = np.zeros(m, bool)
    rm[:loss] = True
    restored = dev_decode(eng, original, recovery, om, rm)
    assert np.array_equal(restored, original)
    # 1 % loss
    loss = min(k, m) // 100
    if loss:
        om = np.ones(k, bool)
        om[k - loss:] = False
        rm = np.zeros(m, bool)
        rm[:loss] = True
        assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


@pytest.mark.parametrize("k,m", [(1, 1), (2, 1), (3, 5), (100, 1000), (1000, 100), (1025, 1024), (1024, 1025),
                                 (2048, 1025), (4096, 61440), (61440, 4096)])
def test_device_path_vs_oracle(eng, k, m):
    sb = 128 if k * m > 10**7 else 1024
    original = generate_original(k, sb, k % 251)
    recovery = dev_encode(eng, original, m)
    want = O.encode(k, m, original)
    assert np.array_equal(recovery, want)
    rng = np.random.default_rng(k * 7 + m)
    # random erasures: keep exactly k of the k+m shards
    keep = rng.permutation(k + m)[:k]
    om = np.zeros(k, bool)
    rm = np.zeros(m, bool)
    om[keep[keep < k]] = True
    rm[keep[keep >= k] - k] = True
    assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


def test_decode_nothing_to_do_and_not_enough(eng):
    original = generate_original(4, 64, 1)
    recovery = dev_encode(eng, original, 2)
    out = dev_decode(eng, original, recovery, np.ones(4, bool), np.zeros(2, bool))
    assert np.array_equal(out, original)
    with pytest.raises(rs16.Error) as e:
        dev_decode(eng, original, recovery, np.array([1, 0, 0, 1], bool), np.array([1, 0], bool))
    assert e.value == rs16.Error("NotEnoughShards", original_count=4, original_received_count=2,
                                 recovery_received_count=1)


@pytest.mark.parametrize("k,m,sb", [(32768, 32768, 64), (1000, 1000, 64 * 3), (300, 300, 64 * 9)])
def test_odd_shard_widths(eng, k, m, sb):
    # shard widths that are not a multiple of the 512-byte tile slab
    original = generate_original(k, sb, 5)
    recovery = dev_encode(eng, original, m)
    assert np.array_equal(recovery, O.encode(k, m, original))
    om = np.zeros(k, bool)
    om[::3] = True
    rm = np.zeros(m, bool)
    rm[: k - om.sum()] = True
    assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)
