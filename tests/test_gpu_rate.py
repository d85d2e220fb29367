"""GPU parity of the Rate / ReedSolomon layers (through the C ABI).

Same cases and the same golden SHA-256 values as the reference's own tests
(roundtrip_single! / roundtrip_two_rounds!, src/test_util.rs:93-359, hash
tables :583-837), now with the MI355X engine in place of Naive/NoSimd; plus
the error-path tests of test_rate_{en,de}coder_errors! (src/test_util.rs:364-568)
and src/lib.rs:375-581.
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import rs16
from conftest import expand
from rs16.util import generate_original

pytestmark = pytest.mark.gpu
GOLD = json.loads((Path(__file__).parent / "golden" / "reference_hashes.json").read_text())
E = rs16.Error


def roundtrip(enc, dec, case, device_input=False):
    k, sb = case["k"], case["shard_bytes"]
    original = generate_original(k, sb, case["seed"])
    for s in original:
        enc.add_original_shard(s)
    with enc.encode() as result:
        recovery = list(result.recovery_iter())
    assert hashlib.sha256(b"".join(recovery)).hexdigest() == case["hash"]
    got = set()
    for i in expand(case["dec_original"]):
        dec.add_original_shard(i, original[i])
        got.add(i)
    for i in expand(case["dec_recovery"]):
        dec.add_recovery_shard(i, recovery[i])
    with dec.decode() as result:
        restored = dict(result.restored_original_iter())
    assert set(restored) == set(range(k)) - got
    for i, r in restored.items():
        assert r == original[i].tobytes(), i


def single(case):
    enc = rs16.RateEncoder(case["k"], case["m"], case["shard_bytes"], case["rate"])
    dec = rs16.RateDecoder(case["k"], case["m"], case["shard_bytes"], case["rate"])
    roundtrip(enc, dec, case)


@pytest.mark.parametrize("rate", ["default", "high", "low"])
def test_tiny_tables(rate):
    for case in GOLD["tiny"][rate]:
        single(case)


@pytest.mark.parametrize("case", GOLD["single"], ids=lambda c: f'{c["rate"]}-{c["k"]}-{c["m"]}')
def test_single_round(case):
    single(case)


@pytest.mark.parametrize("case", GOLD["two_rounds"], ids=lambda c: f'{c["rate"]}-{c["a"]["k"]}:{c["a"]["m"]}-{c["b"]["k"]}:{c["b"]["m"]}')
def test_two_rounds(case):
    a, b = case["a"], case["b"]
    enc = rs16.RateEncoder(a["k"], a["m"], a["shard_bytes"], case["rate"])
    dec = rs16.RateDecoder(a["k"], a["m"], a["shard_bytes"], case["rate"])
    roundtrip(enc, dec, a)
    if case["explicit_reset"]:
        enc.reset(b["k"], b["m"], b["shard_bytes"])
        dec.reset(b["k"], b["m"], b["shard_bytes"])
    roundtrip(enc, dec, b)


@pytest.mark.parametrize("case", GOLD["large"], ids=lambda c: f'{c["rate"]}-{c["k"]}-{c["m"]}')
def test_large_reference_vectors(case):
    # The reference's #[ignore] cases: max shard counts, multi-chunk high
    # rate (60000:3000), low rate with partial chunks.
    single(case)


def test_one_shot_roundtrip():
    # src/lib.rs:356-369
    original = generate_original(2, 1024, 123)
    recovery = rs16.encode(2, 3, list(original))
    assert hashlib.sha256(b"".join(recovery)).hexdigest() == next(
        c["hash"] for c in GOLD["single"] if c["rate"] == "default")
    restored = rs16.decode(2, 3, [], [(0, recovery[0]), (1, recovery[1])])
    assert restored == {0: original[0].tobytes(), 1: original[1].tobytes()}


def test_encoder_result_views():
    # src/encoder_result.rs:100-134
    original = generate_original(2, 1024, 123)
    enc = rs16.ReedSolomonEncoder(2, 3, 1024)
    for o in original:
        enc.add_original_shard(o)
    res = enc.encode()
    allr = [res.recovery(0), res.recovery(1), res.recovery(2)]
    assert res.recovery(3) is None
    assert list(res.recovery_iter()) == allr


def test_decoder_result_views():
    # src/decoder_result.rs:101-140
    original = generate_original(3, 1024, 0)
    enc = rs16.ReedSolomonEncoder(3, 2, 1024)
    dec = rs16.ReedSolomonDecoder(3, 2, 1024)
    for o in original:
        enc.add_original_shard(o)
    with enc.encode() as r:
        recovery = list(r.recovery_iter())
    dec.add_original_shard(1, original[1])
    dec.add_recovery_shard(0, recovery[0])
    dec.add_recovery_shard(1, recovery[1])
    res = dec.decode()
    assert res.restored_original(0) == original[0].tobytes()
    assert res.restored_original(1) is None
    assert res.restored_original(2) == original[2].tobytes()
    assert res.restored_original(3) is None
    assert list(res.restored_original_iter()) == [(0, original[0].tobytes()), (2, original[2].tobytes())]


@pytest.mark.parametrize("rate", ["high", "low", "default"])
def test_encoder_errors(rate):
    # test_rate_encoder_errors! (src/test_util.rs:364-440)
    R = lambda *a: rs16.RateEncoder(*a, rate=rate)
    enc = R(1, 1, 64)
    with pytest.raises(E) as e:
        enc.add_original_shard(bytes(128))
    assert e.value == E("DifferentShardSize", shard_bytes=64, got=128)
    with pytest.raises(E) as e:
        R(1, 1, 123)
    assert e.value == E("InvalidShardSize", shard_bytes=123)
    with pytest.raises(E) as e:
        R(1, 1, 64).reset(1, 1, 123)
    assert e.value == E("InvalidShardSize", shard_bytes=123)
    with pytest.raises(E) as e:
        R(1, 1, 64).encode()
    assert e.value == E("TooFewOriginalShards", original_count=1, original_received_count=0)
    enc = R(1, 1, 64)
    enc.add_original_shard(bytes(64))
    with pytest.raises(E) as e:
        enc.add_original_shard(bytes(64))
    assert e.value == E("TooManyOriginalShards", original_count=1)
    with pytest.raises(E) as e:
        R(0, 1, 64)
    assert e.value == E("UnsupportedShardCount", original_count=0, recovery_count=1)
    with pytest.raises(E) as e:
        R(1, 1, 64).reset(0, 1, 64)
    assert e.value == E("UnsupportedShardCount", original_count=0, recovery_count=1)


@pytest.mark.parametrize("rate", ["high", "low", "default"])
def test_decoder_errors(rate):
    # test_rate_decoder_errors! (src/test_util.rs:445-568)
    R = lambda *a: rs16.RateDecoder(*a, rate=rate)
    with pytest.raises(E) as e:
        R(1, 1, 64).add_original_shard(0, bytes(128))
    assert e.value == E("DifferentShardSize", shard_bytes=64, got=128)
    with pytest.raises(E) as e:
        R(1, 1, 64).add_recovery_shard(0, bytes(128))
    assert e.value == E("DifferentShardSize", shard_bytes=64, got=128)
    d = R(1, 1, 64)
    d.add_original_shard(0, bytes(64))
    with pytest.raises(E) as e:
        d.add_original_shard(0, bytes(64))
    assert e.value == E("DuplicateOriginalShardIndex", index=0)
    d = R(1, 1, 64)
    d.add_recovery_shard(0, bytes(64))
    with pytest.raises(E) as e:
        d.add_recovery_shard(0, bytes(64))
    assert e.value == E("DuplicateRecoveryShardIndex", index=0)
    with pytest.raises(E) as e:
        R(1, 1, 64).add_original_shard(1, bytes(64))
    assert e.value == E("InvalidOriginalShardIndex", original_count=1, index=1)
    with pytest.raises(E) as e:
        R(1, 1, 64).add_recovery_shard(1, bytes(64))
    assert e.value == E("InvalidRecoveryShardIndex", recovery_count=1, index=1)
    with pytest.raises(E) as e:
        R(1, 1, 123)
    assert e.value == E("InvalidShardSize", shard_bytes=123)
    with pytest.raises(E) as e:
        R(1, 1, 64).reset(1, 1, 123)
    assert e.value == E("InvalidShardSize", shard_bytes=123)
    with pytest.raises(E) as e:
        R(1, 1, 64).decode()
    assert e.value == E("NotEnoughShards", original_count=1, original_received_count=0, recovery_received_count=0)
    with pytest.raises(E) as e:
        R(0, 1, 64)
    assert e.value == E("UnsupportedShardCount", original_count=0, recovery_count=1)
    with pytest.raises(E) as e:
        R(1, 1, 64).reset(0, 1, 64)
    assert e.value == E("UnsupportedShardCount", original_count=0, recovery_count=1)


def test_rate_limits():
    # src/rate/rate_high.rs:458-486, rate_low.rs:458-486
    with pytest.raises(E) as e:
        rs16.RateDecoder(4096, 61440, 64, "high")
    assert e.value == E("UnsupportedShardCount", original_count=4096, recovery_count=61440)
    rs16.RateDecoder(61440, 4096, 64, "high")
    rs16.RateEncoder(61440, 4096, 64, "high")
    rs16.RateEncoder(4096, 61440, 64, "low")
    with pytest.raises(E):
        rs16.RateEncoder(61440, 4096, 64, "low")


def test_one_shot_errors():
    # src/lib.rs:375-581 (the cases that reach an encoder/decoder)
    with pytest.raises(E) as e:
        rs16.encode(2, 1, [bytes(64), bytes(128)])
    assert e.value == E("DifferentShardSize", shard_bytes=64, got=128)
    with pytest.raises(E) as e:
        rs16.encode(1, 1, [b""])
    assert e.value == E("InvalidShardSize", shard_bytes=0)
    with pytest.raises(E) as e:
        rs16.encode(1, 1, [bytes(64), bytes(64)])
    assert e.value == E("TooManyOriginalShards", original_count=1)
    with pytest.raises(E) as e:
        rs16.decode(2, 1, [(0, bytes(64)), (1, bytes(128))], [(0, bytes(64))])
    assert e.value == E("DifferentShardSize", shard_bytes=64, got=128)
    with pytest.raises(E) as e:
        rs16.decode(1, 2, [(0, bytes(64))], [(0, bytes(64)), (1, bytes(128))])
    assert e.value == E("DifferentShardSize", shard_bytes=64, got=128)
    with pytest.raises(E) as e:
        rs16.decode(1, 1, [(0, b"")], [(0, bytes(64))])
    assert e.value == E("DifferentShardSize", shard_bytes=64, got=0)
    with pytest.raises(E) as e:
        rs16.decode(2, 1, [(0, bytes(64)), (0, bytes(64))], [(0, bytes(64))])
    assert e.value == E("DuplicateOriginalShardIndex", index=0)
    with pytest.raises(E) as e:
        rs16.decode(1, 2, [(0, bytes(64))], [(0, bytes(64)), (0, bytes(64))])
    assert e.value == E("DuplicateRecoveryShardIndex", index=0)
    with pytest.raises(E) as e:
        rs16.decode(1, 1, [(1, bytes(64))], [(0, bytes(64))])
    assert e.value == E("InvalidOriginalShardIndex", original_count=1, index=1)
    with pytest.raises(E) as e:
        rs16.decode(1, 1, [(0, bytes(64))], [(1, bytes(64))])
    assert e.value == E("InvalidRecoveryShardIndex", recovery_count=1, index=1)
    with pytest.raises(E) as e:
        rs16.decode(1, 1, [(0, bytes(64))], [(0, b"")])
    assert e.value == E("InvalidShardSize", shard_bytes=0)
