"""Pin the CPU oracle to the reference's golden vectors.

Mirrors roundtrip_single! / roundtrip_two_rounds! (src/test_util.rs:93-359):
every case is run with BOTH restated engines (Naive and NoSimd) and must
produce the reference's SHA-256 over the concatenated recovery shards, then
decode the listed subset and restore every missing original exactly.
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as O
from conftest import expand
from rs16.util import generate_original

GOLD = json.loads((Path(__file__).parent / "golden" / "reference_hashes.json").read_text())


def roundtrip(enc, dec, case):
    k, sb = case["k"], case["shard_bytes"]
    original = generate_original(k, sb, case["seed"])
    for s in original:
        enc.add_original_shard(s)
    recovery = enc.encode()
    assert hashlib.sha256(recovery.tobytes()).hexdigest() == case["hash"]
    got = set()
    for i in expand(case["dec_original"]):
        dec.add_original_shard(i, original[i])
        got.add(i)
    for i in expand(case["dec_recovery"]):
        dec.add_recovery_shard(i, recovery[i])
    restored = dec.decode()
    for i in range(k):
        if i not in got:
            assert np.array_equal(restored[i], original[i]), i
    assert set(restored) == set(range(k)) - got


def single(case, engine):
    k, m, sb = case["k"], case["m"], case["shard_bytes"]
    enc = O.Encoder(case["rate"], engine, k, m, sb)
    dec = O.Decoder(case["rate"], engine, k, m, sb)
    roundtrip(enc, dec, case)


TINY = [c for rate in ("default", "high", "low") for c in GOLD["tiny"][rate]]


@pytest.mark.parametrize("engine", ["naive", "nosimd"])
def test_tiny_tables(engine):
    for case in TINY:
        single(case, engine)


@pytest.mark.parametrize("engine", ["naive", "nosimd"])
@pytest.mark.parametrize("case", GOLD["single"], ids=lambda c: f'{c["rate"]}-{c["k"]}-{c["m"]}')
def test_single_round(case, engine):
    single(case, engine)


@pytest.mark.parametrize("engine", ["naive", "nosimd"])
@pytest.mark.parametrize("case", GOLD["two_rounds"], ids=lambda c: f'{c["rate"]}-{c["a"]["k"]}:{c["a"]["m"]}-{c["b"]["k"]}:{c["b"]["m"]}')
def test_two_rounds(case, engine):
    a, b = case["a"], case["b"]
    enc = O.Encoder(case["rate"], engine, a["k"], a["m"], a["shard_bytes"])
    dec = O.Decoder(case["rate"], engine, a["k"], a["m"], a["shard_bytes"])
    roundtrip(enc, dec, a)
    if case["explicit_reset"]:
        enc.reset(b["k"], b["m"], b["shard_bytes"])
        dec.reset(b["k"], b["m"], b["shard_bytes"])
    roundtrip(enc, dec, b)


@pytest.mark.parametrize("case", GOLD["large"], ids=lambda c: f'{c["rate"]}-{c["k"]}-{c["m"]}')
def test_large_nosimd(case):
    # The reference's #[ignore] large cases (S = 64).  NoSimd only: ~0.1-0.5 s each.
    single(case, "nosimd")


@pytest.mark.slow
@pytest.mark.parametrize("case", GOLD["large"], ids=lambda c: f'{c["rate"]}-{c["k"]}-{c["m"]}')
def test_large_naive(case):
    single(case, "naive")
