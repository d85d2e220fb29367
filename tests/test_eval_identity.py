"""The identity-multiplier decode (rs16_engine::identity_logs, DESIGN.md
3.13) rests on one fact about eval_poly (src/engine.rs:207-218): when the
erased work rows are exactly one half of the n = 2^(L+1) rows -- every
original lost, every recovery shard received, k = m = n / 2 -- every erasure
log is 0 mod 65535, so "MULTIPLY SHARDS" (src/rate/rate_high.rs:203-228,
rate_low.rs:203-228) and REVEAL ERASURES (:236-242) multiply by exp(0) = 1.
Checked here on the oracle's eval_poly for every L and both rates (the low
rate also erases the tail [n, 65536), rate_low.rs:183-197), and shown not
to hold for patterns one row off (where the engine evaluates the polynomial).
"""
import numpy as np
import pytest

import oracle_bind as O


def erasures(L, high, shift=0):
    n, half = 2 << L, 1 << L
    e = np.zeros(65536, np.uint16)
    if high:  # recovery = rows [0, half), originals = [half, n): originals erased
        e[half + shift:n] = 1
        return e, n
    e[:half + shift] = 1  # low rate: originals = rows [0, half), recovery [half, n)
    e[n:] = 1
    return e, 65536


@pytest.mark.parametrize("high", [True, False])
@pytest.mark.parametrize("L", range(0, 16))
def test_whole_half_erasure_logs_are_zero(L, high):
    e, trunc = erasures(L, high)
    O.eval_poly(e, trunc)
    n = 2 << L
    assert set((e[:n].astype(np.int64) % 65535).tolist()) == {0}


@pytest.mark.parametrize("high", [True, False])
@pytest.mark.parametrize("L", [4, 11, 15])
def test_one_row_off_is_not_identity(L, high):
    # one more / one fewer erased row: the logs are no longer all 0
    e, trunc = erasures(L, high, shift=1)
    O.eval_poly(e, trunc)
    n = 2 << L
    assert len(set((e[:n].astype(np.int64) % 65535).tolist())) > 1
