"""The algebra of the sparse eval_poly kernel (rs16_misc.hip eval_small_kernel,
DESIGN.md §3.3) against the oracle's eval_poly (src/engine.rs:207-218): for a
high-rate erasure vector that is zero from row n on (rate_high.rs:183-197),
rows [0, n) of FWHT(LogWalsh . FWHT(e)) follow from the n/256 live blocks of
row bits 8-15 alone.  CPU only; the kernel itself is covered by the GPU decode
parity tests at every high-rate n <= 2048."""
import numpy as np
import pytest

import oracle_bind as O

_POP = np.array([bin(i).count("1") & 1 for i in range(256)])
SIGN = np.where(_POP[np.arange(256)[:, None] & np.arange(256)[None, :]] == 1, -1, 1).astype(np.int64)


def sparse_eval(e, n):
    nb = max(1, n // 256)
    lw = O.table("log_walsh").astype(np.int64).reshape(256, 256)  # [h, j]: LogWalsh[256 h + j]
    x = (e[:nb * 256].astype(np.int64).reshape(nb, 256) @ SIGN.T) % 65535  # H_lo of the live blocks
    y = (SIGN[:, :nb] @ x) % 65535                                          # H_hi, all 256 h
    z = (SIGN[:nb, :] @ ((y * lw) % 65535)) % 65535                         # H_hi, live outputs
    return ((z @ SIGN.T) % 65535).reshape(-1)                               # last H_lo


@pytest.mark.parametrize("n", [64, 256, 512, 1024, 2048])
def test_sparse_eval_matches_oracle(n):
    rng = np.random.default_rng(n)
    e = np.zeros(65536, np.uint16)
    e[:n] = rng.integers(0, 2, n)
    e[n // 3: n // 2] = 1  # a padding run, as rows [m, chunk) of a high-rate decode
    want = e.copy()
    O.eval_poly(want, n)
    got = sparse_eval(e, n)[:n]
    # 65535 and 0 are the same residue (exp[65535] = exp[0], src/engine/tables.rs:118)
    assert np.array_equal(got % 65535, want[:n].astype(np.int64) % 65535)
