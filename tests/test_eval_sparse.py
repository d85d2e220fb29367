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


def _nz80(f):
    """rs16_misc.hip nz80: 0x80 in every nonzero byte of u32 words."""
    return (((f & 0x7F7F7F7F) + 0x7F7F7F7F) | f) & 0x80808080


def fused_column_x(flags, j):
    """x[t] of eval_fused_kernel's workgroup j for all-flagged blocks: 256 [j == 0]
    plus (v_dot4_i32_i8 of the nonzero bits (0x80 = -128) with the +-1 Walsh
    sign bytes of each dword, accumulated) >> 7."""
    words = flags.reshape(256, 64, 4).astype(np.uint32)
    words = (words << np.array([0, 8, 16, 24], np.uint32)).sum(axis=2, dtype=np.uint64).astype(np.uint32)
    n = _nz80(words)                                                   # [block, dword]
    nb = ((n[..., None] >> np.array([0, 8, 16, 24], np.uint32)) & 0xFF).astype(np.int64)
    nb = np.where(nb > 127, nb - 256, nb)                             # as signed bytes
    sp = np.array([-1 if _POP[j & b] else 1 for b in range(4)], np.int64)
    sq = np.array([-1 if _POP[(j >> 2) & q] else 1 for q in range(64)], np.int64)
    acc = (nb * sp[None, None, :]).sum(axis=2) @ sq                    # per block
    return (256 if j == 0 else 0) + (acc >> 7)


@pytest.mark.parametrize("seed", [0, 1])
def test_fused_eval_formulation_matches_oracle(seed):
    # e = 1 - received for a decode whose segments are whole 256-row blocks
    # (eval_fused_ok); arbitrary nonzero flag bytes count as received
    rng = np.random.default_rng(seed)
    flags = rng.choice(np.array([0, 1, 2, 127, 128, 255], np.uint8), 65536, p=[0.4, 0.3, 0.1, 0.1, 0.05, 0.05])
    flags[4096:8192] = 0
    flags[8192:12288] = 1
    e = (flags == 0).astype(np.uint16)
    x = np.stack([fused_column_x(flags, j) for j in range(256)], axis=1)  # [t, j] = H_lo(e) of block t, column j
    assert np.array_equal(x, e.astype(np.int64).reshape(256, 256) @ SIGN.T)
    lw = O.table("log_walsh").astype(np.int64).reshape(256, 256)
    y = (SIGN @ x) % 65535                       # exact integers, then Z/65535
    z = (SIGN @ ((y * lw) % 65535)) % 65535
    got = ((z @ SIGN.T) % 65535).reshape(-1)
    want = e.copy()
    O.eval_poly(want, 65536)
    assert np.array_equal(got % 65535, want.astype(np.int64) % 65535)


def _fwht_int(x):
    x = x.astype(np.int64).copy()
    n = x.size
    d = 1
    while d < n:
        x = x.reshape(-1, 2, d)
        a, b = x[:, 0, :].copy(), x[:, 1, :].copy()
        x[:, 0, :], x[:, 1, :] = a + b, a - b
        x = x.reshape(-1)
        d *= 2
    return x


def conv_eval(e, n):
    """The column codec's eval_poly (rs16_col.hip col_eval; V built like
    rs16_tables.cpp col_v): for e zero outside [0, n), rows [0, n) of
    H(LogWalsh . H(e)) are the XOR convolution e (*) W, W = H(LogWalsh):
    H_n(H_n(e) . V), V = n^-1 H_n(W[0, n)) mod 65535, n^-1 = 2^(16 - log2 n)."""
    w = _fwht_int(O.table("log_walsh")) % 65535
    inv = 1 << (16 - (n.bit_length() - 1))  # n^-1 = 2^(16 - log2 n) mod 65535
    v = (_fwht_int(w[:n]) % 65535) * inv % 65535
    x = _fwht_int(e[:n]) % 65535
    return _fwht_int((x * v) % 65535) % 65535


@pytest.mark.parametrize("n", [64, 256, 1024, 2048])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_conv_eval_matches_oracle(n, seed):
    rng = np.random.default_rng(seed * 7 + n)
    e = np.zeros(65536, np.uint16)
    e[:n] = rng.integers(0, 2, n) if seed else 0
    e[n // 2 - 24: n // 2] = 1  # the padding rows [m, chunk) of a high-rate decode
    if seed == 0:
        e[n // 2:] = 0
        e[n // 2: n // 2 + 1000 * n // 2048] = 1  # 100 % original loss
    want = e.copy()
    O.eval_poly(want, n)
    assert np.array_equal(conv_eval(e, n), want[:n].astype(np.int64) % 65535)


@pytest.mark.parametrize("n", [64, 512, 2048])
def test_conv_eval_low_rate_tail(n):
    """The low rate's erasure vector is 1 from recovery_end on
    (rate_low.rs:183-197), past row n too: rows [0, n) of eval_poly are the
    n-point convolution of e[0, n) plus the constant LogWalsh[0] - sum_{j<n} W[j]
    (HostTables::col_k)."""
    rng = np.random.default_rng(n + 11)
    e = np.zeros(65536, np.uint16)
    chunk = n // 4
    e[:chunk // 2] = rng.integers(0, 2, chunk // 2)           # originals, some lost
    e[chunk: chunk + n // 2] = rng.integers(0, 2, n // 2)     # recovery, some lost
    e[chunk + n // 2:] = 1                                     # the tail, past n as well
    want = e.copy()
    O.eval_poly(want, 65536)
    lw = O.table("log_walsh").astype(np.int64)
    w = _fwht_int(lw) % 65535
    k = (int(lw[0]) - int(w[:n].sum())) % 65535
    got = (conv_eval(e, n) + k) % 65535
    assert np.array_equal(got, want[:n].astype(np.int64) % 65535)
