"""The general decode's middle pass as a matrix (rs16_tables.cpp
mid_matrix_entries, mid_direct_kernel): the decode's core
FFT(FD(IFFT(x))) over n = 2^L rows (src/rate/rate_high.rs:203-247 with the
sequential formal derivative, src/engine.rs formal_derivative) equals
FFT_lo(M z + L z) per 2^lo-row block, z = IFFT_lo(x), where M is one
2^hi x 2^hi matrix for every column j (rows t << lo | j) built from the unit
vectors exactly as mid_matrix_entries builds it, and L is the formal
derivative's low-bit terms.  Checked against the oracle's own IFFT / formal
derivative / FFT on random data; the GPU kernel is checked end to end by
tests/test_gpu_mid_direct.py."""
import numpy as np
import pytest

import oracle_bind as O

GM = 65535


def tables():
    return (O.table("exp").astype(np.int64), O.table("log").astype(np.int64), O.table("skew").astype(np.int64))


def gmul(x, lm, exp, log):
    """x (array of elements) times the element of log lm."""
    x = np.asarray(x, np.int64)
    out = exp[(log[x] + lm) % GM]
    return np.where(x == 0, 0, out)


def mid_matrix(L, exp, log, skew):
    """mid_matrix_entries, element form: M[o][t] (rs16_tables.cpp)."""
    lo, hi = L // 2, L - L // 2
    N = 1 << hi
    v = np.zeros((N, N), np.int64)  # column c of the identity in column c
    v[np.arange(N), np.arange(N)] = exp[0]
    for kb in range(hi):  # IFFT, low layers first
        d = 1 << kb
        for r in range(0, N, 2 * d):
            lm = int(skew[(r << lo) + (1 << (lo + kb)) - 1])
            a, b = v[r:r + d].copy(), v[r + d:r + 2 * d].copy()
            b ^= a
            if lm != GM:
                a ^= gmul(b, lm, exp, log)
            v[r:r + d], v[r + d:r + 2 * d] = a, b
    w = v.copy()  # (I + H): row i takes row i | b for every tile bit b clear in i
    for i in range(N):
        b = 1
        while b < N:
            if not i & b:
                w[i] ^= v[i | b]
            b <<= 1
    for kb in range(hi - 1, -1, -1):  # FFT, high layers first
        d = 1 << kb
        for r in range(0, N, 2 * d):
            lm = int(skew[(r << lo) + (1 << (lo + kb)) - 1])
            a, b = w[r:r + d].copy(), w[r + d:r + 2 * d].copy()
            if lm != GM:
                a ^= gmul(b, lm, exp, log)
            b ^= a
            w[r:r + d], w[r + d:r + 2 * d] = a, b
    return w


def to_shards(vals):  # rows x 32 elements -> rows x 64 bytes (low bytes, then high bytes)
    out = np.zeros((vals.shape[0], 64), np.uint8)
    out[:, :32] = vals & 0xFF
    out[:, 32:] = vals >> 8
    return out


def from_shards(sh):
    return sh[:, :32].astype(np.int64) | (sh[:, 32:].astype(np.int64) << 8)


@pytest.mark.parametrize("L", [6, 9])
def test_decode_core_equals_matrix_form(L):
    exp, log, skew = tables()
    lo, hi = L // 2, L - L // 2
    n = 1 << L
    x = np.random.default_rng(L).integers(0, 65536, (n, 32))
    full = to_shards(x)
    O.ifft(full, 0, n, n, 0)
    O.formal_derivative(full)
    O.fft(full, 0, n, n, 0)
    z = to_shards(x)
    for b in range(n >> lo):
        O.ifft(z, b << lo, 1 << lo, 1 << lo, b << lo)
    zv = from_shards(z)
    M = mid_matrix(L, exp, log, skew)
    u = np.zeros_like(zv)
    for j in range(1 << lo):
        rows = (np.arange(1 << hi) << lo) | j
        for o in range(1 << hi):
            acc = np.zeros(32, np.int64)
            for t in range(1 << hi):
                if M[o, t]:
                    acc ^= gmul(zv[rows[t]], int(log[M[o, t]]), exp, log)
            u[rows[o]] = acc
    y = u.copy()
    for r in range(n):
        for b in range(lo):
            if not (r >> b) & 1:
                y[r] ^= zv[r | (1 << b)]
    ys = to_shards(y)
    for b in range(n >> lo):
        O.fft(ys, b << lo, 1 << lo, 1 << lo, b << lo)
    assert np.array_equal(from_shards(ys), from_shards(full))
