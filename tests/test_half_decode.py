"""The half-transform decode identity, on the CPU oracle (no GPU).

When every original is lost, the decoder's transform input is zero on the
originals' half of the n work rows and only that half of its output is
needed.  Then (rs16_engine.cpp, DESIGN.md "Half-transform decode"):

    FFT(FD(IFFT(x)))[dst half] == FFT_dst(IFFT_src(x[src half]))

with FFT/IFFT/FD the reference's Engine ops over all n rows, skew_delta 0
(src/rate/rate_high.rs:230-234), and IFFT_src / FFT_dst the n/2-row
transforms over rows [src, src + n/2) / [dst, dst + n/2) with the twiddles of
those rows (skew_delta = the half's first row, as Engine::fft_skew_end does,
src/engine.rs:222-250).  Checked bit for bit with the restated NoSimd and
Naive engines, both halves (high rate: src = lower half; low rate: upper).
"""
import numpy as np
import pytest

import oracle_bind as O


@pytest.mark.parametrize("engine", ["nosimd", "naive"])
@pytest.mark.parametrize("L", [1, 2, 3, 4, 5, 7, 8, 9, 11])
@pytest.mark.parametrize("src_upper", [False, True])
def test_half_identity(engine, L, src_upper):
    n, sb = 1 << L, 64
    h = n // 2
    rng = np.random.default_rng(L * 2 + src_upper)
    x = rng.integers(0, 256, (n, sb), dtype=np.uint8)
    src, dst = (h, 0) if src_upper else (0, h)
    x[dst:dst + h] = 0  # no received row on the originals' half
    full = x.copy()
    O.ifft(full, 0, n, n, 0, engine)
    O.formal_derivative(full, engine)
    O.fft(full, 0, n, n, 0, engine)
    half = np.zeros_like(x)
    half[:h] = x[src:src + h]
    if h > 1:
        w = np.zeros_like(x)
        w[src:src + h] = half[:h]
        O.ifft(w, src, h, h, src, engine)  # IFFT_src (skew_delta = src)
        w[dst:dst + h] = w[src:src + h]
        O.fft(w, dst, h, h, dst, engine)   # FFT_dst (skew_delta = dst)
        got = w[dst:dst + h]
    else:
        got = half[:1]
    assert np.array_equal(got, full[dst:dst + h])


def test_truncated_trailing_rows_unaffected():
    # the decoder truncates at k + chunk (rate_high.rs:230-234); with a zero
    # tail the truncated transforms equal the full ones on the consumed rows
    n, sb, h = 256, 64, 128
    rng = np.random.default_rng(9)
    x = rng.integers(0, 256, (n, sb), dtype=np.uint8)
    x[h:] = 0
    x[100:h] = 0  # recovery count 100 < chunk 128: padding rows are zero
    a, b = x.copy(), x.copy()
    O.ifft(a, 0, n, 100 + h, 0)
    O.formal_derivative(a)
    O.fft(a, 0, n, 100 + h, 0)
    O.ifft(b, 0, n, n, 0)
    O.formal_derivative(b)
    O.fft(b, 0, n, n, 0)
    assert np.array_equal(a[h:h + 100], b[h:h + 100])
