"""GPU parity of the Engine-level ops (through the C ABI) against the oracle.

Reference semantics: src/engine.rs:140-260 (trait), NoSimd
(src/engine/engine_nosimd.rs) as the bit-exact target.  Integer work, so the
bar is bit equality.  Truncated transforms are compared on the shards the
reference contract defines: [pos, pos+truncated_size) (src/engine.rs:150-195);
IFFT inputs have the zero tail the contract requires.
"""
import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return rs16.default_engine()


def rand_shards(n, sb, seed):
    return np.random.default_rng(seed).integers(0, 256, (n, sb), dtype=np.uint8)


@pytest.mark.parametrize("log_m", [0, 1, 255, 12345, 65534, 65535])
@pytest.mark.parametrize("sb", [64, 1024, 64 * 33])
def test_mul(eng, log_m, sb):
    x = rand_shards(3, sb, log_m)
    d = DeviceArray.from_numpy(eng, x)
    eng.mul(d.ptr, x.nbytes, log_m)
    want = x.copy()
    O.mul(want.reshape(-1), log_m)
    assert np.array_equal(d.download(shape=x.shape), want)


def test_xor_and_xor_within(eng):
    x, y = rand_shards(8, 128, 1), rand_shards(8, 128, 2)
    dx, dy = DeviceArray.from_numpy(eng, x), DeviceArray.from_numpy(eng, y)
    eng.xor(dx.ptr, dy.ptr, x.nbytes)
    assert np.array_equal(dx.download(shape=x.shape), x ^ y)
    eng.xor_within(dx.ptr, 8, 128, 0, 4, 4)
    z = x ^ y
    z[0:4] ^= z[4:8]
    assert np.array_equal(dx.download(shape=x.shape), z)


FFT_CASES = [
    # (shard_count, shard_bytes, pos, size, trunc, skew_delta)
    (1, 64, 0, 1, 1, 0),
    (2, 64, 0, 2, 2, 0),
    (4, 64, 0, 4, 3, 0),
    (16, 128, 0, 16, 16, 16),
    (32, 1024, 0, 32, 20, 0),
    (64, 192, 0, 64, 64, 64),
    (256, 1024, 0, 256, 200, 0),
    (512, 64, 0, 512, 512, 512),
    (1024, 1024, 0, 1024, 1000, 1024),
    (2048, 1024, 0, 2048, 2024, 0),
    (4096, 576, 0, 2048, 2048, 2048),
    (4096, 64, 2048, 2048, 2048, 4096),
    (8192, 64, 4096, 4096, 100, 8192),
    (32768, 64, 0, 32768, 32768, 32768),
    (65536, 64, 0, 65536, 65536, 0),
]


@pytest.mark.parametrize("case", FFT_CASES, ids=lambda c: "x".join(map(str, c)))
def test_fft(eng, case):
    n, sb, pos, size, trunc, skew = case
    x = rand_shards(n, sb, n + size)
    d = DeviceArray.from_numpy(eng, x)
    eng.fft(d.ptr, n, sb, pos, size, trunc, skew)
    want = x.copy()
    O.fft(want, pos, size, trunc, skew)
    got = d.download(shape=x.shape)
    assert np.array_equal(got[pos:pos + trunc], want[pos:pos + trunc])
    assert np.array_equal(got[:pos], x[:pos]) and np.array_equal(got[pos + size:], x[pos + size:])


@pytest.mark.parametrize("case", FFT_CASES, ids=lambda c: "x".join(map(str, c)))
def test_ifft(eng, case):
    n, sb, pos, size, trunc, skew = case
    x = rand_shards(n, sb, 7 * n + size)
    x[pos + trunc:pos + size] = 0  # contract: zero tail (src/engine.rs:182-187)
    d = DeviceArray.from_numpy(eng, x)
    eng.ifft(d.ptr, n, sb, pos, size, trunc, skew)
    want = x.copy()
    O.ifft(want, pos, size, trunc, skew)
    got = d.download(shape=x.shape)
    assert np.array_equal(got, want)


def test_fft_skew_end_and_ifft_skew_end(eng):
    x = rand_shards(1024, 64, 3)
    d = DeviceArray.from_numpy(eng, x)
    eng.ifft_skew_end(d.ptr, 1024, 64, 256, 256, 256)
    eng.fft_skew_end(d.ptr, 1024, 64, 512, 512, 512)
    want = x.copy()
    O.ifft(want, 256, 256, 256, 512)
    O.fft(want, 512, 512, 512, 1024)
    assert np.array_equal(d.download(shape=x.shape), want)


@pytest.mark.parametrize("n", [1, 2, 4, 64, 1024])
def test_formal_derivative(eng, n):
    x = rand_shards(n, 128, n)
    d = DeviceArray.from_numpy(eng, x)
    eng.formal_derivative(d.ptr, n, 128)
    want = x.copy()
    O.formal_derivative(want)
    assert np.array_equal(d.download(shape=x.shape), want)


@pytest.mark.parametrize("trunc", [65536, 2024, 3])
def test_fwht_and_eval_poly(eng, trunc):
    # bit-exact u16 outputs (not only residues mod 65535): the engine-level
    # ops run the reference's layer order with its add_mod / sub_mod
    rng = np.random.default_rng(trunc)
    e = np.zeros(65536, np.uint16)
    e[:trunc] = rng.integers(0, 2, trunc)
    d = DeviceArray.from_numpy(eng, e)
    eng.fwht(d.ptr, trunc)
    want = e.copy()
    O.fwht(want, trunc)
    assert np.array_equal(d.download(np.uint16), want)
    d.upload(e)
    eng.eval_poly(d.ptr, trunc)
    want = e.copy()
    O.eval_poly(want, trunc)
    assert np.array_equal(d.download(np.uint16), want)


def test_fwht_full_range_values(eng):
    # arbitrary u16 inputs (65535 included) -- exercises every add_mod /
    # sub_mod wrap, where 0 and 65535 outputs differ bit-wise
    rng = np.random.default_rng(5)
    e = rng.integers(0, 65536, 65536, dtype=np.uint32).astype(np.uint16)
    e[:64] = 65535
    d = DeviceArray.from_numpy(eng, e)
    eng.fwht(d.ptr, 65536)
    want = e.copy()
    O.fwht(want, 65536)
    assert np.array_equal(d.download(np.uint16), want)


def test_invalid_arguments(eng):
    d = DeviceArray(eng, 64 * 8)
    with pytest.raises(rs16.Error) as ex:
        eng.fft(d.ptr, 8, 64, 0, 3, 3, 0)  # size not a power of two
    assert ex.value.kind == "InvalidArgument"
    with pytest.raises(rs16.Error):
        eng.fft(d.ptr, 8, 64, 4, 8, 8, 0)  # out of range
    with pytest.raises(rs16.Error):
        eng.formal_derivative(d.ptr, 6, 64)  # not a power of two
