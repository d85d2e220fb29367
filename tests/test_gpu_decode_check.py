"""rs16_decode_check (include/rs16.h): the eval_poly kernels count the rows
the device flags mark received, per 64-row chunk and segment, and the checked
mode compares the sums with the counts the caller passed to
rs16_decode_device (a count that disagrees with the flags
restores wrong data; the reference derives its counts from its own received
set, src/rate/decoder_work.rs:62-139, so it cannot disagree there).  Every
eval_poly form is covered: one-kernel (block-aligned), two-kernel (unaligned
flag arrays), the n <= 2048 form, the low rate."""
import numpy as np
import pytest

import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,m,sb,unaligned", [(4096, 4096, 128, False), (4096, 4096, 128, True), (1000, 1000, 64, False),
                                             (100, 300, 64, False), (3000, 60000, 64, False)])
def test_counts_checked(k, m, sb, unaligned):
    eng = rs16.default_engine()
    orig = generate_original(k, sb, 9)
    d_o, d_r = DeviceArray.from_numpy(eng, orig), DeviceArray(eng, m * sb)
    rs16.encode_device(k, m, sb, d_o.ptr, d_r.ptr, engine=eng)
    rng = np.random.default_rng(k)
    lost = rng.choice(k, min(k, m) // 3 + 1, replace=False)
    om = np.ones(k, np.uint8)
    om[lost] = 0
    rm = np.zeros(m, np.uint8)
    rm[rng.choice(m, len(lost), replace=False)] = 1
    pad = 1 if unaligned else 0
    fo = np.concatenate([np.zeros(pad, np.uint8), om])
    fr = np.concatenate([np.zeros(pad, np.uint8), rm])
    d_fo, d_fr = DeviceArray.from_numpy(eng, fo), DeviceArray.from_numpy(eng, fr)
    holes = orig.copy()
    holes[lost] = 0
    d_x = DeviceArray.from_numpy(eng, holes)
    rs16.decode_device(k, m, sb, d_x.ptr, d_fo.ptr + pad, d_r.ptr, d_fr.ptr + pad, int(om.sum()), int(rm.sum()),
                       engine=eng, check=True)
    assert np.array_equal(d_x.download(shape=(k, sb)), orig)
    # the same flags with a wrong original count: detected, with the flags' counts
    d_x.upload(holes)
    with pytest.raises(rs16.Error) as e:
        rs16.decode_device(k, m, sb, d_x.ptr, d_fo.ptr + pad, d_r.ptr, d_fr.ptr + pad, int(om.sum()) - 1,
                           int(rm.sum()) + 1, engine=eng, check=True)
    assert e.value.kind == "InvalidArgument"


@pytest.mark.parametrize("k,m", [(1000, 1000), (100, 300)])
def test_counts_checked_nothing_to_restore(k, m):
    # a decode whose counts claim every original was received
    # returns without a kernel; the checked mode still compares the counts
    # with the flags (read back) instead of the previous decode's counts
    eng = rs16.default_engine()
    sb = 64
    orig = generate_original(k, sb, 5)
    d_o, d_r = DeviceArray.from_numpy(eng, orig), DeviceArray(eng, m * sb)
    rs16.encode_device(k, m, sb, d_o.ptr, d_r.ptr, engine=eng)
    om = np.ones(k, np.uint8)
    rm = np.zeros(m, np.uint8)
    rm[:3] = 1
    d_fo, d_fr = DeviceArray.from_numpy(eng, om), DeviceArray.from_numpy(eng, rm)
    # a correct "nothing to do" decode: OK
    rs16.decode_device(k, m, sb, d_o.ptr, d_fo.ptr, d_r.ptr, d_fr.ptr, k, 3, engine=eng, check=True)
    # the flags say 3 originals are lost, the counts say none: detected
    om[[0, 7, k - 1]] = 0
    d_fo.upload(om)
    with pytest.raises(rs16.Error) as e:
        rs16.decode_device(k, m, sb, d_o.ptr, d_fo.ptr, d_r.ptr, d_fr.ptr, k, 3, engine=eng, check=True)
    assert e.value.kind == "InvalidArgument"
    assert np.array_equal(d_o.download(shape=(k, sb)), orig)  # nothing written


def test_nothing_to_restore_snapshot_and_null_flags():
    # the check of a decode with nothing to restore counts a copy
    # of the flags taken at the decode's place in stream order, so flag arrays
    # the caller rewrites (or frees) afterwards do not change the answer, and
    # a NULL flag array counts as "none received".
    import ctypes as C
    from rs16._lib import RS16Error, lib

    eng = rs16.Engine(0)
    k, m, sb = 300, 300, 64
    orig = generate_original(k, sb, 6)
    d_o, d_r = DeviceArray.from_numpy(eng, orig), DeviceArray(eng, m * sb)
    rs16.encode_device(k, m, sb, d_o.ptr, d_r.ptr, engine=eng)
    om = np.ones(k, np.uint8)
    rm = np.zeros(m, np.uint8)
    rm[:5] = 1
    d_fo, d_fr = DeviceArray.from_numpy(eng, om), DeviceArray.from_numpy(eng, rm)
    rs16.decode_device(k, m, sb, d_o.ptr, d_fo.ptr, d_r.ptr, d_fr.ptr, k, 5, engine=eng)
    # the caller reuses its flag arrays before checking: the check still sees
    # the flags the decode was given
    d_fo.upload(np.zeros(k, np.uint8))
    d_fr.upload(np.ones(m, np.uint8))
    err = RS16Error()
    assert lib().rs16_decode_check(eng.h, None, C.byref(err)) == 0, err.code
    # NULL recovery flags with a zero recovery count: OK; with a nonzero count: detected
    d_fo.upload(om)
    rs16.decode_device(k, m, sb, d_o.ptr, d_fo.ptr, d_r.ptr, 0, k, 0, engine=eng, check=True)
    with pytest.raises(rs16.Error) as e:
        rs16.decode_device(k, m, sb, d_o.ptr, d_fo.ptr, d_r.ptr, 0, k, 2, engine=eng, check=True)
    assert e.value.kind == "InvalidArgument"
    assert np.array_equal(d_o.download(shape=(k, sb)), orig)
    eng.close()
