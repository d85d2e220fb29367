"""RCCL column-slice scatter / gather (include/rs16.h "RCCL over xGMI";
SURVEY.md 8(e), BASELINE configs[4]) on the one GPU of the test box: a
one-rank communicator (both ncclCommInitAll and ncclCommInitRank with a
unique id), so the scatter and gather are the root's own-slice copies (the
root's slice never goes through RCCL).  More ranks need more GPUs; the partition
rule they share is checked on CPU (tests/test_cabi.py), the multi-rank data
flow with gloo (tests/test_distributed.py).  Here: the slices round-trip bit
for bit, and encode + 100 %-loss decode through scatter -> device codec per
slice -> gather equals the oracle's encode of the whole stripe."""
import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = rs16.Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("how", ["init_all", "unique_id"])
def test_scatter_gather_roundtrip(eng, how):
    if how == "init_all":
        (comm,) = rs16.Comm.init_all([eng])
    else:
        comm = rs16.Comm(eng, 1, 0, rs16.Comm.unique_id())
    assert (comm.rank, comm.size) == (0, 1)
    rows, sb = 777, 1024 + 192
    data = np.random.default_rng(1).integers(0, 256, (rows, sb), dtype=np.uint8)
    full = DeviceArray.from_numpy(eng, data)
    off, w = rs16.column_slice(sb, 1, 0)
    assert (off, w) == (0, sb)
    sl = DeviceArray(eng, rows * w)
    rs16.scatter_columns([comm], 0, rows, sb, [full.ptr], [sl.ptr])
    eng.synchronize()
    assert np.array_equal(sl.download(shape=(rows, w)), data)
    back = DeviceArray.from_numpy(eng, np.zeros_like(data))
    rs16.gather_columns([comm], 0, rows, sb, [sl.ptr], [back.ptr])
    eng.synchronize()
    assert np.array_equal(back.download(shape=(rows, sb)), data)
    comm.close()


def test_configs4_flow_one_rank(eng):
    # configs[4] shape scaled down: the root's stripe -> column slices -> the
    # device codec on each slice -> recovery gathered back to the root
    (comm,) = rs16.Comm.init_all([eng])
    k = m = 4096
    sb = 8192
    original = generate_original(k, sb, 4)
    d_full = DeviceArray.from_numpy(eng, original)
    off, w = rs16.column_slice(sb, 1, 0)
    d_slice = DeviceArray(eng, k * w)
    d_rec_slice = DeviceArray(eng, m * w)
    d_rec = DeviceArray(eng, m * sb)
    rs16.scatter_columns([comm], 0, k, sb, [d_full.ptr], [d_slice.ptr])
    rs16.encode_device(k, m, w, d_slice.ptr, d_rec_slice.ptr, engine=eng)
    rs16.gather_columns([comm], 0, m, sb, [d_rec_slice.ptr], [d_rec.ptr])
    eng.synchronize()
    rec = d_rec.download(shape=(m, sb))
    assert np.array_equal(rec[:, :1024], O.encode(k, m, np.ascontiguousarray(original[:, :1024])))
    # decode at 100 % loss through the same flow: recovery scattered, the
    # originals restored per slice and gathered
    of = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    rf = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    d_rs = DeviceArray(eng, m * w)
    d_os = DeviceArray.from_numpy(eng, np.zeros((k, w), np.uint8))
    d_out = DeviceArray.from_numpy(eng, np.zeros_like(original))
    rs16.scatter_columns([comm], 0, m, sb, [d_rec.ptr], [d_rs.ptr])
    rs16.decode_device(k, m, w, d_os.ptr, of.ptr, d_rs.ptr, rf.ptr, 0, m, engine=eng)
    rs16.gather_columns([comm], 0, k, sb, [d_os.ptr], [d_out.ptr])
    eng.synchronize()
    assert np.array_equal(d_out.download(shape=(k, sb)), original)
    comm.close()


# ---- the multi-rank data path on one GPU: virtual slices
# rs16_scatter_columns_virtual / rs16_gather_columns_virtual run the same
# code as a P-rank scatter / gather (staging pack, one grouped ncclSend /
# ncclRecv per slice, unpack), with every slice owned by the one rank: RCCL
# moves P - 1 slices to the rank itself.


def _virtual_slices(eng, P, rows, sb):
    out = []
    for j in range(P):
        off, w = rs16.column_slice(sb, P, j)
        out.append((off, w, DeviceArray(eng, max(1, rows * w))))
    return out


@pytest.mark.parametrize("P,rows,sb", [(8, 333, 8192), (8, 100, 8192 + 192), (8, 64, 320), (3, 1000, 1024)])
def test_virtual_slices_roundtrip(eng, P, rows, sb):
    (comm,) = rs16.Comm.init_all([eng])
    data = np.random.default_rng(P * rows).integers(0, 256, (rows, sb), dtype=np.uint8)
    full = DeviceArray.from_numpy(eng, data)
    sl = _virtual_slices(eng, P, rows, sb)
    assert sum(w for _, w, _ in sl) == sb
    rs16.scatter_columns_virtual(comm, P, rows, sb, full.ptr, [d.ptr for _, _, d in sl])
    eng.synchronize()
    for off, w, d in sl:
        if w:
            assert np.array_equal(d.download()[:rows * w].reshape(rows, w), data[:, off:off + w])
    # gather on a caller stream (the staging buffer's last use was on the engine stream)
    st = eng.create_stream()
    back = DeviceArray.from_numpy(eng, np.zeros_like(data))
    rs16.gather_columns_virtual(comm, P, rows, sb, [d.ptr for _, _, d in sl], back.ptr, stream=st)
    eng.synchronize(st)
    assert np.array_equal(back.download(shape=(rows, sb)), data)
    eng.destroy_stream(st)
    comm.close()


def test_virtual_configs4_flow(eng):
    # BASELINE configs[4]'s data path with P = 8 (scaled to a 4096:4096 x
    # 8 KiB stripe): scatter the originals' column slices, encode every slice,
    # gather the recovery; scatter the recovery, decode every slice at 100 %
    # original loss, gather the originals.  Recovery against the oracle's
    # encode of the whole stripe, originals restored bit for bit.
    (comm,) = rs16.Comm.init_all([eng])
    P, k, m, sb = 8, 4096, 4096, 8192
    original = generate_original(k, sb, 8)
    d_full = DeviceArray.from_numpy(eng, original)
    so = _virtual_slices(eng, P, k, sb)
    sr = _virtual_slices(eng, P, m, sb)
    d_rec = DeviceArray(eng, m * sb)
    rs16.scatter_columns_virtual(comm, P, k, sb, d_full.ptr, [d.ptr for _, _, d in so])
    for (_, w, d_o), (_, _, d_r) in zip(so, sr):
        rs16.encode_device(k, m, w, d_o.ptr, d_r.ptr, engine=eng)
    rs16.gather_columns_virtual(comm, P, m, sb, [d.ptr for _, _, d in sr], d_rec.ptr)
    eng.synchronize()
    rec = d_rec.download(shape=(m, sb))
    assert np.array_equal(rec, O.encode(k, m, original))
    of = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    rf = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    for _, w, d_o in so:
        d_o.upload(np.zeros(k * w, np.uint8))  # the lost originals' slots
    rs16.scatter_columns_virtual(comm, P, m, sb, d_rec.ptr, [d.ptr for _, _, d in sr])
    for (_, w, d_o), (_, _, d_r) in zip(so, sr):
        rs16.decode_device(k, m, w, d_o.ptr, of.ptr, d_r.ptr, rf.ptr, 0, m, engine=eng)
    d_out = DeviceArray.from_numpy(eng, np.zeros_like(original))
    rs16.gather_columns_virtual(comm, P, k, sb, [d.ptr for _, _, d in so], d_out.ptr)
    eng.synchronize()
    assert np.array_equal(d_out.download(shape=(k, sb)), original)
    comm.close()
