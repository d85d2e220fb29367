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
