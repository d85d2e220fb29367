"""Object lifetime, result borrowing and stream-ordering rules of the C ABI
(include/rs16.h "Conventions"):

- encoders/decoders that outlive their engine (module globals at interpreter
  exit, an explicit Engine.close()) are detached, not freed twice;
- encode / decode work in place, so a second encode/decode (or add) while the
  result is held is an error -- the reference's &mut borrow of the result
  (src/rate.rs:157-166, 235-244) makes that a compile error;
- one engine used on two streams orders the calls that share its scratch.
"""
import subprocess
import sys
import textwrap
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_module_level_objects_at_exit():
    # globals torn down after the atexit engine close: must not touch freed memory
    code = textwrap.dedent(f"""
        import sys
        sys.path[:0] = [{str(ROOT / 'reed-solomon-16_amd')!r}]
        import rs16
        ENC = rs16.ReedSolomonEncoder(4, 4, 64)
        DEC = rs16.ReedSolomonDecoder(4, 4, 64)
        for i in range(4):
            ENC.add_original_shard(bytes([i]) * 64)
        RES = ENC.encode()                   # result still held at exit
        REC = [RES.recovery(i) for i in range(4)]
        for i in range(4):
            DEC.add_recovery_shard(i, REC[i])
        DRES = DEC.decode()
        assert DRES.restored_original(2) == bytes([2]) * 64
        print("ok")
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip() == "ok"


def test_objects_outlive_closed_engine():
    eng = rs16.Engine(0)
    enc = rs16.RateEncoder(2, 2, 64, engine=eng)
    dec = rs16.RateDecoder(2, 2, 64, engine=eng)
    enc.add_original_shard(bytes(64))
    eng.close()
    with pytest.raises(rs16.Error) as e:
        enc.add_original_shard(bytes(64))
    assert e.value.kind == "InvalidArgument"
    with pytest.raises(rs16.Error):
        enc.encode()
    with pytest.raises(rs16.Error):
        dec.add_recovery_shard(0, bytes(64))
    with pytest.raises(rs16.Error):
        dec.reset(2, 2, 64)
    del enc, dec  # frees host memory only


def test_encode_while_result_held():
    original = generate_original(3, 128, 1)
    enc = rs16.ReedSolomonEncoder(3, 5, 128)
    for o in original:
        enc.add_original_shard(o)
    res = enc.encode()
    first = list(res.recovery_iter())
    with pytest.raises(rs16.Error) as e:
        enc.encode()
    assert e.value.kind == "InvalidArgument"
    with pytest.raises(rs16.Error) as e:
        enc.add_original_shard(original[0])
    assert e.value == rs16.Error("TooManyOriginalShards", original_count=3)
    assert list(res.recovery_iter()) == first  # the held result is intact
    want = O.encode(3, 5, original)
    assert b"".join(first) == want.tobytes()
    res.drop()
    for o in original:
        enc.add_original_shard(o)
    with enc.encode() as r2:
        assert list(r2.recovery_iter()) == first


def test_decode_while_result_held():
    original = generate_original(4, 64, 2)
    recovery = O.encode(4, 4, original)
    dec = rs16.ReedSolomonDecoder(4, 4, 64)
    dec.add_original_shard(1, original[1])
    for i in range(3):
        dec.add_recovery_shard(i, recovery[i])
    res = dec.decode()
    with pytest.raises(rs16.Error) as e:
        dec.decode()
    assert e.value.kind == "InvalidArgument"
    with pytest.raises(rs16.Error) as e:
        dec.add_recovery_shard(3, recovery[3])
    assert e.value.kind == "InvalidArgument"
    assert dict(res.restored_original_iter()) == {i: original[i].tobytes() for i in (0, 2, 3)}
    res.drop()  # resets the received set (DecoderResult Drop, src/decoder_result.rs:44-48)
    dec.add_original_shard(0, original[0])
    for i in (1, 2, 3):
        dec.add_recovery_shard(i, recovery[i])
    with dec.decode() as r2:
        assert dict(r2.restored_original_iter()) == {i: original[i].tobytes() for i in (1, 2, 3)}


def test_two_streams_share_engine_scratch():
    # encode of stripe X on stream A and 100 %-loss decode of stripe Y on
    # stream B, issued back to back without a host sync: both use the
    # engine's Z scratch, so the engine must order them.
    eng = rs16.Engine(0)
    k = m = 8192
    sb = 1024
    x = generate_original(k, sb, 11)
    y = generate_original(k, sb, 12)
    y_rec = O.encode(k, m, y)
    d_x = DeviceArray.from_numpy(eng, x)
    d_xr = DeviceArray(eng, m * sb)
    d_y = DeviceArray.from_numpy(eng, np.zeros_like(y))
    d_yr = DeviceArray.from_numpy(eng, y_rec)
    d_of = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    d_rf = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    sa, sb_ = eng.create_stream(), eng.create_stream()
    for _ in range(3):
        rs16.encode_device(k, m, sb, d_x.ptr, d_xr.ptr, stream=sa, engine=eng)
        rs16.decode_device(k, m, sb, d_y.ptr, d_of.ptr, d_yr.ptr, d_rf.ptr, 0, m, stream=sb_, engine=eng)
    eng.synchronize(sa)
    eng.synchronize(sb_)
    assert np.array_equal(d_xr.download(shape=(m, sb)), O.encode(k, m, x))
    assert np.array_equal(d_y.download(shape=(k, sb)), y)
    eng.destroy_stream(sa)
    eng.destroy_stream(sb_)
    eng.close()


def test_engine_own_queue():
    """rs16_engine_new_ex(RS16_ENGINE_OWN_QUEUE): the engine's stream has a
    hardware queue of its own (a CU-masked stream).  Results are those of any
    engine; two such engines run a stripe each at the same time; unknown
    flags are refused."""
    k = m = 4096
    sb = 128
    with pytest.raises(rs16.Error) as e:
        rs16.Engine(0, 1 << 7)
    assert e.value.kind == "InvalidArgument"
    engs = [rs16.Engine(0, rs16.Engine.OWN_QUEUE), rs16.Engine(0, rs16.Engine.OWN_QUEUE)]
    try:
        data = []
        for i, eng in enumerate(engs):
            o = generate_original(k, sb, 40 + i)
            d_o, d_r, d_x = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * sb), DeviceArray(eng, k * sb)
            fo = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
            fr = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
            data.append((eng, o, d_o, d_r, d_x, fo, fr))
        for _ in range(3):  # both engines' work in flight together
            for eng, o, d_o, d_r, d_x, fo, fr in data:
                rs16.encode_device(k, m, sb, d_o.ptr, d_r.ptr, engine=eng)
                rs16.decode_device(k, m, sb, d_x.ptr, fo.ptr, d_r.ptr, fr.ptr, 0, m, engine=eng)
        for eng, o, d_o, d_r, d_x, fo, fr in data:
            eng.synchronize()
            assert np.array_equal(d_r.download(shape=(m, sb)), O.encode(k, m, o))
            assert np.array_equal(d_x.download(shape=(k, sb)), o)
        del data
    finally:
        for eng in engs:
            eng.close()
