"""What in bench.py's configs4_rccl extra slows the pipelined host batch that
runs after it in the same process (scripts/probe_hb_bisect.sh
found configs4 to be the one extra that does)?  One fresh process per mode:
a preamble, then 8 x 32768:32768 x 1 KiB stripes through
rs16_encode_host_batch / rs16_decode_host_batch, 4 reps, every decode checked.
Modes:
  none      nothing first
  configs4  bench.configs4_rccl itself at one rank
  rccl      rs16.Comm.init_all + close (no collective)
  scatter   init_all + one 2 GiB scatter / gather round trip at one rank
  dev       3 x 2 GiB device arrays: upload 2 GiB, download 2 GiB, free
  host      2 x 2 GiB numpy arrays written and freed (no device)
Usage: probe_hb_cause.py MODE"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

import rs16  # noqa: E402
from rs16.device import DeviceArray, PinnedArray  # noqa: E402

k = m = 32768
S = 1024
nb = 8
GIB = 2.0 ** 30
mode = sys.argv[1] if len(sys.argv) > 1 else "none"
eng = rs16.Engine(0)
S4 = 65536
t0 = time.perf_counter()
if mode == "configs4":
    import bench
    timed, barrier = bench.make_timed(eng.synchronize, None, 1)
    res = bench.configs4_rccl(eng, k, m, 1, 0, None, timed, barrier, 8)
    print("configs4 ok", res.get("restored_stripe_verified"), flush=True)
elif mode in ("rccl", "scatter"):
    (comm,) = rs16.Comm.init_all([eng])
    if mode == "scatter":
        src = DeviceArray(eng, k * S4)
        dst = DeviceArray(eng, k * S4)
        rs16.scatter_columns([comm], 0, k, S4, [src.ptr], [dst.ptr])
        rs16.gather_columns([comm], 0, k, S4, [dst.ptr], [src.ptr])
        eng.synchronize()
        del src, dst
    comm.close()
elif mode == "dev":
    a = np.frombuffer(np.random.default_rng(4).bytes(k * S4), np.uint8)
    d1, d2, d3 = DeviceArray.from_numpy(eng, a), DeviceArray(eng, k * S4), DeviceArray(eng, k * S4)
    b = d1.download(shape=(k * S4,))
    assert np.array_equal(a, b)
    del d1, d2, d3, a, b
elif mode == "host":
    a = np.frombuffer(np.random.default_rng(4).bytes(k * S4), np.uint8)
    b = a.copy()
    assert b[123] == a[123]
    del a, b
print(f"preamble {mode}: {time.perf_counter() - t0:.2f} s", flush=True)

o = np.random.default_rng(5).integers(0, 256, (k, S), dtype=np.uint8)
ho, hr = PinnedArray(eng, nb * k * S), PinnedArray(eng, nb * m * S)
ho.array.reshape(nb, k * S)[:] = o.reshape(1, -1)
fo = np.zeros(nb * k, np.uint8)
fr = np.ones(nb * m, np.uint8)
for rep in range(4):
    t = time.perf_counter()
    rs16.encode_host_batch(k, m, S, nb, ho.ptr, k * S, hr.ptr, m * S, engine=eng)
    te = time.perf_counter() - t
    ho.array.reshape(nb, k, S)[:] = 0
    t = time.perf_counter()
    rs16.decode_host_batch(k, m, S, nb, ho.ptr, k * S, fo, k, hr.ptr, m * S, fr, m, engine=eng)
    td = time.perf_counter() - t
    ok = all(np.array_equal(ho.array.reshape(nb, k, S)[i], o) for i in range(nb))
    print(f"{mode} rep {rep}: encode {nb * (k + m) * S / te / GIB:.1f} GiB/s, "
          f"decode {nb * (k + m) * S / td / GIB:.1f} GiB/s, restored {ok}", flush=True)
