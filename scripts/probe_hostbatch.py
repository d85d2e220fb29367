"""Pipelined host stripes (rs16_encode_host_batch / rs16_decode_host_batch):
8 x 32768:32768 x 1 KiB stripes in pinned memory, encode then 100 %-loss
decode, timed; meant to run under rocprofv3 --memory-copy-trace so that the
copy timeline shows whether H2D and D2H overlap."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import numpy as np  # noqa: E402

import rs16  # noqa: E402
from rs16.device import PinnedArray  # noqa: E402

k = m = 32768
S = 1024
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 8
pre = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # streams created before the first host call
GIB = 2.0 ** 30
eng = rs16.Engine(0)
extra_streams = [eng.create_stream() for _ in range(pre)]
if len(sys.argv) > 4 and sys.argv[4] == "rccl":  # an RCCL communicator created and closed first (as in bench.py)
    (comm,) = rs16.Comm.init_all([eng])
    comm.close()

o = np.random.default_rng(5).integers(0, 256, (k, S), dtype=np.uint8)
ho, hr = PinnedArray(eng, nb * k * S), PinnedArray(eng, nb * m * S)
ho.array.reshape(nb, k * S)[:] = o.reshape(1, -1)
fo = np.zeros(nb * k, np.uint8)
fr = np.ones(nb * m, np.uint8)
hfo, hfr = PinnedArray(eng, nb * k), PinnedArray(eng, nb * m)
hfo.array[:] = fo
hfr.array[:] = fr
if len(sys.argv) > 4 and sys.argv[4] == "oneshot":  # the one-shot host path first (as in bench.py)
    for _ in range(3):
        rs16.encode_host(k, m, S, ho.ptr, hr.ptr, engine=eng)
if len(sys.argv) > 4 and sys.argv[4].startswith("hot"):  # seconds of device-resident steps right before
    from rs16.device import DeviceArray
    d_o, d_r = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S)
    f0 = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    f1 = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    d_x = DeviceArray(eng, k * S)
    t_end = time.perf_counter() + float(sys.argv[4][3:] or 1)
    while time.perf_counter() < t_end:
        for _ in range(50):
            rs16.encode_device(k, m, S, d_o.ptr, d_r.ptr, engine=eng)
            rs16.decode_device(k, m, S, d_x.ptr, f0.ptr, d_r.ptr, f1.ptr, 0, m, engine=eng)
        eng.synchronize()
for rep in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    t = time.perf_counter()
    rs16.encode_host_batch(k, m, S, nb, ho.ptr, k * S, hr.ptr, m * S, engine=eng)
    te = time.perf_counter() - t
    ho.array.reshape(nb, k, S)[:] = 0
    t = time.perf_counter()
    rs16.decode_host_batch(k, m, S, nb, ho.ptr, k * S, hfo.ptr, k, hr.ptr, m * S, hfr.ptr, m, engine=eng)
    td = time.perf_counter() - t
    ok = all(np.array_equal(ho.array.reshape(nb, k, S)[i], o) for i in range(nb))
    print(f"rep {rep}: encode {nb * (k + m) * S / te / GIB:.1f} GiB/s ({te * 1e3:.2f} ms), "
          f"decode {nb * (k + m) * S / td / GIB:.1f} GiB/s ({td * 1e3:.2f} ms), restored {ok}", flush=True)
    # one-shot host path for comparison
    t = time.perf_counter()
    for i in range(nb):
        rs16.encode_host(k, m, S, ho.ptr + i * k * S, hr.ptr + i * m * S, engine=eng)
    t1 = time.perf_counter() - t
    print(f"rep {rep}: one-shot encode x {nb}: {nb * (k + m) * S / t1 / GIB:.1f} GiB/s (pre-created streams: {pre})",
          flush=True)
