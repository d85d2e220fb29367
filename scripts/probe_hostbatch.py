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
o = np.random.default_rng(5).integers(0, 256, (k, S), dtype=np.uint8)
ho, hr = PinnedArray(eng, nb * k * S), PinnedArray(eng, nb * m * S)
ho.array.reshape(nb, k * S)[:] = o.reshape(1, -1)
fo = np.zeros(nb * k, np.uint8)
fr = np.ones(nb * m, np.uint8)
hfo, hfr = PinnedArray(eng, nb * k), PinnedArray(eng, nb * m)
hfo.array[:] = fo
hfr.array[:] = fr
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
