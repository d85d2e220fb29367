"""Host-resident encode/decode (rs16_encode_host / rs16_decode_host) at
32768:32768 x 1024 B for several column-slice widths: how the 2-D pinned
copies behave as the slice narrows (diagnostic; prints one JSON line)."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import rs16  # noqa: E402
from rs16.device import PinnedArray  # noqa: E402
from rs16.util import generate_original  # noqa: E402

k = m = 32768
S = 1024
eng = rs16.Engine(0)
orig = generate_original(k, S, 0)
ho, hr, hx = PinnedArray(eng, k * S), PinnedArray(eng, m * S), PinnedArray(eng, k * S)
ho.array[:] = orig.reshape(-1)
of, rf = np.zeros(k, np.uint8), np.ones(m, np.uint8)
out = {}
for sl in (1024, 512, 256, 128):
    rs16.encode_host(k, m, S, ho.ptr, hr.ptr, sl, engine=eng)
    t0 = time.perf_counter()
    for _ in range(5):
        rs16.encode_host(k, m, S, ho.ptr, hr.ptr, sl, engine=eng)
    te = (time.perf_counter() - t0) / 5
    rs16.decode_host(k, m, S, hx.ptr, of, hr.ptr, rf, sl, engine=eng)
    assert np.array_equal(hx.array.reshape(k, S), orig)
    t0 = time.perf_counter()
    for _ in range(5):
        rs16.decode_host(k, m, S, hx.ptr, of, hr.ptr, rf, sl, engine=eng)
    td = (time.perf_counter() - t0) / 5
    out[sl] = {"encode_us": round(te * 1e6), "decode_us": round(td * 1e6)}
print(json.dumps(out))
