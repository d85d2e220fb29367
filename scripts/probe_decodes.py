"""Decode latencies of the non-specialised loss patterns at 32768:32768 x
1 KiB (bench.py general_decodes' patterns plus the reference bench's 1 %):
per pattern, us per decode over a loop of `reps` calls after a warm-up, and
the per-program hipEvent times of one more call; every pattern's restore is
checked.  For same-box A/Bs run it once per library (RS16_LIB).
Usage: probe_decodes.py [reps]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import numpy as np  # noqa: E402

import rs16  # noqa: E402
from rs16.device import DeviceArray  # noqa: E402
from rs16.util import generate_original  # noqa: E402

S = 1024
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
eng = rs16.Engine(0)


def pattern(name, k, m, rng):
    of = np.ones(k, np.uint8)
    rf = np.zeros(m, np.uint8)
    if name == "scattered_1pct":
        L = k // 100
        of[rng.choice(k, L, replace=False)] = 0
        rf[rng.choice(m, L, replace=False)] = 1
    elif name == "random_50pct":
        L = k // 2
        of[rng.choice(k, L, replace=False)] = 0
        rf[rng.choice(m, L, replace=False)] = 1
    elif name == "tail_1pct":
        L = k // 100
        of[k - L:] = 0
        rf[:L] = 1
    else:  # every original lost
        of[:] = 0
        rf[:k] = 1
    return of, rf


out = []
for name, k in (("scattered_1pct", 32768), ("random_50pct", 32768), ("tail_1pct", 32768), ("all_30000", 30000)):
    m = k
    orig = generate_original(k, S, 1)
    d_o, d_r = DeviceArray.from_numpy(eng, orig), DeviceArray(eng, m * S)
    rs16.encode_device(k, m, S, d_o.ptr, d_r.ptr, engine=eng)
    of, rf = pattern(name, k, m, np.random.default_rng(11))
    held = orig.copy()
    held[of == 0] = 0
    d_h = DeviceArray.from_numpy(eng, held)
    d_of, d_rf = DeviceArray.from_numpy(eng, of), DeviceArray.from_numpy(eng, rf)
    nof, nrf = int(of.sum()), int(rf.sum())

    def dec():
        rs16.decode_device(k, m, S, d_h.ptr, d_of.ptr, d_r.ptr, d_rf.ptr, nof, nrf, engine=eng)

    for _ in range(5):
        dec()
    eng.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        dec()
    eng.synchronize()
    us = (time.perf_counter() - t) / reps * 1e6
    ok = bool(np.array_equal(d_h.download(shape=(k, S)), orig))
    eng.set_profiling(True)
    eng.profile_reset()
    for _ in range(3):
        dec()
    eng.synchronize()
    prof = {p: round(ms * 1e3 / n, 1) for p, (ms, n) in eng.profile().items()}
    eng.set_profiling(False)
    print(f"{name:16s} {us:7.1f} us ok={ok} {prof}", flush=True)
    assert ok
