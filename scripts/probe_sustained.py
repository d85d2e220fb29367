"""Sustained-rate probe: the bench step (32768:32768 x
1 KiB encode + 100 %-loss decode) run back to back for `--seconds` of GPU
time with a hipEvent pair around every step on the engine stream, after an
idle pause, to see how the per-step time evolves from a cold (idle-clocked)
GPU: first / last medians, and the median of each 10 % slice of the run."""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import numpy as np  # noqa: E402

import rs16  # noqa: E402
from rs16.device import DeviceArray  # noqa: E402
from rs16.util import generate_original  # noqa: E402

from rs16._lib import hip_runtime  # noqa: E402
hip = hip_runtime()
hip.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
hip.hipEventSynchronize.argtypes = [C.c_void_p]
hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--idle", type=float, default=2.0, help="idle pause before the run")
    a = ap.parse_args()
    k = m = 32768
    S = 1024
    eng = rs16.Engine(0)
    o = generate_original(k, S, 0)
    d_o, d_r, d_x = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S), DeviceArray(eng, k * S)
    f0 = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    f1 = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))

    def step():
        rs16.encode_device(k, m, S, d_o.ptr, d_r.ptr, engine=eng)
        rs16.decode_device(k, m, S, d_x.ptr, f0.ptr, d_r.ptr, f1.ptr, 0, m, engine=eng)

    step()
    eng.synchronize()
    assert np.array_equal(d_x.download(shape=(k, S)), o)
    n = int(a.seconds / 170e-6)
    evs = [C.c_void_p() for _ in range(n + 1)]
    for e in evs:
        assert hip.hipEventCreate(C.byref(e)) == 0
    s = C.c_void_p(eng.stream)
    time.sleep(a.idle)
    hip.hipEventRecord(evs[0], s)
    for i in range(n):
        step()
        hip.hipEventRecord(evs[i + 1], s)
    hip.hipEventSynchronize(evs[n])
    t = np.empty(n)
    f = C.c_float()
    for i in range(n):
        hip.hipEventElapsedTime(C.byref(f), evs[i], evs[i + 1])
        t[i] = f.value * 1e3
    step_bytes = 2 * (k + m) * S
    dec = [round(float(np.median(x)), 1) for x in np.array_split(t, 10)]
    out = {"steps": n, "gpu_s": round(float(t.sum()) / 1e6, 3),
           "gib_s_all": round(step_bytes * n / (t.sum() * 1e-6) / 2**30, 1),
           "first20_median_us": round(float(np.median(t[:20])), 1),
           "last20_median_us": round(float(np.median(t[-20:])), 1),
           "first5_us": [round(float(x), 1) for x in t[:5]],
           "steps_1_25_us": [round(float(x), 1) for x in t[:25]],
           "decile_median_us": dec}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
