"""Where the time of a 1000:1000 x 1 KiB call goes: host
enqueue time per call (the Python + C ABI + HIP launch path, no sync), the
host-timed rate with a sync at the end (what bench.py's extra reports), the
kernels' own hipEvent time, and a C++ caller's rate (rs16_bench_small, no
Python in the loop)."""
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import numpy as np  # noqa: E402

import rs16  # noqa: E402
from rs16.device import DeviceArray  # noqa: E402
from rs16.util import generate_original  # noqa: E402


def main():
    k = m = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    S = 1024
    eng = rs16.Engine(0)
    o = generate_original(k, S, 0)
    a, r, x = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S), DeviceArray(eng, k * S)
    f0 = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    f1 = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    enc = lambda: rs16.encode_device(k, m, S, a.ptr, r.ptr, engine=eng)
    dec = lambda: rs16.decode_device(k, m, S, x.ptr, f0.ptr, r.ptr, f1.ptr, 0, m, engine=eng)
    enc(); dec(); eng.synchronize()
    assert np.array_equal(x.download(shape=(k, S)), o)
    out = {}
    for name, fn in (("encode", enc), ("decode", dec)):
        for _ in range(200):
            fn()
        eng.synchronize()
        n = 2000
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        t1 = time.perf_counter()
        eng.synchronize()
        t2 = time.perf_counter()
        eng.profile_reset()
        eng.set_profiling(True)
        for _ in range(200):
            fn()
        eng.set_profiling(False)
        prof = {p: round(ms / c * 1e3, 2) for p, (ms, c) in eng.profile().items()}
        out[name] = {"enqueue_us_per_call": round((t1 - t0) / n * 1e6, 2),
                     "host_timed_us_per_call": round((t2 - t0) / n * 1e6, 2), "kernel_event_us": prof}
    tool = ROOT / "reed-solomon-16_amd" / "build" / "rs16_bench_small"
    if tool.exists():
        res = subprocess.run([str(tool), str(k), str(m), str(S)], capture_output=True, text=True, timeout=120)
        out["cxx_caller"] = json.loads(res.stdout) if res.returncode == 0 else res.stderr[-500:]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
