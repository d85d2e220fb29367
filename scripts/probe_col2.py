"""Column codec forms at 1000:1000 x 1 KiB (configs[1] / [2]) and other
2^8..2^10-row transforms: kernel hipEvent time and host-timed call rate of the
radix-2 kernel (default) and the 4-rows-per-thread kernel
(RS16_DIAG_COL_RADIX4), encode and 100 %-loss decode, results checked."""
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


def run(eng, k, m, S, flag):
    o = generate_original(k, S, 0)
    # decode: the first min(k, m) originals lost, recovery 0.. given (100 %
    # original loss when k <= m; benches/benchmarks.rs:82-87)
    lost = min(k, m)
    held = o.copy()
    held[:lost] = 0
    a, r, x = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S), DeviceArray.from_numpy(eng, held)
    fo = np.ones(k, np.uint8)
    fo[:lost] = 0
    fr = np.zeros(m, np.uint8)
    fr[:lost] = 1
    f0, f1 = DeviceArray.from_numpy(eng, fo), DeviceArray.from_numpy(eng, fr)
    old = rs16.set_diagnostics(flag)
    try:
        enc = lambda: rs16.encode_device(k, m, S, a.ptr, r.ptr, engine=eng)
        dec = lambda: rs16.decode_device(k, m, S, x.ptr, f0.ptr, r.ptr, f1.ptr, k - lost, lost, engine=eng)
        enc(); dec(); eng.synchronize()
        ok = bool(np.array_equal(x.download(shape=(k, S)), o))
        res = {"exact": ok}
        for name, fn in (("encode", enc), ("decode", dec)):
            for _ in range(300):
                fn()
            eng.synchronize()
            n = 2000
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            eng.synchronize()
            host = (time.perf_counter() - t0) / n * 1e6
            eng.profile_reset()
            eng.set_profiling(True)
            for _ in range(200):
                fn()
            eng.set_profiling(False)
            prof = {p: round(ms / c * 1e3, 2) for p, (ms, c) in eng.profile().items() if c}
            res[name] = {"host_us": round(host, 2), "kernel_us": prof}
        return res
    finally:
        rs16.set_diagnostics(old)


def run_1pct(eng, k, m, S, flag):
    """The reference bench's 1 % loss (originals 0..k-L lost? no: the last L
    originals lost, recovery 0..L given; benches/benchmarks.rs:84-87)."""
    L = max(1, min(k, m) // 100)
    o = generate_original(k, S, 1)
    a, r = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S)
    held = o.copy()
    held[k - L:] = 0
    x = DeviceArray.from_numpy(eng, held)
    fo = np.ones(k, np.uint8)
    fo[k - L:] = 0
    fr = np.zeros(m, np.uint8)
    fr[:L] = 1
    f0, f1 = DeviceArray.from_numpy(eng, fo), DeviceArray.from_numpy(eng, fr)
    old = rs16.set_diagnostics(flag)
    try:
        rs16.encode_device(k, m, S, a.ptr, r.ptr, engine=eng)
        dec = lambda: rs16.decode_device(k, m, S, x.ptr, f0.ptr, r.ptr, f1.ptr, k - L, L, engine=eng)
        dec(); eng.synchronize()
        ok = bool(np.array_equal(x.download(shape=(k, S)), o))
        for _ in range(300):
            dec()
        eng.synchronize()
        t0 = time.perf_counter()
        for _ in range(2000):
            dec()
        eng.synchronize()
        return {"exact": ok, "decode_1pct_host_us": round((time.perf_counter() - t0) / 2000 * 1e6, 2)}
    finally:
        rs16.set_diagnostics(old)


def main():
    eng = rs16.Engine(0)
    out = {}
    for k, m in ((1000, 1000), (512, 512), (200, 256), (100, 100), (1000, 100), (100, 1000)):
        if len(sys.argv) > 1 and sys.argv[1] == "gen":
            continue
        forms = (("radix2", 0), ("radix4", rs16.DIAG_COL_RADIX4)) if k == m else (("column", 0), ("passes", rs16.DIAG_NO_COLUMN))
        for name, flag in forms:
            out[f"{k}:{m} {name}"] = run(eng, k, m, 1024, flag)
            print(f"{k}:{m} {name}", json.dumps(out[f"{k}:{m} {name}"]), flush=True)
    for k, m in ((1000, 1000), (1000, 100), (100, 1000), (100, 100), (300, 300)):
        for name, flag in (("radix2", 0), ("radix4", rs16.DIAG_COL_RADIX4)):
            print(f"{k}:{m} 1% {name}", json.dumps(run_1pct(eng, k, m, 1024, flag)), flush=True)


if __name__ == "__main__":
    main()
