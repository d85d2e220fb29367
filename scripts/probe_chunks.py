"""Multi-chunk encodes of 2^8..2^10-row chunks: the radix-2 column codec
(default) against the pass codec (RS16_DIAG_NO_COLUMN), host-timed call rate
over back-to-back calls plus hipEvent kernel time, recovery checked equal."""
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

CASES = ((10000, 1000), (1000, 10000), (3000, 1000), (1000, 3000), (2000, 300), (300, 2000),
         (30000, 1000), (1000, 30000), (60000, 1000), (1000, 60000), (8000, 300), (300, 8000))
if len(sys.argv) > 1 and sys.argv[1] == "edge":
    CASES = ((4000, 1000), (1000, 4000), (6000, 1000), (1000, 6000), (8000, 1000), (1000, 8000),
             (6000, 300), (300, 6000), (6000, 200), (200, 6000), (8000, 200), (200, 8000))


def run(eng, k, m, S, flag):
    o = generate_original(k, S, 3)
    a, r = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S)
    old = rs16.set_diagnostics(flag)
    try:
        enc = lambda: rs16.encode_device(k, m, S, a.ptr, r.ptr, engine=eng)
        enc()
        eng.synchronize()
        rec = r.download(shape=(m, S))
        for _ in range(100):
            enc()
        eng.synchronize()
        n = 1000
        t0 = time.perf_counter()
        for _ in range(n):
            enc()
        eng.synchronize()
        host = (time.perf_counter() - t0) / n * 1e6
        eng.profile_reset()
        eng.set_profiling(True)
        for _ in range(100):
            enc()
        eng.set_profiling(False)
        prof = {p: round(ms / c * 1e3, 2) for p, (ms, c) in eng.profile().items() if c}
        return rec, {"host_us": round(host, 2), "kernel_us": prof}
    finally:
        rs16.set_diagnostics(old)


def main():
    eng = rs16.Engine(0)
    for k, m in CASES:
        rc, col = run(eng, k, m, 1024, 0)
        rp, pas = run(eng, k, m, 1024, rs16.DIAG_NO_COLUMN)
        print(f"{k}:{m}", json.dumps({"column": col, "passes": pas, "equal": bool(np.array_equal(rc, rp))}), flush=True)


if __name__ == "__main__":
    main()
