"""Column codec vs pass codec at n <= 2048 (run on the GPU box):
wall time per call (perf_counter over N synchronized calls, as bench.py) and
per-kernel hipEvent times (engine profiling), for 1000:1000 at several shard
widths and as batched stripes, with the column codec on and off
(rs16.DIAG_NO_COLUMN).  Prints one JSON line per case."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "reed-solomon-16_amd"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import rs16  # noqa: E402
from rs16.device import DeviceArray  # noqa: E402
from rs16.util import generate_original  # noqa: E402


def timed(eng, fn, n):
    fn()
    eng.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    eng.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def case(eng, k, m, S, nst, diag, n=200):
    rs16.set_diagnostics(diag)
    o = generate_original(k, S, 5)
    so, sr = k * S, m * S
    a = DeviceArray.from_numpy(eng, np.tile(o.reshape(-1), nst))
    r = DeviceArray(eng, m * S * nst)
    x = DeviceArray(eng, k * S * nst)
    f0 = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    f1 = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    if nst == 1:
        enc = lambda: rs16.encode_device(k, m, S, a.ptr, r.ptr, engine=eng)
        dec = lambda: rs16.decode_device(k, m, S, x.ptr, f0.ptr, r.ptr, f1.ptr, 0, m, engine=eng)
    else:
        enc = lambda: rs16.encode_device_batch(k, m, S, nst, a.ptr, so, r.ptr, sr, engine=eng)
        dec = lambda: rs16.decode_device_batch(k, m, S, nst, x.ptr, so, f0.ptr, r.ptr, sr, f1.ptr, 0, m, engine=eng)
    enc()
    dec()
    eng.synchronize()
    ok = np.array_equal(x.download(shape=(nst * k, S))[:k], o)
    n = max(10, min(n, int(2e9 / ((k + m) * S * nst))))
    te = timed(eng, enc, n)
    td = timed(eng, dec, n)
    eng.set_profiling(True)
    eng.profile_reset()
    for _ in range(20):
        enc()
        dec()
    eng.synchronize()
    prof = {kk: round(ms / cnt * 1e3, 2) for kk, (ms, cnt) in eng.profile().items()}
    eng.set_profiling(False)
    rs16.set_diagnostics(0)
    gib = (k + m) * S * nst / 2**30
    print(json.dumps({"k": k, "m": m, "S": S, "stripes": nst, "column": diag == rs16.DIAG_FORCE_COLUMN, "restored": ok,
                      "encode_us": round(te, 2), "decode_us": round(td, 2),
                      "encode_gib_s": round(gib / te * 1e6, 1), "decode_gib_s": round(gib / td * 1e6, 1),
                      "kernels_us": prof}), flush=True)


def main():
    eng = rs16.default_engine()
    for (k, m, S, nst) in [(1000, 1000, 1024, 1), (512, 512, 1024, 1), (1000, 1000, 2048, 1),
                           (1000, 1000, 4096, 1), (1000, 1000, 1024, 2), (1000, 1000, 1024, 4),
                           (1000, 1000, 16384, 1), (1000, 1000, 1024, 32)]:
        for diag in (rs16.DIAG_FORCE_COLUMN, rs16.DIAG_NO_COLUMN):
            case(eng, k, m, S, nst, diag)


if __name__ == "__main__":
    main()
