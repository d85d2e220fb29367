"""General-decode path choices at 32768:32768 x 1 KiB.

For loss patterns whose lost originals span s last-pass tiles (256 rows
each), time the decode with the last pass as tile_last_kernel (one wave per
quad column, RS16_DIAG_TILE_LAST) and as 8-wave items (RS16_DIAG_NO_TILE_LAST),
with and without the direct middle pass's launch (RS16_DIAG_NO_MID_DIRECT);
then the default path.  Every result is checked against the originals.
Usage: probe_general.py [reps]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import numpy as np  # noqa: E402

import rs16  # noqa: E402
from rs16.device import DeviceArray  # noqa: E402
from rs16.util import generate_original  # noqa: E402

k = m = 32768
S = 1024
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
eng = rs16.Engine(0)
orig = generate_original(k, S, 0)
d_o, d_r = DeviceArray.from_numpy(eng, orig), DeviceArray(eng, m * S)
rs16.encode_device(k, m, S, d_o.ptr, d_r.ptr, engine=eng)
rng = np.random.default_rng(5)


def pattern(span, nlost):
    """nlost originals lost, spread over `span` consecutive 256-row tiles at
    the end of the originals; nlost random recovery shards received."""
    of = np.ones(k, np.uint8)
    lo = k - span * 256
    of[rng.choice(np.arange(lo, k), nlost, replace=False)] = 0
    of[k - 1] = 0
    of[lo] = 0
    nl = int((of == 0).sum())
    rf = np.zeros(m, np.uint8)
    rf[rng.choice(m, nl, replace=False)] = 1
    return of, rf, nl


def run(of, rf, nl, flags):
    old = eng.set_diagnostics(flags)
    held = orig.copy()
    held[of == 0] = 0
    x = DeviceArray.from_numpy(eng, held)
    a, b = DeviceArray.from_numpy(eng, of), DeviceArray.from_numpy(eng, rf)
    f = lambda: rs16.decode_device(k, m, S, x.ptr, a.ptr, d_r.ptr, b.ptr, k - nl, nl, engine=eng)
    f()
    ok = np.array_equal(x.download(shape=(k, S)), orig)
    for _ in range(20):
        f()
    eng.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    eng.synchronize()
    us = (time.perf_counter() - t) / reps * 1e6
    eng.set_profiling(True)
    eng.profile_reset()
    for _ in range(10):
        f()
    eng.synchronize()
    prof = {n: round(ms * 1e3 / c, 1) for n, (ms, c) in eng.profile().items()}
    eng.set_profiling(False)
    eng.set_diagnostics(old)
    return round(us, 1), ok, prof


TL, NTL, NMD = 32, 64, 1024
for span, nlost in ((1, 20), (2, 327), (4, 327), (8, 327), (16, 327), (32, 327), (64, 327), (128, 327),
                    (128, 2000)):
    of, rf, nl = pattern(span, nlost)
    for name, fl in (("default", 0), ("tile_last", TL), ("items", NTL), ("tile_last,no_md", TL | NMD),
                     ("items,no_md", NTL | NMD)):
        us, ok, prof = run(of, rf, nl, fl)
        print(f"span {span:3d} lost {nl:5d} {name:16s} {us:7.1f} us ok={ok} {prof}", flush=True)
