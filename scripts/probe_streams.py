"""Concurrency probe: one 32768:32768 stripe of S-byte shards on one stream vs
NS stripes of S/NS-byte shards (the same bytes) on NS engines (streams)."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import numpy as np
import rs16
from rs16.device import DeviceArray

k = m = 32768
S = 1024
GIB = 2.0 ** 30


def setup(eng, sb, seed):
    o = np.random.default_rng(seed).integers(0, 256, (k, sb), dtype=np.uint8)
    d_o, d_r, d_x = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * sb), DeviceArray(eng, k * sb)
    f0 = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    f1 = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    enc = lambda: rs16.encode_device(k, m, sb, d_o.ptr, d_r.ptr, engine=eng)
    dec = lambda: rs16.decode_device(k, m, sb, d_x.ptr, f0.ptr, d_r.ptr, f1.ptr, 0, m, engine=eng)
    enc(); dec(); eng.synchronize()
    assert np.array_equal(d_x.download(shape=(k, sb)), o)
    return enc, dec, (d_o, d_r, d_x, f0, f1)


def run(engs, jobs, steps=30):
    for _ in range(3):
        for e, d in jobs: e(); d()
    for g in engs: g.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        for e, _d in jobs: e()
        for _e, d in jobs: d()
    for g in engs: g.synchronize()
    return 2 * (k + m) * S * steps / (time.perf_counter() - t) / GIB


e0 = rs16.Engine(0)
one = setup(e0, S, 1)
print("1 stream x 1024 B:", round(run([e0], [one[:2]]), 1), flush=True)
for ns in (2, 4):
    engs = [rs16.Engine(0) for _ in range(ns)]
    jobs = [setup(g, S // ns, 2 + i) for i, g in enumerate(engs)]
    print(f"{ns} streams x {S // ns} B:", round(run(engs, [j[:2] for j in jobs]), 1), flush=True)
    print(f"1 stream, {ns} x {S // ns} B sequential:", round(run([engs[0]], [j[:2] for j in jobs[:1]] * 1) / 1, 1),
          "(one slice only, x", ns, "bytes accounted)", flush=True)
