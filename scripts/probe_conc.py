"""Concurrency probe: does one 32768:32768 x 1 KiB stripe
gain from running as two column halves on two engines (two streams) with NO
cross-stream events inside the timed loop?  Variants, all encode + 100 %-loss
decode per stripe, GiB/s over (k + m) x S x 2 bytes per step:

  one      1 engine,  1 x 1024 B stripe                 (the metric today)
  seq2     1 engine,  2 x  512 B stripes back to back   (narrow-row cost alone)
  half2    2 engines, 2 x  512 B stripes, one per stream (column halves)
  quart4   4 engines, 4 x  256 B stripes
  full2    2 engines, 2 x 1024 B stripes (serving mode; 2 stripes per step)
  encdec   2 engines: engine A encodes stripe i while engine B decodes
           stripe i - 1's recovery (a producer / consumer pipeline)

Each is timed over `--steps` steps (default 200, ~40 ms: sustained, not a
burst) after a warm-up; the first-20 / last-20 medians of per-step host
timestamps are not meaningful with async launches, so only totals are printed.
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import numpy as np  # noqa: E402

import rs16  # noqa: E402
from rs16.device import DeviceArray  # noqa: E402

k = m = 32768
GIB = 2.0 ** 30


class Stripe:
    def __init__(self, eng, sb, seed):
        o = np.random.default_rng(seed).integers(0, 256, (k, sb), dtype=np.uint8)
        self.eng, self.sb, self.o = eng, sb, o
        self.d_o, self.d_r, self.d_x = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * sb), DeviceArray(eng, k * sb)
        self.f0 = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
        self.f1 = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
        self.enc()
        self.dec()
        eng.synchronize()
        assert np.array_equal(self.d_x.download(shape=(k, sb)), o)

    def enc(self):
        rs16.encode_device(k, m, self.sb, self.d_o.ptr, self.d_r.ptr, engine=self.eng)

    def dec(self):
        rs16.decode_device(k, m, self.sb, self.d_x.ptr, self.f0.ptr, self.d_r.ptr, self.f1.ptr, 0, m, engine=self.eng)


def timed(engs, body, steps, bytes_per_step):
    for _ in range(5):
        body()
    for g in engs:
        g.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        body()
    for g in engs:
        g.synchronize()
    dt = time.perf_counter() - t
    return round(bytes_per_step * steps / dt / GIB, 1), round(dt / steps * 1e6, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--offsets", default="", help="comma list of MiB: half2 with stream B delayed by an xor of that size")
    a = ap.parse_args()
    S = 1024
    step_bytes = 2 * (k + m) * S
    engs = [rs16.Engine(0) for _ in range(4)]
    one = Stripe(engs[0], S, 1)
    h = [Stripe(engs[i], S // 2, 2 + i) for i in range(2)]
    q = [Stripe(engs[i], S // 4, 4 + i) for i in range(4)]
    f2 = Stripe(engs[1], S, 9)
    hs = [Stripe(engs[0], S // 2, 12 + i) for i in range(2)]

    def b_one():
        one.enc(); one.dec()

    def b_seq2():
        for s in hs:
            s.enc(); s.dec()

    def b_half2():
        for s in h:
            s.enc()
        for s in h:
            s.dec()

    def b_half2i():  # per-stripe enc+dec interleaved submission
        h[0].enc(); h[1].enc(); h[0].dec(); h[1].dec()

    def b_quart4():
        for s in q:
            s.enc()
        for s in q:
            s.dec()

    def b_full2():
        one.enc(); f2.enc(); one.dec(); f2.dec()

    def b_encdec():  # engine 0 encodes `one`, engine 1 decodes f2 (its recovery is ready)
        one.enc(); f2.dec()

    out = {}
    if a.offsets:
        xb = DeviceArray(engs[1], 64 << 20)
        yb = DeviceArray(engs[1], 64 << 20)

        def b_half2_off():
            for s in h:
                s.enc()
            for s in h:
                s.dec()

        for mib in [int(x) for x in a.offsets.split(",")]:
            for rep in range(a.reps):
                for g in engs[:2]:
                    g.synchronize()
                t = time.perf_counter()
                if mib:
                    engs[1].xor(xb.ptr, yb.ptr, mib << 20)
                for _ in range(a.steps):
                    b_half2_off()
                for g in engs[:2]:
                    g.synchronize()
                dt = time.perf_counter() - t
                print("half2 offset", mib, "MiB", rep, round(step_bytes * a.steps / dt / GIB, 1), "GiB/s",
                      round(dt / a.steps * 1e6, 1), "us/step", flush=True)
        return
    for rep in range(a.reps):
        for name, body, eg, nb in (("one", b_one, engs[:1], step_bytes),
                                   ("seq2", b_seq2, engs[:1], step_bytes),
                                   ("half2", b_half2, engs[:2], step_bytes),
                                   ("half2i", b_half2i, engs[:2], step_bytes),
                                   ("quart4", b_quart4, engs, step_bytes),
                                   ("full2", b_full2, engs[:2], 2 * step_bytes),
                                   ("encdec", b_encdec, engs[:2], step_bytes)):
            gib, us = timed(eg, body, a.steps, nb)
            out.setdefault(name, []).append({"gib_s": gib, "us_per_step": us})
            print(name, rep, gib, "GiB/s", us, "us/step", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
