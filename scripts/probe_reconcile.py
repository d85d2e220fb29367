"""why does scripts/probe_conc.py's `full2` (two independent
32768:32768 x 1 KiB stripes on two engines) reach ~900 GiB/s while bench.py's
`two_stripes_two_streams` -- the same call sequence -- reports ~756?

The two differ in (a) the number of timed steps (200 vs 20), (b) when the
second engine is created (before anything else vs after the configs4_rccl
extra, which creates and frees an RCCL communicator, and after other streams
exist) and (c) the data (random vs ChaCha8).  Each variant below changes one
of them; all run encode + 100 %-loss decode per stripe, GiB/s over
2 (k + m) S bytes per stripe.
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
S = 1024
GIB = 2.0 ** 30
STEP = 2 * (k + m) * S


class Stripe:
    def __init__(self, eng, seed):
        o = np.random.default_rng(seed).integers(0, 256, (k, S), dtype=np.uint8)
        self.eng, self.o = eng, o
        self.d_o, self.d_r, self.d_x = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S), DeviceArray(eng, k * S)
        self.f0 = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
        self.f1 = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
        self.enc()
        self.dec()
        eng.synchronize()
        assert np.array_equal(self.d_x.download(shape=(k, S)), o)

    def enc(self):
        rs16.encode_device(k, m, S, self.d_o.ptr, self.d_r.ptr, engine=self.eng)

    def dec(self):
        rs16.decode_device(k, m, S, self.d_x.ptr, self.f0.ptr, self.d_r.ptr, self.f1.ptr, 0, m, engine=self.eng)


def timed(engs, body, steps, nbytes, warmup=5):
    for _ in range(warmup):
        body()
    for g in engs:
        g.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        body()
    for g in engs:
        g.synchronize()
    dt = time.perf_counter() - t
    return {"gib_s": round(nbytes * steps / dt / GIB, 1), "us_per_step": round(dt / steps * 1e6, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    out = {}

    def rec(name, r):
        out.setdefault(name, []).append(r)
        print(name, r, flush=True)

    A, B = rs16.Engine(0), rs16.Engine(0)
    sa, sb = Stripe(A, 1), Stripe(B, 2)
    one = lambda: (sa.enc(), sa.dec())
    full2 = lambda x, y: (lambda: (x.enc(), y.enc(), x.dec(), y.dec()))
    encdec = lambda x, y: (lambda: (x.enc(), y.dec()))
    for rep in range(a.reps):
        rec("one_200", timed([A], one, 200, STEP))
        rec("one_20", timed([A], one, 20, STEP))
        rec("full2_fresh_200", timed([A, B], full2(sa, sb), 200, 2 * STEP))
        rec("full2_fresh_20", timed([A, B], full2(sa, sb), 20, 2 * STEP))
        rec("encdec_fresh_200", timed([A, B], encdec(sa, sb), 200, STEP))
    # (b1) other streams on the device before the second engine: HIP maps
    # streams onto GPU_MAX_HW_QUEUES (4) hardware queues round robin, so a
    # new engine's stream may share a hardware queue with engine A's
    extra = [A.create_stream() for _ in range(6)]
    C = rs16.Engine(0)
    sc = Stripe(C, 3)
    for rep in range(a.reps):
        rec("full2_after_6_streams_200", timed([A, C], full2(sa, sc), 200, 2 * STEP))
        rec("full2_after_6_streams_20", timed([A, C], full2(sa, sc), 20, 2 * STEP))
    for s in extra:
        A.destroy_stream(s)
    # (b2) an RCCL communicator created and closed before the second engine
    # (bench.py's configs4_rccl extra runs before two_stripes_two_streams)
    (comm,) = rs16.Comm.init_all([A])
    comm.close()
    D = rs16.Engine(0)
    sd = Stripe(D, 4)
    for rep in range(a.reps):
        rec("full2_after_comm_200", timed([A, D], full2(sa, sd), 200, 2 * STEP))
        rec("full2_after_comm_20", timed([A, D], full2(sa, sd), 20, 2 * STEP))
        rec("full2_fresh_again_20", timed([A, B], full2(sa, sb), 20, 2 * STEP))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
