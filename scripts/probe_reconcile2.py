"""VERDICT r4 item 1, second probe: bench.py's own two-stripe extra gives
~752 GiB/s even right after its timed loop, scripts/probe_reconcile.py ~900.
This replays bench.py's sequence on one engine pair and measures the two
stripes (and encode-while-decode) after each stage:
  S0  engines and buffers made, correctness step done (nothing else)
  S1  after the bench's event-profiled loop on engine A
      (rs16_engine_set_profiling on, 40 + 20 steps, off)
  S2  after warm-up + timed loop + encode-only / decode-only loops
  S3  a fresh engine pair created now (same process)
"""
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

k = m = 32768
S = 1024
GIB = 2.0 ** 30
STEP = 2 * (k + m) * S


class Stripe:
    def __init__(self, eng, seed):
        o = generate_original(k, S, seed)
        self.eng = eng
        self.d_o, self.d_r, self.d_x = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S), DeviceArray(eng, k * S)
        self.f0 = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
        self.f1 = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
        self.enc()
        self.dec()
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
    return round(nbytes * steps / dt / GIB, 1)


def measure(tag, A, B, sa, sb, out):
    r = {"one": timed([A], lambda: (sa.enc(), sa.dec()), 100, STEP),
         "two": timed([A, B], lambda: (sa.enc(), sb.enc(), sa.dec(), sb.dec()), 100, 2 * STEP),
         "enc_while_dec": timed([A, B], lambda: (sa.enc(), sb.dec()), 100, STEP)}
    out[tag] = r
    print(tag, r, flush=True)


def main():
    out = {}
    A, B = rs16.Engine(0), rs16.Engine(0)
    sa, sb = Stripe(A, 0), Stripe(B, 1)
    measure("S0_fresh", A, B, sa, sb, out)
    A.set_profiling(True)
    for _ in range(40):
        sa.enc(); sa.dec()
    A.synchronize()
    A.profile()
    A.profile_reset()
    for _ in range(20):
        sa.enc(); sa.dec()
    A.synchronize()
    A.set_profiling(False)
    measure("S1_after_profiled_loop", A, B, sa, sb, out)
    for _ in range(25):
        sa.enc(); sa.dec()
    for _ in range(20):
        sa.enc()
    for _ in range(20):
        sa.dec()
    A.synchronize()
    measure("S2_after_timed_loops", A, B, sa, sb, out)
    C, D = rs16.Engine(0), rs16.Engine(0)
    sc, sd = Stripe(C, 2), Stripe(D, 3)
    measure("S3_fresh_pair_now", C, D, sc, sd, out)
    measure("S3b_A_with_fresh", A, D, sa, sd, out)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
