"""Two stripes in flight on two engines (serving mode):
does a second engine created with RS16_ENGINE_OWN_QUEUE (its stream on a
CU-masked, i.e. dedicated, hardware queue) overlap with the first engine
deterministically, where a default second engine may share the first one's
queue?  Steady state (warm clocks), 200-step loops, alternating pairs, 3 reps.
Every decode is checked once.  Usage: probe_own_queue.py [steps]"""
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
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200


class Stripe:
    def __init__(self, eng, seed):
        self.o = generate_original(k, S, seed)
        self.eng = eng
        self.d_o, self.d_r, self.d_x = DeviceArray.from_numpy(eng, self.o), DeviceArray(eng, m * S), DeviceArray(eng, k * S)
        self.f0 = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
        self.f1 = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))

    def enc(self):
        rs16.encode_device(k, m, S, self.d_o.ptr, self.d_r.ptr, engine=self.eng)

    def dec(self):
        rs16.decode_device(k, m, S, self.d_x.ptr, self.f0.ptr, self.d_r.ptr, self.f1.ptr, 0, m, engine=self.eng)

    def check(self):
        self.enc()
        self.dec()
        self.eng.synchronize()
        assert np.array_equal(self.d_x.download(shape=(k, S)), self.o)


def timed(engs, body):
    for _ in range(30):
        body()
    for e in engs:
        e.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        body()
    for e in engs:
        e.synchronize()
    return time.perf_counter() - t


A = rs16.Engine(0)
B = rs16.Engine(0, rs16.Engine.OWN_QUEUE)
C = rs16.Engine(0)
D = rs16.Engine(0, rs16.Engine.OWN_QUEUE)
sa, sb, sc, sd = Stripe(A, 1), Stripe(B, 2), Stripe(C, 3), Stripe(D, 4)
for s in (sa, sb, sc, sd):
    s.check()


def one(s):
    def f():
        s.enc()
        s.dec()
    return f


def two(x, y):
    def f():
        x.enc()
        y.enc()
        x.dec()
        y.dec()
    return f


def ewd(x, y):  # x encodes while y decodes (y's recovery already encoded)
    def f():
        x.enc()
        y.dec()
    return f


for rep in range(3):
    row = {}
    t1 = timed([A], one(sa))
    row["one_A"] = STEP * steps / t1 / GIB
    row["one_B_ownq"] = STEP * steps / timed([B], one(sb)) / GIB
    for name, x, y in (("A+B_ownq", sa, sb), ("A+C_default", sa, sc), ("B+D_both_ownq", sb, sd),
                       ("C+D", sc, sd)):
        t = timed([x.eng, y.eng], two(x, y))
        row[name] = 2 * STEP * steps / t / GIB
        row[name + "_ratio"] = t / t1
    row["enc_A_while_dec_B_ownq"] = STEP * steps / timed([A, B], ewd(sa, sb)) / GIB
    row["enc_A_while_dec_C_default"] = STEP * steps / timed([A, C], ewd(sa, sc)) / GIB
    print(f"rep {rep}: " + " ".join(f"{k2} {v:.3f}" if k2.endswith("ratio") else f"{k2} {v:.1f}"
                                     for k2, v in row.items()), flush=True)
for s in (sa, sb, sc, sd):
    s.check()
print("restored True")
