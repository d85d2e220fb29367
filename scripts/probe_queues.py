"""Which stream is fast?  scripts/probe_reconcile2.py found that a pair of
engines created late in a process ran one stripe at ~733 GiB/s (vs ~783 for
the first engine) and two stripes without overlap (780 vs ~919).  HIP maps
streams onto GPU_MAX_HW_QUEUES hardware queues; this probe runs the same
stripe (engine A's buffers and scratch) on each of 8 streams in creation
order (A's own stream first), then two stripes (engines A and B) on stream
pairs, to see whether speed and overlap follow the stream / queue.
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

k = m = 32768
S = 1024
GIB = 2.0 ** 30
STEP = 2 * (k + m) * S


class Stripe:
    def __init__(self, eng, seed):
        o = np.random.default_rng(seed).integers(0, 256, (k, S), dtype=np.uint8)
        self.eng = eng
        self.d_o, self.d_r, self.d_x = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S), DeviceArray(eng, k * S)
        self.f0 = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
        self.f1 = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
        self.o = o

    def step(self, s=None):
        rs16.encode_device(k, m, S, self.d_o.ptr, self.d_r.ptr, stream=s, engine=self.eng)
        rs16.decode_device(k, m, S, self.d_x.ptr, self.f0.ptr, self.d_r.ptr, self.f1.ptr, 0, m, stream=s,
                           engine=self.eng)


def timed(sync, body, steps, nbytes, warmup=5):
    for _ in range(warmup):
        body()
    sync()
    t = time.perf_counter()
    for _ in range(steps):
        body()
    sync()
    return round(nbytes * steps / (time.perf_counter() - t) / GIB, 1)


def main():
    out = {}
    A, B = rs16.Engine(0), rs16.Engine(0)
    sa, sb = Stripe(A, 1), Stripe(B, 2)
    sa.step(), sb.step()
    A.synchronize(), B.synchronize()
    assert np.array_equal(sa.d_x.download(shape=(k, S)), sa.o)
    sA = [A.stream] + [A.create_stream() for _ in range(7)]
    sB = [B.stream] + [B.create_stream() for _ in range(7)]
    for i, s in enumerate(sA):
        sync = lambda s=s: (A.synchronize(s), A.synchronize())
        out[f"one_A_stream{i}"] = timed(sync, lambda s=s: sa.step(s), 100, STEP)
        print(f"one_A_stream{i}", out[f"one_A_stream{i}"], flush=True)
    for i, s in enumerate(sB):
        sync = lambda s=s: (B.synchronize(s), B.synchronize())
        out[f"one_B_stream{i}"] = timed(sync, lambda s=s: sb.step(s), 100, STEP)
        print(f"one_B_stream{i}", out[f"one_B_stream{i}"], flush=True)
    for i in range(8):
        for j in (0, 1, 3, 4):
            sa_, sb_ = sA[i], sB[j]

            def sync():
                A.synchronize(sa_), B.synchronize(sb_), A.synchronize(), B.synchronize()

            def two():
                rs16.encode_device(k, m, S, sa.d_o.ptr, sa.d_r.ptr, stream=sa_, engine=A)
                rs16.encode_device(k, m, S, sb.d_o.ptr, sb.d_r.ptr, stream=sb_, engine=B)
                rs16.decode_device(k, m, S, sa.d_x.ptr, sa.f0.ptr, sa.d_r.ptr, sa.f1.ptr, 0, m, stream=sa_, engine=A)
                rs16.decode_device(k, m, S, sb.d_x.ptr, sb.f0.ptr, sb.d_r.ptr, sb.f1.ptr, 0, m, stream=sb_, engine=B)

            key = f"two_A{i}_B{j}"
            out[key] = timed(sync, two, 60, 2 * STEP)
            print(key, out[key], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
