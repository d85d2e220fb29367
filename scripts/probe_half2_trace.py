"""Kernel trace of two column halves (512 B) of a 32768:32768 stripe on two
engines / streams, stream B started 8 MiB of XOR later (see probe_conc.py):
run under rocprofv3 --kernel-trace to see how the two streams' pass kernels
overlap in time."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
sys.path.insert(0, str(ROOT / "scripts"))
from probe_conc import Stripe, k, m  # noqa: E402

import rs16  # noqa: E402
from rs16.device import DeviceArray  # noqa: E402

engs = [rs16.Engine(0) for _ in range(2)]
h = [Stripe(engs[i], 512, 2 + i) for i in range(2)]
xb, yb = DeviceArray(engs[1], 64 << 20), DeviceArray(engs[1], 64 << 20)
for g in engs:
    g.synchronize()
engs[1].xor(xb.ptr, yb.ptr, 8 << 20)
for _ in range(30):
    for s in h:
        s.enc()
    for s in h:
        s.dec()
for g in engs:
    g.synchronize()
print("done")
