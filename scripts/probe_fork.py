"""Cost of the device codec's column slicing: 1000:1000 and 32768:32768 x 1 KiB
encode / decode at 1, 2, 3, 4 slices, and the host time to issue one call."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import numpy as np
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

eng = rs16.Engine(0)
S = 1024
for k in (1000, 32768):
    m = k
    o = generate_original(k, S, 0)
    d_o, d_r, d_x = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S), DeviceArray(eng, k * S)
    f0 = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    f1 = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    enc = lambda: rs16.encode_device(k, m, S, d_o.ptr, d_r.ptr, engine=eng)
    dec = lambda: rs16.decode_device(k, m, S, d_x.ptr, f0.ptr, d_r.ptr, f1.ptr, 0, m, engine=eng)
    for n in (1, 2, 3, 4):
        eng.set_slices(n)
        for _ in range(5):
            enc(); dec()
        eng.synchronize()
        steps = 30
        t = time.perf_counter()
        for _ in range(steps):
            enc()
        th = time.perf_counter() - t
        eng.synchronize()
        te = time.perf_counter() - t
        t = time.perf_counter()
        for _ in range(steps):
            dec()
        eng.synchronize()
        td = time.perf_counter() - t
        print(f"{k}:{m} slices {n}: encode {te / steps * 1e6:7.1f} us (host issue {th / steps * 1e6:6.1f} us)  "
              f"decode {td / steps * 1e6:7.1f} us", flush=True)
