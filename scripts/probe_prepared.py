"""The bench step (32768:32768 x 1 KiB encode + 100 %-loss decode) with the
decode split (rs16_decode_prepare on a side stream before the encode,
rs16_decode_device_prepared after it) against the serial step; eval_poly in
its one-kernel form (141 VGPRs: cannot share a CU with the T = 7 passes) and
in the two-kernel form (24 / 28 VGPRs), and several side streams (a side
stream on the engine stream's hardware queue cannot overlap)."""
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


def main():
    eng = rs16.Engine(0)
    o = generate_original(k, S, 0)
    d_o, d_r, d_x = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S), DeviceArray(eng, k * S)
    fo = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    fr = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    sides = [eng.create_stream() for _ in range(4)]

    def serial():
        rs16.encode_device(k, m, S, d_o.ptr, d_r.ptr, engine=eng)
        rs16.decode_device(k, m, S, d_x.ptr, fo.ptr, d_r.ptr, fr.ptr, 0, m, engine=eng)

    def split(side):
        def f():
            rs16.decode_prepare(k, m, S, fo.ptr, fr.ptr, 0, m, stream=side, engine=eng)
            rs16.encode_device(k, m, S, d_o.ptr, d_r.ptr, engine=eng)
            rs16.decode_device_prepared(k, m, S, d_x.ptr, d_r.ptr, engine=eng)
        return f

    def timed(body, steps=200):
        for _ in range(20):
            body()
        eng.synchronize()
        for s in sides:
            eng.synchronize(s)
        t = time.perf_counter()
        for _ in range(steps):
            body()
        eng.synchronize()
        dt = time.perf_counter() - t
        return round(STEP * steps / dt / GIB, 1)

    out = {}
    for rep in range(2):
        for diag, name in ((0, "fused"), (rs16.DIAG_EVAL_TWO_KERNEL, "two_kernel")):
            eng.set_diagnostics(diag)
            out.setdefault(f"serial_{name}", []).append(timed(serial))
            for i, s in enumerate(sides):
                d_x.upload(np.zeros_like(o))
                split(s)()
                eng.synchronize()
                assert np.array_equal(d_x.download(shape=(k, S)), o)
                out.setdefault(f"split_{name}_side{i}", []).append(timed(split(s)))
            print(rep, name, {kk: v[-1] for kk, v in out.items() if name in kk}, flush=True)
    eng.set_diagnostics(0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
