"""Time the 1 %-loss decode (32768:32768 x 1 KiB) per call and in a loop."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import numpy as np
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

k = m = 32768; S = 1024
eng = rs16.Engine(0)
orig = generate_original(k, S, 0)
d_o = DeviceArray.from_numpy(eng, orig); d_r = DeviceArray(eng, m * S)
rs16.encode_device(k, m, S, d_o.ptr, d_r.ptr, engine=eng)
for L1 in (327, 32768):
    of = np.ones(k, np.uint8); of[k - L1:] = 0
    rf = np.zeros(m, np.uint8); rf[:L1] = 1
    o1 = orig.copy(); o1[k - L1:] = 0
    a, b, x = DeviceArray.from_numpy(eng, of), DeviceArray.from_numpy(eng, rf), DeviceArray.from_numpy(eng, o1)
    f = lambda: rs16.decode_device(k, m, S, x.ptr, a.ptr, d_r.ptr, b.ptr, k - L1, L1, engine=eng)
    f(); eng.synchronize()
    per = []
    for _ in range(5):
        t = time.perf_counter(); f(); t1 = time.perf_counter(); eng.synchronize(); per.append((t1 - t, time.perf_counter() - t))
    t = time.perf_counter()
    for _ in range(20): f()
    eng.synchronize()
    print(L1, "per-call (launch, total) us:", [(round(p * 1e6), round(q * 1e6)) for p, q in per],
          "loop us/call:", round((time.perf_counter() - t) / 20 * 1e6), flush=True)

# per-pass hipEvent times of the 1 %-loss (general) decode
of = np.ones(k, np.uint8); of[k - 327:] = 0
rf = np.zeros(m, np.uint8); rf[:327] = 1
o1 = orig.copy(); o1[k - 327:] = 0
a, b, x = DeviceArray.from_numpy(eng, of), DeviceArray.from_numpy(eng, rf), DeviceArray.from_numpy(eng, o1)
eng.set_profiling(True)
eng.profile_reset()
for _ in range(10):
    rs16.decode_device(k, m, S, x.ptr, a.ptr, d_r.ptr, b.ptr, k - 327, 327, engine=eng)
eng.synchronize()
prof = eng.profile()
eng.set_profiling(False)
print("1 % decode per pass (us):", {n: round(ms * 1e3 / max(c, 1), 2) for n, (ms, c) in prof.items() if c})

# the last pass in both forms (identical results)
for name, flag in (("default", 0), ("fd_lds", rs16.DIAG_FD_LDS), ("items", rs16.DIAG_NO_TILE_LAST)):
    old = rs16.set_diagnostics(flag)
    x.upload(o1)
    eng.set_profiling(True)
    eng.profile_reset()
    for _ in range(10):
        rs16.decode_device(k, m, S, x.ptr, a.ptr, d_r.ptr, b.ptr, k - 327, 327, engine=eng)
    eng.synchronize()
    prof = eng.profile()
    eng.set_profiling(False)
    ok = np.array_equal(x.download(shape=(k, S)), orig)
    for _ in range(30):  # back to full clocks after the download
        rs16.decode_device(k, m, S, x.ptr, a.ptr, d_r.ptr, b.ptr, k - 327, 327, engine=eng)
    eng.synchronize()
    t = time.perf_counter()
    for _ in range(50):
        rs16.decode_device(k, m, S, x.ptr, a.ptr, d_r.ptr, b.ptr, k - 327, 327, engine=eng)
    eng.synchronize()
    us = (time.perf_counter() - t) / 50 * 1e6
    rs16.set_diagnostics(old)
    print(name, "exact:", ok, "loop us/call:", round(us, 1), "GiB/s:", round(2 * k * S / us / 1e-6 / 2**30, 1),
          {n: round(ms * 1e3 / max(c, 1), 2) for n, (ms, c) in prof.items() if c}, flush=True)
