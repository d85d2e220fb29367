"""Every row of the reference's main benchmark table (benches/benchmarks.rs:
36-47, published in README.md:129-137) on the GPU, device-resident: encode,
and decode at 1 % and 100 % of min(k, m) originals lost with the
benchmark's pattern (originals 0..k-loss and recovery 0..loss provided,
benches/benchmarks.rs:81-105).  Throughput over (k + m) x 1024 bytes as the
reference counts it (Throughput::Bytes, :57-59).  Every decode is checked to
restore the lost originals bit for bit.  One JSON line per row (run on the
GPU box: scripts/gpu_reference_rows.sh)."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "reed-solomon-16_amd")]
import numpy as np  # noqa: E402

import rs16  # noqa: E402
from rs16.device import DeviceArray  # noqa: E402
from rs16.util import generate_original  # noqa: E402

S = 1024
# the reference's single-thread NoSimd numbers (MiB/s: encode, decode 1 %, 100 %), README.md:129-137
REF = {(100, 100): (229, 73, 71), (100, 1000): (229, 66, 66), (1000, 100): (222, 65, 64),
       (1000, 1000): (171, 77, 74), (1000, 10000): (149, 53, 53), (10000, 1000): (154, 55, 55),
       (10000, 10000): (103, 39, 38), (16385, 16385): (89, 31, 31), (32768, 32768): (107, 50, 49)}


def timed(eng, fn, n):
    fn()
    eng.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    eng.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    eng = rs16.default_engine()
    only = os.environ.get("RS16_ROWS_ONLY")  # e.g. "1000:1000,100:100"
    for (k, m), ref in REF.items():
        if only and f"{k}:{m}" not in only.split(","):
            continue
        original = generate_original(k, S, 0)
        d_orig = DeviceArray.from_numpy(eng, original)
        d_rec = DeviceArray(eng, m * S)
        enc = lambda: rs16.encode_device(k, m, S, d_orig.ptr, d_rec.ptr, engine=eng)
        mib = (k + m) * S / 2**20
        n = max(5, min(200, int(2e9 / ((k + m) * S))))
        row = {"k": k, "m": m, "shard_bytes": S, "rate": "high" if rs16.use_high_rate(k, m) else "low",
               "encode_us": round(timed(eng, enc, n) * 1e6, 2)}
        row["encode_mib_s"] = round(mib / row["encode_us"] * 1e6, 1)
        for pct in (1, 100):
            loss = min(k, m) * pct // 100
            of = np.ones(k, np.uint8)
            of[k - loss:] = 0
            rf = np.zeros(m, np.uint8)
            rf[:loss] = 1
            held = original.copy()
            held[k - loss:] = 0xA5
            d_rest = DeviceArray.from_numpy(eng, held)
            d_of, d_rf = DeviceArray.from_numpy(eng, of), DeviceArray.from_numpy(eng, rf)
            dec = lambda: rs16.decode_device(k, m, S, d_rest.ptr, d_of.ptr, d_rec.ptr, d_rf.ptr, k - loss, loss,
                                             engine=eng)
            t = timed(eng, dec, n)
            ok = bool(np.array_equal(d_rest.download(shape=(k, S)), original))
            # (RS16_ROWS_NOCHECK=1: timing probes of deliberately wrong builds)
            assert ok or os.environ.get("RS16_ROWS_NOCHECK"), f"{k}:{m} {pct}% decode did not restore"
            row[f"decode_{pct}pct_us"] = round(t * 1e6, 2)
            row[f"decode_{pct}pct_mib_s"] = round(mib / t, 1)
        row["reference_cpu_mib_s"] = {"encode": ref[0], "decode_1pct": ref[1], "decode_100pct": ref[2],
                                      "source": "README.md:129-137 (i5-3570K, 1 thread, NoSimd)"}
        row["restored"] = True
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
