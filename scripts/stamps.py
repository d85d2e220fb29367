"""Phase timeline of the pass kernels (diagnostic; needs a -DRS16_STAMPS=1
library, e.g. RS16_LIB=reed-solomon-16_amd/build_stamps/librs16.so).

Runs the bench's step (32768:32768 x 1 KiB encode + 100 %-loss decode) with
the stamps of one pass program at a time and prints, per pass: the spread
of workgroup start / end times (s_memrealtime, 100 MHz) and the median
duration of each phase of a workgroup (s_memtime cycles at the workgroup's
own clock).  Phases (rs16_pass.hip stamp()): 0 start, 1 loads issued,
2 tables staged, 3 first layout-A layers, 4 layout switch, 5 first
direction done, 6 formal derivative, 7 layout-B FFT layers, 8 layout
switch, 9 last layers, 10 stores issued, 11 stores done; EVAL_POLY (the
n <= 2048 eval kernel, rs16_misc.hip): 0 start, 1 flags in, 2 sums done,
10 store issued, 11 store done.  Programs: RS16_STAMP_PROGS (comma list);
size: argv[1] (k = m); loss pattern: RS16_STAMPS_LOSS, RS16_STAMPS_SCATTER
(below)."""
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import rs16  # noqa: E402
from rs16._lib import RS16Error, lib  # noqa: E402
from rs16.device import DeviceArray  # noqa: E402
from rs16.util import generate_original  # noqa: E402

PH = ["start", "loads", "staged", "A-layers", "switch1", "dir1", "fd", "B-fft", "switch2", "last", "stores", "drain"]
# the column codec (rs16_col.hip cstamp)
PH_COL = ["start", "issued", "staged", "iblk0", "iblk2", "ifft", "fblk0", "fblk2", "fxchg3", "fft", "stores", "drain"]


def main():
    k = m = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    S = 1024
    eng = rs16.Engine(0)
    original = generate_original(k, S, 0)
    d_orig = DeviceArray.from_numpy(eng, original)
    d_rec = DeviceArray(eng, m * S)
    # RS16_STAMPS_LOSS=L: the decode loses the last L originals and receives
    # recovery 0..L (the reference bench's 1 % pattern for L = k / 100);
    # default: every original lost (the half-transform decode)
    # RS16_STAMPS_SCATTER=1: the L lost originals and the L received recovery
    # shards are drawn at random instead (bench.py general_decodes)
    L = int(os.environ.get("RS16_STAMPS_LOSS", k))
    of = np.ones(k, np.uint8)
    rf = np.zeros(m, np.uint8)
    if os.environ.get("RS16_STAMPS_SCATTER"):
        rng = np.random.default_rng(7)
        of[rng.choice(k, L, replace=False)] = 0
        rf[rng.choice(m, L, replace=False)] = 1
    else:
        of[k - L:] = 0
        rf[:L] = 1
    held = original.copy()
    held[of == 0] = 0
    d_rest = DeviceArray.from_numpy(eng, held)
    d_of = DeviceArray.from_numpy(eng, of)
    d_rf = DeviceArray.from_numpy(eng, rf)

    def step():
        rs16.encode_device(k, m, S, d_orig.ptr, d_rec.ptr, engine=eng)
        rs16.decode_device(k, m, S, d_rest.ptr, d_of.ptr, d_rec.ptr, d_rf.ptr, k - L, L, engine=eng)

    for _ in range(3):
        step()
    eng.synchronize()
    if not os.environ.get("RS16_NO_VERIFY"):
        assert np.array_equal(d_rest.download(shape=(k, S)), original)
    names = {lib().rs16_prog_name(i).decode(): i for i in range(lib().rs16_prog_count())}
    nwg = 8192
    buf = DeviceArray(eng, nwg * 16 * 8)
    err = RS16Error()
    out = {}
    raw = {}
    progs = os.environ.get("RS16_STAMP_PROGS", "ENC_FIRST,ENC_MID,ENC_LAST,DEC_HALF_FIRST,DEC_HALF_MID,DEC_HALF_LAST")
    for name in progs.split(","):
        buf.upload(np.zeros(nwg * 16, np.uint64))
        lib().rs16_engine_set_stamps(eng.h, buf.ptr, names[name], C.byref(err))
        step()
        eng.synchronize()
        lib().rs16_engine_set_stamps(eng.h, None, -1, C.byref(err))
        st = buf.download(np.uint64).reshape(nwg, 16).astype(np.int64)
        st = st[st[:, 0] != 0]
        if len(st) == 0:
            continue
        raw[name] = st
        rt0 = st[:, 14].min()
        start_us = (st[:, 14] - rt0) / 100.0
        end_us = (st[:, 15] - rt0) / 100.0
        ghz = (st[:, 11] - st[:, 0]) / np.maximum(st[:, 15] - st[:, 14], 1) / 100.0 * 1e-0 * 100 / 100
        ghz = (st[:, 11] - st[:, 0]) / np.maximum((st[:, 15] - st[:, 14]) * 10.0, 1)  # cycles per ns
        rec = [p for p in range(12) if (st[:, p] != 0).all()]
        phases = {}
        for a, b in zip(rec, rec[1:]):
            dur = (st[:, b] - st[:, a]) / ghz / 1000.0  # us
            ph = PH_COL if name.startswith("COL") else PH
            phases[f"{ph[a]}->{ph[b]}"] = round(float(np.median(dur)), 2)
        out[name] = {
            "workgroups": int(len(st)),
            "clock_ghz_median": round(float(np.median(ghz)), 3),
            "start_spread_us": round(float(start_us.max()), 2),
            "end_min_max_us": [round(float(end_us.min()), 2), round(float(end_us.max()), 2)],
            "lifetime_median_us": round(float(np.median(end_us - start_us)), 2),
            "phase_median_us": phases,
        }
        # by XCD (HW reg XCC_ID) and by start order within a CU (HW_ID cu/sh/se)
        xcc = st[:, 13] & 15
        by = {}
        for x in np.unique(xcc):
            sel = xcc == x
            by[int(x)] = [round(float(np.median(end_us[sel])), 1), round(float(end_us[sel].max()), 1),
                          round(float(np.median((end_us - start_us)[sel])), 1)]
        out[name]["xcd_end_median_max_life"] = by
        hw = st[:, 12]
        cu = (xcc << 16) | (((hw >> 8) & 15) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5))
        rank = np.zeros(len(st), np.int64)
        for c in np.unique(cu):
            idx = np.nonzero(cu == c)[0]
            rank[idx[np.argsort(start_us[idx], kind="stable")]] = np.arange(len(idx))
        out[name]["cu_rank_life_median"] = {int(r): round(float(np.median((end_us - start_us)[rank == r])), 1)
                                            for r in np.unique(rank)}
        out[name]["cu_rank_end_median"] = {int(r): round(float(np.median(end_us[rank == r])), 1)
                                           for r in np.unique(rank)}
        print(name, json.dumps(out[name]), flush=True)
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / os.environ.get("RS16_STAMPS_OUT", "stamps.json")).write_text(json.dumps(out, indent=1))
    np.savez_compressed(ROOT / "gpurun_out" / "stamps_raw.npz", **raw)


if __name__ == "__main__":
    main()
