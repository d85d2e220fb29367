#!/usr/bin/env python3
"""Benchmark: device-resident GF(2^16) Reed-Solomon encode+decode on MI355X.

Metric (BASELINE.json): "encode+decode GiB/s (device-resident, 1024B shards);
% of HBM roofline".  A step = one encode (reed_solomon_16::encode,
src/lib.rs:242-279) plus one decode at 100 % original loss (recovery shards
0..k given, no originals; benches/benchmarks.rs:82-106) of one stripe of
32768:32768 x 1024 B shards (BASELINE configs[3], the largest single-GPU
configuration), inputs resident in HBM, through the C ABI
(rs16_encode_device / rs16_decode_device).  GiB/s counts
(original + recovery) bytes for the encode and again for the decode
(README.md:114-116; benches/benchmarks.rs:56-58).

Multi-GPU (--gpus N, one process per GPU via torch.distributed.run): every
rank encodes+decodes its own independent stripe (seed = rank), no data-path
collective; value = all ranks' bytes / max-over-ranks time ("weak").

Also reported: roofline of the dominant kernel (hipEvent-timed live in a
profiled copy of the timed loop; PMC traffic from profiles/ if present) and
the CPU baseline (the oracle's C restatement of the reference NoSimd engine,
1 core, rank 0 at N=1 only, bounded sample).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))

METRIC = "encode+decode GiB/s (device-resident, 1024B shards); % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
GIB = 2.0 ** 30


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--original", type=int, default=32768)
    p.add_argument("--recovery", type=int, default=32768)
    p.add_argument("--shard-bytes", type=int, default=1024)
    p.add_argument("--slices", type=int, default=1, help="concurrent column slices of the device codec")
    p.add_argument("--split-decode", action="store_true",
                   help="issue the step's decode split (rs16_decode_prepare on a side stream during the encode)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="bound of the CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extra", action="store_true", help="skip the 1000:1000 side measurements")
    p.add_argument("--no-verify", action="store_true", help="diagnostic (ablation) builds only")
    p.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    p.add_argument("--cpu-stub", action="store_true",
                   help="tests only: no GPU, a numpy stand-in step through the multi-rank control plane")
    return p.parse_args()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def pass_bytes(prog: str, k: int, m: int, S: int, orig_rcv=None, rec_rcv=None) -> float:
    """Algorithmic HBM bytes of one launch of a pass program (rows read + rows
    written, S bytes each) for a single-chunk high-rate k:m codec.  Decode
    passes follow the received masks (default: the bench's 100 % loss,
    recovery [0, k) given).  Full decode: a DEC_FIRST tile without a received
    row is neither read nor written, and its rows are not read again by
    DEC_MID / DEC_LAST (rs16_pass.hip, "decode zero tiles").  Half-transform
    decode (every original lost, rs16_engine.cpp half_decode): DEC_HALF_FIRST
    reads the received rows and writes n/2 work rows, DEC_HALF_MID reads and
    writes n/2 rows, DEC_HALF_LAST reads the tiles that hold originals and
    writes the lost originals."""
    import numpy as np

    chunk = 1 << (m - 1).bit_length()
    n_dec = 1 << (chunk + k - 1).bit_length()
    L_enc, L_dec = chunk.bit_length() - 1, n_dec.bit_length() - 1
    lo_e, lo_d = L_enc // 2, L_dec // 2
    if orig_rcv is None:
        orig_rcv = np.zeros(k, bool)
    if rec_rcv is None:
        rec_rcv = np.arange(m) < min(k, m)
    rcv = np.zeros(n_dec, bool)
    rcv[:m] = rec_rcv
    rcv[chunk:chunk + k] = orig_rcv
    tile = 1 << lo_d
    live = rcv.reshape(-1, tile).any(axis=1)  # DEC_FIRST tiles that are computed and stored
    t0, t1 = chunk // tile, -(-(chunk + k) // tile)  # DEC_LAST tiles (hold originals)
    h = n_dec // 2
    lo_h = (L_dec - 1) // 2
    if prog == "DEC_HALF_FIRST":
        rows = int(rcv[:h].sum()) + h
    elif prog == "DEC_HALF_MID":
        rows = 2 * h
    elif prog == "DEC_HALF_LAST":
        rows = (-(-k // (1 << lo_h)) << lo_h) + int((~orig_rcv).sum())
    elif prog == "DEC_HALF_SINGLE":
        rows = int(rcv[:h].sum()) + int((~orig_rcv).sum())
    elif prog == "ENC_FIRST":
        rows = k + chunk
    elif prog == "ENC_MID":
        rows = 2 * chunk
    elif prog == "ENC_LAST":
        tiles_rows = -(-m // (1 << lo_e)) << lo_e
        rows = tiles_rows + m
    elif prog == "DEC_FIRST":
        rows = int(rcv.sum()) + int(live.sum()) * tile
    elif prog == "DEC_MID":
        rows = int(live.sum()) * tile + (t1 - t0) * tile
    elif prog == "DEC_LAST":
        rows = (t1 - t0) * tile + int(live[t0:t1].sum()) * tile + int((~orig_rcv).sum())
    elif prog == "ENC_SINGLE":
        rows = k + m
    elif prog == "DEC_SINGLE":
        rows = 2 * k
    else:
        return 0.0
    return float(rows) * S


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_baseline(original, recovery, k, m, S, budget_s):
    """The oracle's NoSimd engine (C restatement of src/engine/engine_nosimd.rs
    + the rates), 1 thread, timed the way the reference bench times it: per
    iteration add_original_shard x k + encode, or add_*_shard + decode at 1 %
    and 100 % original loss (benches/benchmarks.rs:60-109), in a C loop
    (oracle_bench_main) so no Python call sits inside the timed iterations.
    Rows: BASELINE configs[0] (100:100), configs[1]/[2] (1000:1000) and the
    headline k:m; `value` = the headline encode + 100 %-loss decode rate."""
    import ctypes as C

    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np
    import oracle_bind as O
    from rs16.util import generate_original

    L = O.lib()
    f = L.oracle_bench_main
    f.restype = C.c_int
    f.argtypes = [C.c_int, C.c_size_t, C.c_size_t, C.c_size_t, C.c_void_p, C.c_void_p, C.c_int, C.c_double,
                  C.POINTER(C.c_size_t), C.POINTER(C.c_double)]

    def row(kk, mm, orig, rec, loss, min_s):
        it, sec = C.c_size_t(), C.c_double()
        rc = f(1, kk, mm, S, orig.ctypes.data, rec.ctypes.data, loss, min_s, C.byref(it), C.byref(sec))
        assert rc == 0, f"oracle bench failed: {rc}"
        t = sec.value / it.value
        return {"us": round(t * 1e6, 1), "mib_s": round((kk + mm) * S / t / 2**20, 2), "iters": it.value}

    rows = {}
    t_start = time.perf_counter()
    for kk, mm in ((100, 100), (1000, 1000)):
        o = generate_original(kk, S, 0)
        r = O.encode(kk, mm, o)
        rows[f"{kk}:{mm}"] = {"encode": row(kk, mm, o, r, -1, budget_s / 12),
                              "decode_1pct": row(kk, mm, o, r, 1, budget_s / 12),
                              "decode_100pct": row(kk, mm, o, r, 100, budget_s / 12)}
    orig = np.ascontiguousarray(original)
    rec = np.ascontiguousarray(recovery)
    big = {"encode": row(k, m, orig, rec, -1, 0.0), "decode_100pct": row(k, m, orig, rec, 100, 0.0)}
    if k >= 100:
        big["decode_1pct"] = row(k, m, orig, rec, 1, 0.0)
    rows[f"{k}:{m}"] = big
    t_e, t_d = big["encode"]["us"] * 1e-6, big["decode_100pct"]["us"] * 1e-6
    value = 2 * (k + m) * S / (t_e + t_d) / GIB
    return {"value": round(value, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"reference bench loop (benches/benchmarks.rs:60-109) in C on the oracle's NoSimd restatement, "
                      f"1 thread of {cpu_model()} (nproc {os.cpu_count()}); value = {k}:{m} x {S} B encode + "
                      f"100%-loss decode (one iteration each); rows in MiB/s as the reference README reports "
                      f"(README.md:127-137); {time.perf_counter() - t_start:.1f} s of CPU work in all; Rust "
                      f"reference not buildable here",
            "rows": rows}


def api_reference_loop(S, seconds):
    """The reference's own benchmark loop (benches/benchmarks.rs:60-109) over
    the C ABI: reed-solomon-16_amd/build/rs16_bench_api, a compiled C++ caller
    of librs16.so (as an FFI caller would be), shards in pageable host memory,
    per-shard add_* calls, encode()/decode().  Recovery of the first round is
    checked against the oracle fixture hashes (tests/golden/kib_hashes.json)."""
    import tempfile

    from rs16.util import generate_original

    tool = ROOT / "reed-solomon-16_amd" / "build" / "rs16_bench_api"
    fx = json.loads((ROOT / "tests" / "golden" / "kib_hashes.json").read_text())
    want = {(c["k"], c["m"]): c["recovery_sha256"] for c in fx["cases"] if c["shard_bytes"] == S and c["seed"] == 0}
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for kk, mm in ((100, 100), (1000, 1000), (32768, 32768)):
            fo, fr = Path(td) / "orig.bin", Path(td) / "rec.bin"
            generate_original(kk, S, 0).tofile(fo)
            res = subprocess.run([str(tool), str(kk), str(mm), str(S), str(fo), str(fr), str(seconds)],
                                 capture_output=True, text=True, timeout=300)
            if res.returncode != 0:
                raise RuntimeError(f"rs16_bench_api {kk}:{mm} failed: {res.stderr.strip()}")
            row = json.loads(res.stdout)
            h = hashlib.sha256(fr.read_bytes()).hexdigest()
            if (kk, mm) in want:
                assert h == want[(kk, mm)], f"API-path recovery {kk}:{mm} differs from the oracle fixture"
                row["recovery_sha256_matches_oracle_fixture"] = True
            out[f"{kk}:{mm}"] = row
    return out


def sustained(eng, step, step_bytes, dist, seconds=0.45):
    """The step back to back for `seconds` of GPU time (VERDICT r3 item 5;
    the reference's Criterion bench samples for seconds,
    benches/benchmarks.rs:33-113), one hipEvent pair per step on the engine
    stream, after a 0.5 s idle pause so that the start is cold: whole-run
    GiB/s and the first-20 / last-20 step medians (the difference is the GPU
    settling its clocks, not the codec)."""
    import ctypes as C

    import numpy as np

    from rs16._lib import hip_runtime

    hip = hip_runtime()  # (librs16's HIP runtime, not the copy torch brings along at N > 1)
    hip.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
    hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
    hip.hipEventSynchronize.argtypes = [C.c_void_p]
    hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    hip.hipEventDestroy.argtypes = [C.c_void_p]
    eng.synchronize()
    t0 = time.perf_counter()
    step()
    eng.synchronize()
    n = max(40, int(seconds / max(time.perf_counter() - t0, 50e-6)))
    evs = [C.c_void_p() for _ in range(n + 1)]
    for e in evs:
        assert hip.hipEventCreate(C.byref(e)) == 0
    s = C.c_void_p(eng.stream)
    if dist is not None:
        dist.barrier()
    time.sleep(0.5)
    hip.hipEventRecord(evs[0], s)
    for i in range(n):
        step()
        hip.hipEventRecord(evs[i + 1], s)
    hip.hipEventSynchronize(evs[n])
    t = np.empty(n)
    f = C.c_float()
    for i in range(n):
        hip.hipEventElapsedTime(C.byref(f), evs[i], evs[i + 1])
        t[i] = f.value * 1e-3
    for e in evs:
        hip.hipEventDestroy(e)
    return {"gib_s": round(step_bytes * n / t.sum() / GIB, 1), "gpu_seconds": round(float(t.sum()), 3), "steps": n,
            "first20_median_us": round(float(np.median(t[:20])) * 1e6, 1),
            "last20_median_us": round(float(np.median(t[-20:])) * 1e6, 1),
            "median_us": round(float(np.median(t)) * 1e6, 1),
            "note": "cold start after 0.5 s idle, hipEvent per step on the engine stream"}


def configs4_rccl(eng, k, m, world, rank, dist, timed, barrier, steps):
    """BASELINE configs[4]: one 32768:32768 x 64 KiB stripe resident in rank
    0's HBM, byte-column partitioned across the ranks with RCCL over xGMI
    (rs16_scatter_columns / rs16_gather_columns, include/rs16.h): scatter the
    originals' column slices, every rank encodes its slice, gather the
    recovery slices; then scatter the recovery, every rank decodes its slice
    at 100 % original loss, gather the restored originals.  Timed end to end
    (barrier + max over ranks) and as codec only / collectives only.  At one
    rank the collectives are the root's own-slice copies (no RCCL traffic);
    the whole-stripe restore is checked on rank 0."""
    import numpy as np

    import rs16
    from rs16.device import DeviceArray

    S4 = 65536
    if world == 1:
        (comm,) = rs16.Comm.init_all([eng])
    else:
        # unique id from rank 0 over the gloo control plane; the communicator
        # init has a deadline (rs16_comm.cpp), and every rank learns whether
        # all of them got one before any collective is issued
        import torch
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            uid[:] = torch.frombuffer(bytearray(rs16.Comm.unique_id()), dtype=torch.uint8)
        dist.broadcast(uid, 0)
        comm, why = None, ""
        try:
            comm = rs16.Comm(eng, world, rank, bytes(uid.numpy().tobytes()))
        except Exception as exc:  # reported below, after every rank knows
            why = f"{type(exc).__name__}: {exc}"
        ok = torch.tensor([1 if comm is not None else 0], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            if comm is not None:
                comm.close()
            return {"error": f"RCCL communicator init failed on some rank ({why or 'another rank'})"}
    off, w = rs16.column_slice(S4, world, rank)
    root = rank == 0
    d_orig = d_rec = d_out = None
    if root:
        orig = np.frombuffer(np.random.default_rng(4).bytes(k * S4), np.uint8).reshape(k, S4)
        d_orig = DeviceArray.from_numpy(eng, orig)
        d_rec, d_out = DeviceArray(eng, m * S4), DeviceArray(eng, k * S4)
    d_os, d_rs = DeviceArray(eng, k * w), DeviceArray(eng, m * w)
    d_ds = DeviceArray(eng, k * w)
    of = DeviceArray.from_numpy(eng, np.zeros(k, np.uint8))
    rf = DeviceArray.from_numpy(eng, np.ones(m, np.uint8))
    full = lambda d: [d.ptr if d is not None else 0]

    def scatter_orig():
        rs16.scatter_columns([comm], 0, k, S4, full(d_orig), [d_os.ptr])

    def gather_rec():
        rs16.gather_columns([comm], 0, m, S4, [d_rs.ptr], full(d_rec))

    def scatter_rec():
        rs16.scatter_columns([comm], 0, m, S4, full(d_rec), [d_rs.ptr])

    def gather_out():
        rs16.gather_columns([comm], 0, k, S4, [d_ds.ptr], full(d_out))

    def codec():
        rs16.encode_device(k, m, w, d_os.ptr, d_rs.ptr, engine=eng)
        rs16.decode_device(k, m, w, d_ds.ptr, of.ptr, d_rs.ptr, rf.ptr, 0, m, engine=eng)

    def step():
        scatter_orig()
        rs16.encode_device(k, m, w, d_os.ptr, d_rs.ptr, engine=eng)
        gather_rec()
        scatter_rec()
        rs16.decode_device(k, m, w, d_ds.ptr, of.ptr, d_rs.ptr, rf.ptr, 0, m, engine=eng)
        gather_out()

    step()
    barrier()
    ok = None
    if root:
        ok = bool(np.array_equal(d_out.download(shape=(k, S4)), orig))
        assert ok, "configs[4] via RCCL: decode did not restore the stripe"
    step()
    n4 = max(3, steps // 4)
    t_all = timed(step, n4)
    codec_rank = []
    t_codec = timed(codec, n4, codec_rank)
    t_coll = timed(lambda: (scatter_orig(), gather_rec(), scatter_rec(), gather_out()), n4)
    # Each collective on its own: the bytes that cross
    # the links (every column but the root's own slice: rows x (S - w_root)),
    # the achieved rate over the root's links and per peer link, and the
    # root's own pitched slice copy (rows x w_root, the only data movement at
    # one rank).
    w0 = rs16.column_slice(S4, world, 0)[1]
    peers = world - 1
    coll = {}
    for name, fn, rows in (("scatter_originals", scatter_orig, k), ("gather_recovery", gather_rec, m),
                           ("scatter_recovery", scatter_rec, m), ("gather_originals", gather_out, k)):
        t = timed(fn, n4) / n4
        link_bytes = rows * (S4 - w0) if peers else 0
        coll[name] = {"ms": t * 1e3, "link_bytes": link_bytes,
                      "root_links_gb_s": link_bytes / t / 1e9 if peers else None,
                      "per_peer_gb_s": link_bytes / peers / t / 1e9 if peers else None,
                      "root_own_slice_bytes": rows * w0, "root_own_slice_gb_s": rows * w0 / t / 1e9}
    comm.close()
    step_bytes = 2 * (k + m) * S4
    # The root sends (scatters) and receives (gathers) every column but its
    # own: 2 (k + m) (S - w_root) bytes a step, over min(N - 1, 7) xGMI links
    # of ~153 GB/s each (point to point; one direction per phase, the phases
    # in sequence), plus the codec on 1 / N of the columns per rank.
    link_gbs = 153.0
    bound_ms = (2 * (k + m) * (S4 - w0) / (min(peers, 7) * link_gbs * 1e9) * 1e3) if peers else 0.0
    return {
        "workload": f"{k}:{m} x {S4} B stripe in rank 0's HBM, byte columns split over {world} rank(s) "
                    f"({w} B each) with RCCL scatter/gather; encode + 100%-loss decode (BASELINE configs[4])",
        "gib_s": step_bytes * n4 / t_all / GIB, "ms_per_step": t_all / n4 * 1e3,
        "codec_only_gib_s": step_bytes * n4 / t_codec / GIB, "codec_only_ms": t_codec / n4 * 1e3,
        "codec_ms_per_rank": [round(t / n4 * 1e3, 4) for t in codec_rank],
        "collectives_ms": t_coll / n4 * 1e3,
        # scatter originals (k rows) + gather recovery (m) + scatter recovery (m)
        # + gather originals (k), each moving every column but the root's own slice
        "collective_bytes_per_step": 2 * (k + m) * (S4 - w0) if peers else 0,
        "collectives": coll,
        "root_link_bound_ms": bound_ms,
        "root_link_bound_note": f"2 (k + m) (S - w_root) bytes through rank 0 over min(N-1, 7) links x {link_gbs} GB/s",
        "expected_step_ms_at_link_bound": bound_ms + t_codec / n4 * 1e3,
        "restored_stripe_verified": ok, "whole_configs4": world == 8}


def two_stripes(eng, local, k, m, S, of, rf, loss, encode, decode, args, where):
    """Serving mode (not the metric): two independent stripes per step, one
    per engine / stream, so that one stripe's load and store phases overlap
    the other's butterflies; and the producer / consumer form, engine A
    encoding a stripe while engine B decodes another one's (already encoded)
    recovery.  Both restorations are checked.

    Two streams that share a hardware queue run one stripe after the other
    (scripts/probe_queues.py, profiles/r05_queues.txt).  The second engine is
    created with RS16_ENGINE_OWN_QUEUE (include/rs16.h: its stream gets a
    hardware queue of its own), so the pair overlaps by construction: ONE
    engine, no selection among candidates.  A second engine created the
    default way is measured beside it for comparison (`default_second_engine`):
    whether that one overlaps depends on which queue the runtime gives it."""
    import numpy as np

    import rs16
    from rs16.device import DeviceArray
    from rs16.util import generate_original

    o2 = generate_original(k, S, 1)
    step_bytes = 2 * (k + m) * S

    def run(engs, body, steps, warmup):
        for _ in range(warmup):
            body()
        for e in engs:
            e.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            body()
        for e in engs:
            e.synchronize()
        return time.perf_counter() - t0

    def one():
        encode()
        decode()

    # steady state: 30 untimed iterations, then 200 timed (a 20-step loop
    # right after a sync includes the GPU's clock ramp; scripts/probe_own_queue.py)
    nst, nwu = max(200, args.steps), 30
    t1 = run([eng], one, nst, nwu) / nst

    def pair(flags):
        eng2 = rs16.Engine(local, flags)
        a2, r2, x2 = DeviceArray.from_numpy(eng2, o2), DeviceArray(eng2, m * S), DeviceArray(eng2, k * S)
        f2o, f2r = DeviceArray.from_numpy(eng2, of), DeviceArray.from_numpy(eng2, rf)
        if loss < k:
            x2.upload(o2)

        def enc2():
            rs16.encode_device(k, m, S, a2.ptr, r2.ptr, engine=eng2)

        def dec2():
            rs16.decode_device(k, m, S, x2.ptr, f2o.ptr, r2.ptr, f2r.ptr, k - loss, loss, engine=eng2)

        def two():
            encode()
            enc2()
            decode()
            dec2()

        def enc_dec():
            encode()
            dec2()

        two()
        eng2.synchronize()
        assert np.array_equal(x2.download(shape=(k, S)), o2), "second stream: decode did not restore"
        t2 = run([eng, eng2], two, nst, nwu)
        t3 = run([eng, eng2], enc_dec, nst, nwu)
        assert np.array_equal(x2.download(shape=(k, S)), o2), "second stream: decode did not restore"
        del a2, r2, x2, f2o, f2r
        eng2.close()
        return t2, t3

    t2, t3 = pair(rs16.Engine.OWN_QUEUE)
    t2d, t3d = pair(0)
    return {"gib_s": 2 * step_bytes * nst / t2 / GIB, "ms_per_two_stripes": t2 / nst * 1e3,
            "encode_while_decode_gib_s": step_bytes * nst / t3 / GIB,
            "encode_while_decode_us": t3 / nst * 1e6, "where": where, "steps": nst, "warmup": nwu,
            "one_stripe_gib_s": step_bytes / t1 / GIB,
            "two_stripe_time_over_one": round(t2 / nst / t1, 3),
            "second_engine": "rs16_engine_new_ex(RS16_ENGINE_OWN_QUEUE): one engine, no selection",
            "default_second_engine": {"gib_s": 2 * step_bytes * nst / t2d / GIB,
                                      "encode_while_decode_gib_s": step_bytes * nst / t3d / GIB,
                                      "two_stripe_time_over_one": round(t2d / nst / t1, 3),
                                      "note": "second engine from rs16_engine_new: its stream's hardware queue is "
                                              "the runtime's choice (a shared queue runs the pair serially, ~2.0)"},
            "note": "serving-mode throughput: two independent 32768:32768 x 1 KiB stripes in flight "
                    "(gib_s), or one stripe encoding on engine A while another's recovery decodes on "
                    "engine B (encode_while_decode); not the metric"}


def extra_on(name):
    """Extras to leave out of a diagnostic run: RS16_BENCH_SKIP = comma list of
    extra names (two_stripes, sustained, kib1000, batched, decode_1pct,
    general_decodes, rate_paths, column_slices, configs4, host_resident,
    host_batch, api_loop).  Unset for every real measurement."""
    return name not in os.environ.get("RS16_BENCH_SKIP", "").split(",")


def make_timed(sync, dist, world):
    """timed(fn, steps[, per_rank]): run fn `steps` times between two
    barriers (device sync + gloo barrier) and return the MAX over ranks of the
    wall time; `per_rank` (a list) receives every rank's own time, in rank
    order, so that a straggler of a multi-GPU run can be named."""
    def barrier():
        sync()
        if dist is not None:
            dist.barrier()

    def timed(fn, steps, per_rank=None):
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        sync()
        dt = time.perf_counter() - t0
        barrier()
        if dist is not None:
            import torch
            t = torch.tensor([dt], dtype=torch.float64)
            if per_rank is not None:
                allt = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
                dist.all_gather(allt, t)
                per_rank[:] = [float(x.item()) for x in allt]
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        elif per_rank is not None:
            per_rank[:] = [dt]
        return dt

    return timed, barrier


def rank_identity(local, device):
    """Who this rank is: host, local rank, the HIP device index it runs on and
    the visible-device list the launcher gave it."""
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") or \
        os.environ.get("CUDA_VISIBLE_DEVICES")
    return {"hostname": socket.gethostname(), "local_rank": local, "device": device, "visible_devices": vis,
            "pid": os.getpid()}


def gather_ranks(dist, world, ident, per_rank_dt, steps, rank_bytes):
    """Per-rank rows of the timed loop for the JSON line (rank order): the
    rank's identity, its own time per step and its own GiB/s.  The metric
    itself stays world x bytes / max-over-ranks time."""
    idents = [ident]
    if dist is not None:
        idents = [None] * world
        dist.all_gather_object(idents, ident)
    rows = []
    for r, (who, dt) in enumerate(zip(idents, per_rank_dt)):
        row = {"rank": r}
        row.update(who)
        row.update({"ms_per_step": round(dt / steps * 1e3, 4), "gib_s": round(rank_bytes * steps / dt / GIB, 3)})
        rows.append(row)
    return rows


def stub_main(args, world, rank, local, dist, json_fd):
    """--cpu-stub (tests only, no GPU): the multi-rank control plane of main()
    -- barriers, max over ranks, per-rank rows, the configs4 per-rank codec
    times -- around a numpy stand-in for the step, so that a CPU test can run
    `bench.py --gpus 2` under gloo and check the line's fields.  The line says
    "stub": it is never a measurement."""
    import numpy as np

    buf = np.random.default_rng(rank).integers(0, 256, 1 << 20, dtype=np.uint8)

    def step():
        np.bitwise_xor(buf, 0x5A, out=buf)

    timed, _ = make_timed(lambda: None, dist, world)
    per_rank = []
    for _ in range(args.warmup):
        step()
    dt = timed(step, args.steps, per_rank)
    codec_rank = []
    timed(step, max(3, args.steps // 4), codec_rank)
    step_bytes = 2 * buf.size
    ranks = gather_ranks(dist, world, rank_identity(local, -1), per_rank, args.steps, step_bytes)
    if rank == 0:
        out = {"metric": METRIC, "value": round(world * step_bytes * args.steps / dt / GIB, 3), "unit": "GiB/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(dt / args.steps * 1e3, 4), "stub": True, "ranks": ranks,
               "extra": {"configs4_rccl": {"codec_ms_per_rank": [round(t * 1e3, 4) for t in codec_rank]}}}
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()


def general_decodes(eng, k, m, S, original, d_rec, timed, args, world):
    """Decodes that take the general path: none of the
    metric decode's shortcuts applies (whole-half erasure -> identity logs,
    DESIGN.md 3.13; lost originals in <= 4 last-pass tiles -> direct middle
    pass, 3.14), as the reference runs its one sequence for every pattern
    (src/rate/rate_high.rs:181-242; random loss sets as
    examples/test-random-roundtrips.rs:118-128):
      scattered_1pct  - 327 random originals lost, 327 random recovery shards
      random_50pct    - 16384 random originals lost, as many random recovery shards
      30000:30000_100pct - every original lost, k = m not a power of two (no
                        identity logs: eval_poly + both per-row multiplies)
    Each: decode time (GiB/s over (k + m) S, as the metric counts a decode),
    restore checked, and the per-program kernel times of a profiled run."""
    import numpy as np

    import rs16
    from rs16.device import DeviceArray

    rng = np.random.default_rng(11)
    cases = {}
    for name in ("scattered_1pct", "random_50pct", "30000:30000_100pct"):
        kk, mm = k, m
        if name == "30000:30000_100pct":
            kk = mm = 30000
        o = original[:kk]
        lost = {"scattered_1pct": kk // 100, "random_50pct": kk // 2}.get(name, kk)
        of = np.ones(kk, np.uint8)
        rf = np.zeros(mm, np.uint8)
        if lost == kk:
            of[:] = 0
            rf[:lost] = 1
        else:
            of[rng.choice(kk, lost, replace=False)] = 0
            rf[rng.choice(mm, lost, replace=False)] = 1
        if kk == k and mm == m:
            rec = d_rec
        else:
            d_o = DeviceArray.from_numpy(eng, o)
            rec = DeviceArray(eng, mm * S)
            rs16.encode_device(kk, mm, S, d_o.ptr, rec.ptr, engine=eng)
        held = o.copy()
        held[of == 0] = 0
        d_x = DeviceArray.from_numpy(eng, held)
        d_of, d_rf = DeviceArray.from_numpy(eng, of), DeviceArray.from_numpy(eng, rf)
        dec = lambda: rs16.decode_device(kk, mm, S, d_x.ptr, d_of.ptr, rec.ptr, d_rf.ptr, kk - lost, lost,
                                         engine=eng)
        dec()
        assert np.array_equal(d_x.download(shape=(kk, S)), o), f"general decode {name} did not restore"
        for _ in range(args.warmup):
            dec()
        n = max(10, args.steps)
        t = timed(dec, n)
        eng.set_profiling(True)
        eng.profile_reset()
        for _ in range(n):
            dec()
        eng.synchronize()
        prof = eng.profile()
        eng.set_profiling(False)
        eng.profile_reset()
        cases[name] = {"decode_us": t / n * 1e6, "decode_gib_s": world * (kk + mm) * S * n / t / GIB,
                       "lost_originals": lost, "received_recovery": int(rf.sum()),
                       "kernels_us": {p: round(ms / c * 1e3, 2) for p, (ms, c) in prof.items()}}
    return cases


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "LOCAL_RANK" not in os.environ:
        # Relaunch one process per GPU before anything touches the GPU.
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(Path(__file__).resolve())]
        cmd += sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    dist = None
    # gloo and RCCL print connection / version banners on stdout: keep fd 1
    # for the one JSON line of rank 0 and send everything else to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if world > 1:
        # librs16.so first: its RCCL (ROCm's, the one include/rs16.h's
        # rccl.h describes) must be the librccl.so.1 of this process, not the
        # copy torch brings along (a different RCCL version)
        if not args.cpu_stub:
            from rs16._lib import lib as _rs16_lib
            _rs16_lib()
        import torch.distributed as dist  # control plane only (barrier, max of times)
        dist.init_process_group("gloo", init_method="env://")
    if args.cpu_stub:
        return stub_main(args, world, rank, local, dist, json_fd)

    import numpy as np

    import rs16
    from rs16.device import DeviceArray
    from rs16.util import generate_original

    k, m, S = args.original, args.recovery, args.shard_bytes
    # RS16_BENCH_SHARE_GPU=1: every rank on GPU 0 (rehearsal of the N > 1
    # path on a one-GPU box only; the driver's N-GPU runs use one GPU per rank)
    eng = rs16.Engine(0 if os.environ.get("RS16_BENCH_SHARE_GPU") == "1" else local)
    eng.set_slices(args.slices)
    seed = rank & 0xFF
    original = generate_original(k, S, seed)
    d_orig = DeviceArray.from_numpy(eng, original)
    d_rec = DeviceArray(eng, m * S)
    d_rest = DeviceArray(eng, k * S)
    loss = min(k, m)
    of = np.ones(k, np.uint8)
    of[:loss] = 0
    rf = np.zeros(m, np.uint8)
    rf[:loss] = 1
    d_of, d_rf = DeviceArray.from_numpy(eng, of), DeviceArray.from_numpy(eng, rf)
    if loss < k:
        d_rest.upload(original)  # received originals stay in place

    def encode():
        rs16.encode_device(k, m, S, d_orig.ptr, d_rec.ptr, engine=eng)

    def decode():
        rs16.decode_device(k, m, S, d_rest.ptr, d_of.ptr, d_rec.ptr, d_rf.ptr, k - loss, loss, engine=eng)

    # ---- correctness gate (the measured path must be the bit-exact one) ----
    encode()
    recovery = d_rec.download(shape=(m, S))
    verified = "decode restores every original bit-exactly"
    if seed == 0 and S == 1024:
        fx = json.loads((ROOT / "tests" / "golden" / "kib_hashes.json").read_text())
        want = {(c["k"], c["m"]): c["recovery_sha256"] for c in fx["cases"]}.get((k, m))
        if want is not None:
            got = hashlib.sha256(recovery.tobytes()).hexdigest()
            assert args.no_verify or got == want, f"recovery hash {got} != oracle fixture {want}"
            verified = "recovery SHA-256 == oracle fixture; " + verified
    decode()
    assert args.no_verify or np.array_equal(d_rest.download(shape=(k, S)), original), "decode did not restore"
    if args.no_verify:
        verified = "NOT VERIFIED (diagnostic build)"

    timed, barrier = make_timed(eng.synchronize, dist, world)

    # The step: encode the stripe, then decode its recovery at 100 % original
    # loss (encode, then rs16_decode_device, on the engine stream).  With
    # --split-decode the decode's erasure locator (rs16_decode_prepare, DESIGN.md
    # 3.12) is computed on a side stream while the encode runs; measured slower
    # (the locator's workgroups take slots from the encode's first pass, and the
    # cross-stream wait costs more than the 9 us it hides), so it is an extra.
    side = eng.create_stream()

    def step_serial():
        encode()
        decode()

    def step_split():
        rs16.decode_prepare(k, m, S, d_of.ptr, d_rf.ptr, k - loss, loss, stream=side, engine=eng)
        encode()
        rs16.decode_device_prepared(k, m, S, d_rest.ptr, d_rec.ptr, engine=eng)

    step = step_split if args.split_decode else step_serial
    held = original.copy()
    held[:loss] = 0
    d_rest.upload(held)
    step_split()
    assert args.no_verify or np.array_equal(d_rest.download(shape=(k, S)), original), "split decode did not restore"

    # ---- roofline: dominant kernel, hipEvent-timed on its launch stream ----
    # An event-profiled copy of the K-step loop, run BEFORE the W warm-up
    # steps and the timed loop, so that the timed loop runs unprofiled and
    # in the state the profiled copy leaves the GPU in (a GPU coming out of
    # idle runs steps ~10-25 of a cold start ~8 % slower while its clocks
    # settle: extra.sustained, CHANGELOG.md round 4).  Its own first 40 steps warm
    # the clocks and are not counted.  One column slice, so that every
    # timed launch is one kernel running alone.
    # The events are read (host work, GPU idle) only after the timed loop.
    eng.set_slices(1)
    eng.set_profiling(True)
    for _ in range(40):
        step()
    eng.synchronize()
    eng.profile()
    eng.profile_reset()
    timed(step, args.steps)
    eng.set_profiling(False)
    eng.set_slices(args.slices)

    for _ in range(args.warmup):
        step()
    per_rank_dt = []
    dt = timed(step, args.steps, per_rank_dt)
    prof = eng.profile()
    step_bytes = 2 * (k + m) * S  # encode + decode, (original + recovery) bytes each
    value = world * step_bytes * args.steps / dt / GIB
    ranks = gather_ranks(dist, world, rank_identity(local, eng.device), per_rank_dt, args.steps, step_bytes)
    ms_per_step = dt / args.steps * 1e3

    # Separate encode-only / decode-only rates (same data, same engine), and
    # the step issued the other way (split / serial decode).
    dt_e = timed(encode, args.steps)
    dt_d = timed(decode, args.steps)
    other = step_serial if args.split_decode else step_split
    for _ in range(args.warmup):
        other()
    dt_o = timed(other, args.steps)
    other_step = {"gib_s": world * step_bytes * args.steps / dt_o / GIB, "ms_per_step": dt_o / args.steps * 1e3,
                  "decode_issue": "serial: rs16_decode_device" if args.split_decode else
                  "split: rs16_decode_prepare on a side stream during the encode, then rs16_decode_device_prepared"}
    two_early = None
    if not args.no_extra and world == 1 and extra_on("two_stripes"):
        # the serving-mode rate measured right here as well as after the
        # other extras: VERDICT r4 item 1 (probe 900 vs bench 756 GiB/s)
        two_early = two_stripes(eng, local, k, m, S, of, rf, loss, encode, decode, args, "right after the timed loop")
    kernels = {name: {"avg_us": ms / n * 1e3, "launches": n} for name, (ms, n) in prof.items()}
    dom = max(prof, key=lambda p: prof[p][0])
    dom_avg_s = prof[dom][0] / prof[dom][1] / 1e3
    alg = pass_bytes(dom, k, m, S, of.astype(bool), rf.astype(bool))
    achieved = alg / dom_avg_s / 1e9
    traffic = None
    tp = Path(args.traffic_json)
    if tp.exists():
        try:
            tj = json.loads(tp.read_text())
            key = f"{dom}:{k}:{m}:{S}"
            traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": dom,
                "algorithmic_bytes_per_launch": alg,
                "whole_step_frac": round(step_bytes / (dt / args.steps) / 1e9 / HBM_PEAK_GBS, 4)}

    # The passes are bound by VALU issue, not HBM: the
    # same kernel against the VALU ceiling of this GF(2^16) butterfly.  A
    # wave-quad-butterfly (4 elements per lane: 12 v_perm_b32, 2 64-bit
    # selector shifts, 6 masks, 6 v_bitop3_b32, 2 XORs = 28 VALU
    # instructions) measured 110.4 SIMD cycles at 8 waves per SIMD (114.0 at
    # 4; tools/ubench_bfly.hip, profiles/r06_ubench_bfly64.txt; 115.7 with
    # the round-3 form's four 32-bit shifts): v_perm_b32 issues every ~4.2
    # cycles at any occupancy and any stream that mixes it with single-rate
    # ops runs at ~4 cycles per instruction (profiles/r03_ubench_mix.txt),
    # although those ops alone issue every ~2.5 (profiles/r03_ubench_valu.txt).
    # Ceiling = 1024 SIMDs x 256 element-butterflies / 110.4 cycles at the
    # 2.4 GHz peak clock.  Algorithmic work = element-butterflies of the
    # pass's layers.
    chunk = 1 << (m - 1).bit_length()
    L_e = chunk.bit_length() - 1
    lo_e, hi_e = L_e // 2, L_e - L_e // 2
    layers = {"ENC_FIRST": lo_e, "ENC_MID": 2 * hi_e, "ENC_LAST": lo_e, "DEC_HALF_FIRST": lo_e,
              "DEC_HALF_MID": 2 * hi_e, "DEC_HALF_LAST": lo_e}.get(dom)
    valu = None
    if layers is not None and L_e > 8:
        bfly = layers * (chunk // 2) * (S // 2)
        peak = 1024 * 256 / 110.4 * 2.4e9
        valu = {"bound": "valu", "kernel": dom, "achieved": round(bfly / dom_avg_s / 1e12, 3),
                "peak": round(peak / 1e12, 3), "unit": "T element-butterflies/s", "frac": round(bfly / dom_avg_s / peak, 4),
                "butterflies_per_launch": bfly,
                "note": "measured issue ceiling of this kernel's butterfly (110.4 cycles per 28-instruction "
                        "wave-quad-butterfly, profiles/r06_ubench_bfly64.txt) at 2.4 GHz; the zero-twiddle groups "
                        "the two-direction passes skip still count as butterflies here"}

    extra = {"serial_step" if args.split_decode else "split_decode_step": other_step}
    if not args.no_extra and extra_on("sustained"):
        extra["sustained"] = sustained(eng, step, step_bytes * world, dist)
    if not args.no_extra and (k, m) != (1000, 1000) and extra_on("kib1000"):
        # BASELINE configs[1] / [2]: 1000:1000 x 1 KiB encode, decode at 100 % loss
        k2 = m2 = 1000
        o2 = generate_original(k2, S, seed)
        a = DeviceArray.from_numpy(eng, o2)
        r = DeviceArray(eng, m2 * S)
        x = DeviceArray(eng, k2 * S)
        f0 = DeviceArray.from_numpy(eng, np.zeros(k2, np.uint8))
        f1 = DeviceArray.from_numpy(eng, np.ones(m2, np.uint8))
        e2 = lambda: rs16.encode_device(k2, m2, S, a.ptr, r.ptr, engine=eng)
        d2 = lambda: rs16.decode_device(k2, m2, S, x.ptr, f0.ptr, r.ptr, f1.ptr, 0, m2, engine=eng)
        e2()
        d2()
        assert np.array_equal(x.download(shape=(k2, S)), o2)
        # (steady state: each call kind warmed on its own, then >= 400 calls;
        # a few dozen calls after a sync measure the launch latency instead)
        n2 = max(10 * args.steps, 400)
        for _ in range(50):
            e2()
        te = timed(e2, n2)
        for _ in range(50):
            d2()
        td = timed(d2, n2)
        extra["1000:1000x1024"] = {"encode_gib_s": world * (k2 + m2) * S * n2 / te / GIB,
                                   "decode_gib_s": world * (k2 + m2) * S * n2 / td / GIB,
                                   "encode_us": te / n2 * 1e6, "decode_us": td / n2 * 1e6}
        # Many such stripes per call (rs16_encode_device_batch; serving
        # throughput, not the configs[1] latency): every stripe's recovery
        # must equal the single-stripe encode above.
        rec1 = r.download(shape=(m2, S))
        bat = {}
        for kb, nb in ((1000, 32), (100, 256)):
            ob = o2[:kb] if kb <= k2 else generate_original(kb, S, seed)
            db_o = DeviceArray.from_numpy(eng, np.tile(ob.reshape(1, -1), (nb, 1)))
            db_r = DeviceArray(eng, nb * kb * S)
            eb = lambda: rs16.encode_device_batch(kb, kb, S, nb, db_o.ptr, kb * S, db_r.ptr, kb * S, engine=eng)
            eb()
            got = db_r.download(shape=(nb, kb, S))
            if kb == m2:
                want = rec1
            else:
                d1o, d1r = DeviceArray.from_numpy(eng, ob), DeviceArray(eng, kb * S)
                rs16.encode_device(kb, kb, S, d1o.ptr, d1r.ptr, engine=eng)
                want = d1r.download(shape=(kb, S))
            assert all(np.array_equal(got[i], want) for i in (0, nb // 2, nb - 1)), "batched encode differs"
            nt = max(5, args.steps // 2)
            tb = timed(eb, nt)
            # the same stripes decoded at 100 % original loss with one shared
            # pattern (rs16_decode_device_batch: a failed device), restore checked
            fo = DeviceArray.from_numpy(eng, np.zeros(kb, np.uint8))
            fr = DeviceArray.from_numpy(eng, np.ones(kb, np.uint8))
            dx = DeviceArray.from_numpy(eng, np.zeros(nb * kb * S, np.uint8))
            dbf = lambda: rs16.decode_device_batch(kb, kb, S, nb, dx.ptr, kb * S, fo.ptr, db_r.ptr, kb * S, fr.ptr,
                                                   0, kb, engine=eng)
            dbf()
            back = dx.download(shape=(nb, kb, S))
            assert all(np.array_equal(back[i], ob) for i in (0, nb // 2, nb - 1)), "batched decode did not restore"
            td = timed(dbf, nt)
            bat[f"{kb}:{kb}x{S}x{nb}"] = {"encode_gib_s": world * nb * 2 * kb * S * nt / tb / GIB,
                                          "encode_us_per_call": tb / nt * 1e6,
                                          "decode_100pct_gib_s": world * nb * 2 * kb * S * nt / td / GIB,
                                          "decode_us_per_call": td / nt * 1e6, "stripes_per_call": nb}
            if kb == 1000:
                # every stripe with a loss set of its own (rs16_decode_device_batch_varied):
                # stripe i loses a random half of its originals and receives as
                # many random recovery shards; restore checked on every stripe
                rng = np.random.default_rng(7)
                fo_h = np.ones((nb, kb), np.uint8)
                fr_h = np.zeros((nb, kb), np.uint8)
                for i in range(nb):
                    fo_h[i, rng.choice(kb, kb // 2, replace=False)] = 0
                    fr_h[i, rng.choice(kb, kb // 2, replace=False)] = 1
                held = np.tile(ob.reshape(1, kb, S), (nb, 1, 1))
                held[fo_h == 0] = 0
                dv = DeviceArray.from_numpy(eng, held.reshape(-1))
                dfo, dfr = DeviceArray.from_numpy(eng, fo_h.reshape(-1)), DeviceArray.from_numpy(eng, fr_h.reshape(-1))
                oc, rc = [int(x) for x in fo_h.sum(1)], [int(x) for x in fr_h.sum(1)]
                dvf = lambda: rs16.decode_device_batch_varied(kb, kb, S, nb, dv.ptr, kb * S, dfo.ptr, kb, db_r.ptr,
                                                              kb * S, dfr.ptr, kb, oc, rc, engine=eng)
                dvf()
                back = dv.download(shape=(nb, kb, S))
                assert all(np.array_equal(back[i], ob) for i in range(nb)), "varied batched decode did not restore"
                tv = timed(dvf, nt)
                bat[f"{kb}:{kb}x{S}x{nb}"].update({
                    "decode_varied_gib_s": world * nb * 2 * kb * S * nt / tv / GIB,
                    "decode_varied_us_per_call": tv / nt * 1e6,
                    "decode_varied": "every stripe its own random loss of half its originals (general decode)"})
        extra["batched_stripes"] = bat

    if not args.no_extra and loss >= 100 and extra_on("decode_1pct"):
        # 1 % loss (benches/benchmarks.rs:84-87): originals 0..k-L and
        # recovery 0..L received, L = min(k, m) / 100; the last L originals
        # are restored in place.
        L1 = loss // 100
        of1 = np.ones(k, np.uint8)
        of1[k - L1:] = 0
        rf1 = np.zeros(m, np.uint8)
        rf1[:L1] = 1
        d_of1, d_rf1 = DeviceArray.from_numpy(eng, of1), DeviceArray.from_numpy(eng, rf1)
        o1 = original.copy()
        o1[k - L1:] = 0  # lost: must come back from the decode
        d_r1 = DeviceArray.from_numpy(eng, o1)
        d1 = lambda: rs16.decode_device(k, m, S, d_r1.ptr, d_of1.ptr, d_rec.ptr, d_rf1.ptr, k - L1, L1, engine=eng)
        d1()
        assert np.array_equal(d_r1.download(shape=(k, S)), original), "1 % loss decode did not restore"
        for _ in range(args.warmup):
            d1()
        t1 = timed(d1, args.steps)
        extra["decode_1pct_loss"] = {"decode_gib_s": world * (k + m) * S * args.steps / t1 / GIB,
                                     "decode_us": t1 / args.steps * 1e6, "lost_originals": L1,
                                     "received": f"originals 0..{k - L1}, recovery 0..{L1}"}

    if not args.no_extra and (k, m, S) == (32768, 32768, 1024) and extra_on("general_decodes"):
        extra["general_decodes"] = general_decodes(eng, k, m, S, original, d_rec, timed, args, world)

    if not args.no_extra and (k, m, S) == (32768, 32768, 1024) and extra_on("rate_paths"):
        # The multi-chunk rate paths: high rate with k > chunk
        # (60000:3000, 15 chunks of 4096) and low rate (3000:60000); encode,
        # then a decode that loses min(k, m) originals (the last ones for the
        # high rate, all of them for the low rate), restore checked.
        rp = {}
        for k3, m3 in ((60000, 3000), (3000, 60000)):
            o3 = generate_original(k3, S, 3)
            a3, r3 = DeviceArray.from_numpy(eng, o3), DeviceArray(eng, m3 * S)
            lost3 = min(k3, m3)
            of3 = np.ones(k3, np.uint8)
            of3[k3 - lost3:] = 0
            rf3 = np.zeros(m3, np.uint8)
            rf3[:lost3] = 1
            d_of3, d_rf3 = DeviceArray.from_numpy(eng, of3), DeviceArray.from_numpy(eng, rf3)
            h3 = o3.copy()
            h3[k3 - lost3:] = 0
            x3 = DeviceArray.from_numpy(eng, h3)
            e3 = lambda: rs16.encode_device(k3, m3, S, a3.ptr, r3.ptr, engine=eng)
            d3 = lambda: rs16.decode_device(k3, m3, S, x3.ptr, d_of3.ptr, r3.ptr, d_rf3.ptr, k3 - lost3, lost3,
                                            engine=eng)
            e3()
            d3()
            assert np.array_equal(x3.download(shape=(k3, S)), o3), f"{k3}:{m3} decode did not restore"
            n3 = max(5, args.steps // 2)
            te3, td3 = timed(e3, n3), timed(d3, n3)
            rp[f"{k3}:{m3}x{S}"] = {
                "rate": "high" if rs16.use_high_rate(k3, m3) else "low",
                "encode_gib_s": world * (k3 + m3) * S * n3 / te3 / GIB, "encode_us": te3 / n3 * 1e6,
                "decode_gib_s": world * (k3 + m3) * S * n3 / td3 / GIB, "decode_us": td3 / n3 * 1e6,
                "lost_originals": lost3}
        extra["rate_paths"] = rp

    if not args.no_extra and world > 1 and S % (64 * world) == 0 and extra_on("column_slices"):
        # Strong scaling of ONE stripe (the 1 KiB configs over N
        # GPUs as S / N byte-column slices): every rank encodes and decodes its
        # column slice of the same 32768:32768 x 1 KiB stripe (here: slice r
        # of this rank's originals; every slice is its own codeword set); the
        # whole stripe is done when the slowest rank is.
        off_s, w_s = rs16.column_slice(S, world, rank)
        sl = np.ascontiguousarray(original[:, off_s:off_s + w_s])
        d_so, d_sr, d_sx = DeviceArray.from_numpy(eng, sl), DeviceArray(eng, m * w_s), DeviceArray(eng, k * w_s)
        fo_s = DeviceArray.from_numpy(eng, of)
        fr_s = DeviceArray.from_numpy(eng, rf)

        def slice_step():
            rs16.encode_device(k, m, w_s, d_so.ptr, d_sr.ptr, engine=eng)
            rs16.decode_device(k, m, w_s, d_sx.ptr, fo_s.ptr, d_sr.ptr, fr_s.ptr, k - loss, loss, engine=eng)

        slice_step()
        if loss == k:
            assert np.array_equal(d_sx.download(shape=(k, w_s)), sl), "column-slice decode did not restore"
        for _ in range(args.warmup):
            slice_step()
        ts = timed(slice_step, args.steps)
        extra["one_stripe_column_slices"] = {
            "workload": f"one {k}:{m} x {S} B stripe, {w_s} B column slice per rank, encode + "
                        f"{'100%' if loss == k else 'partial'}-loss decode (strong scaling)",
            "gib_s": step_bytes * args.steps / ts / GIB, "ms_per_step": ts / args.steps * 1e3,
            "slice_bytes": w_s}

    if not args.no_extra and (k, m, S) == (32768, 32768, 1024) and extra_on("configs4"):
        extra["configs4_rccl"] = configs4_rccl(eng, k, m, world, rank, dist, timed, barrier, args.steps)

    if two_early is not None:
        extra["two_stripes_two_streams"] = two_early

    if not args.no_extra:
        # Shards that start and end in host memory (north_star: recorded beside
        # the device-resident rate): rs16_encode_host / rs16_decode_host on
        # pinned buffers = H2D of the inputs, the same device codec, D2H of
        # the outputs (whole-width slices: narrower pipelined slices measured
        # slower, CHANGELOG.md round 1).
        from rs16.device import PinnedArray

        if extra_on("host_resident"):
            h_orig, h_rec, h_rest = PinnedArray(eng, k * S), PinnedArray(eng, m * S), PinnedArray(eng, k * S)
            h_orig.array[:] = original.reshape(-1)
            h_rest.array[:] = original.reshape(-1)
            h_rest.array.reshape(k, S)[:loss] = 0

            def host_encode():
                rs16.encode_host(k, m, S, h_orig.ptr, h_rec.ptr, engine=eng)

            def host_decode():
                rs16.decode_host(k, m, S, h_rest.ptr, of, h_rec.ptr, rf, engine=eng)

            host_encode()
            host_decode()
            assert np.array_equal(h_rec.array.reshape(m, S), recovery), "host-resident encode differs"
            assert np.array_equal(h_rest.array.reshape(k, S), original), "host-resident decode did not restore"
            n3 = max(3, args.steps // 4)
            te, td = timed(host_encode, n3), timed(host_decode, n3)
            extra["host_resident_pcie"] = {
                "encode_gib_s": world * (k + m) * S * n3 / te / GIB, "decode_gib_s": world * (k + m) * S * n3 / td / GIB,
                "encode_us": te / n3 * 1e6, "decode_us": td / n3 * 1e6,
                "path": "pinned host buffers -> H2D -> device codec -> D2H (rs16_encode_host / rs16_decode_host)"}
            del h_orig, h_rec, h_rest
        if extra_on("host_batch"):
            # Several stripes, two in flight (rs16_encode_host_batch /
            # rs16_decode_host_batch): stripe i + 1's H2D and stripe i - 1's D2H
            # overlap stripe i's codec, so both link directions carry data.  Every
            # stripe holds this stripe's data: each recovery must equal the one
            # checked against the oracle fixture above, each decode restore it.
            nb = 8
            heng = eng
            hb_o, hb_r = PinnedArray(heng, nb * k * S), PinnedArray(heng, nb * m * S)
            hb_o.array.reshape(nb, k * S)[:] = original.reshape(1, -1)
            fob = np.tile(of, nb)
            frb = np.tile(rf, nb)

            def batch_encode():
                rs16.encode_host_batch(k, m, S, nb, hb_o.ptr, k * S, hb_r.ptr, m * S, engine=heng)

            def batch_decode():
                rs16.decode_host_batch(k, m, S, nb, hb_o.ptr, k * S, fob, k, hb_r.ptr, m * S, frb, m, engine=heng)

            batch_encode()
            assert all(np.array_equal(hb_r.array.reshape(nb, m, S)[i], recovery) for i in range(nb)), \
                "pipelined host encode differs"
            hb_o.array.reshape(nb, k, S)[:, :loss] = 0
            batch_decode()
            assert all(np.array_equal(hb_o.array.reshape(nb, k, S)[i], original) for i in range(nb)), \
                "pipelined host decode did not restore"
            # (the first calls after the buffers are created run at a fraction of
            # the rate: scripts/probe_hostbatch.py reps 0-1; two more of each)
            for _ in range(2):
                batch_encode()
                batch_decode()
            n5 = max(4, args.steps // 4)
            tbe = timed(batch_encode, n5)
            tbd = timed(batch_decode, n5)
            extra["host_batch_pipelined"] = {
                "stripes_per_call": nb,
                "encode_gib_s": world * nb * (k + m) * S * n5 / tbe / GIB,
                "decode_gib_s": world * nb * (k + m) * S * n5 / tbd / GIB,
                "encode_ms_per_call": tbe / n5 * 1e3, "decode_ms_per_call": tbd / n5 * 1e3,
                "link_bytes_per_call": {"encode": nb * (k + m) * S, "decode_100pct": nb * (k + loss) * S},
                "path": "pinned host stripes, two in flight: stripe i runs H2D -> codec -> D2H on lane i & 1 (a "
                        "stream with buffers of its own), the lanes half a period apart so that one lane's D2H "
                        "meets the other's H2D (rs16_encode_host_batch / rs16_decode_host_batch, DESIGN.md 3.10); "
                        "every stripe's recovery == the fixture-checked one, every decode restored"}
            del hb_o, hb_r
            # The same calls in a fresh child process (scripts/probe_hostbatch.py,
            # which checks every restored stripe): in this process, after the
            # extras above, they run slower, and not for any cause found so far
            # (NUMA node, streams created before the lanes, an RCCL communicator,
            # the engine's state, GPU clocks after load: CHANGELOG.md round 5)
            if world == 1:
                res = subprocess.run([sys.executable, str(Path(__file__).resolve().parent / "scripts" / "probe_hostbatch.py"),
                                      str(nb), "4"], capture_output=True, text=True, timeout=300)
                last = [ln for ln in res.stdout.splitlines() if ln.startswith("rep 3: encode")]
                if res.returncode == 0 and last and "restored True" in last[0]:
                    ln = last[0]
                    enc = float(ln.split("encode ")[1].split(" GiB/s")[0])
                    dec = float(ln.split("decode ")[1].split(" GiB/s")[0])
                    extra["host_batch_pipelined"]["fresh_process"] = {
                        "encode_gib_s": enc, "decode_gib_s": dec,
                        "note": "4th call of each in a child process (scripts/probe_hostbatch.py, 8 stripes, restored "
                                "checked); the first calls of a process pay buffer setup"}

    if not args.no_extra and world == 1 and extra_on("api_loop"):
        # The reference's own API benchmark (ReedSolomonEncoder / Decoder with
        # per-shard add_* calls on host shards) through the C ABI.
        eng.synchronize()
        extra["api_reference_loop"] = api_reference_loop(S, 0.5)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(original, recovery, k, m, S, args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u16",
            "data": "synthetic (ChaCha8 seed=rank stream of the reference benches; inputs resident in HBM)",
            "config": {"workload": f"{k}:{m} x {S} B encode + 100%-loss decode per GPU" +
                       (" (BASELINE configs[3])" if (k, m, S) == (32768, 32768, 1024) else
                        " (BASELINE configs[1] + [2])" if (k, m, S) == (1000, 1000, 1024) else ""),
                       "original_count": k, "recovery_count": m, "shard_bytes": S,
                       "parallelism": f"independent stripes x {world} (weak, no collective)",
                       "column_slices": args.slices,
                       "decode_issue": ("split: rs16_decode_prepare (eval_poly of the received pattern) on a side "
                                        "stream while the encode runs, then rs16_decode_device_prepared"
                                        if args.split_decode else "serial: rs16_decode_device after the encode")},
            "encode_gib_s": round(world * (k + m) * S * args.steps / dt_e / GIB, 3),
            "decode_gib_s": round(world * (k + m) * S * args.steps / dt_d / GIB, 3),
            "ranks": ranks,
            "roofline": roofline,
            "valu_roofline": valu,
            "cpu_baseline": cpu,
            "kernels_us": {n: round(v["avg_us"], 2) for n, v in kernels.items()},
            "extra": extra,
            "verified": verified,
        }
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
