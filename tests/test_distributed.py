"""Multi-GPU layout on CPU: world-size-2 gloo ranks (no GPU needed).

BASELINE configs[4] partitions the byte columns of every shard across GPUs
(SURVEY.md §8(e)); each rank runs the whole codec on its own slice and there
is no data-path collective.  Here two gloo ranks each encode and decode
their slice (rs16.columns) with the CPU oracle standing in for the device
(test infrastructure), the slices are all-gathered, and the result must equal
the full-width oracle encode / decode bit for bit -- the partition is exact.
The bench's max-over-ranks timing helper is exercised too.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, k, m, S, lost, q):
    for p in (str(ROOT / "reed-solomon-16_amd"), str(ROOT / "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    import oracle_bind as O
    from rs16.columns import gather_columns, max_over_ranks, take_columns
    from rs16.util import generate_original

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = generate_original(k, S, 11)
        mine = take_columns(full, rank, world)
        rec = O.encode(k, m, mine)
        rec_all = gather_columns(rec, world)
        dec = O.Decoder("default", "nosimd", k, m, mine.shape[1])
        for i in range(lost, k):
            dec.add_original_shard(i, mine[i])
        for j in range(lost):
            dec.add_recovery_shard(j, rec[j])
        restored = dec.decode()
        rest_all = gather_columns(np.stack([restored[i] for i in range(lost)]), world)
        t = max_over_ranks(0.25 + rank)
        if rank == 0:
            q.put((np.array_equal(rec_all, O.encode(k, m, full)), np.array_equal(rest_all, full[:lost]), t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("S", [128, 64 * 5])
def test_column_partition_world2(S):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    k, m, lost = 300, 200, 150
    procs = [ctx.Process(target=_worker, args=(r, 2, port, k, m, S, lost, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        enc_ok, dec_ok, t = q.get(timeout=180)
    finally:
        for p in procs:
            p.join(60)
    assert all(p.exitcode == 0 for p in procs)
    assert enc_ok, "gathered column-slice encodes differ from the full-width encode"
    assert dec_ok, "gathered column-slice decodes differ from the originals"
    assert t == 1.25


def test_column_slices():
    from rs16.columns import column_slices, join_columns, take_columns

    assert column_slices(64 * 1024, 8) == [(i * 8192, 8192) for i in range(8)]  # configs[4]: 8 KiB per GPU
    assert column_slices(1024, 8) == [(i * 128, 128) for i in range(8)]
    assert column_slices(64 * 5, 2) == [(0, 192), (192, 128)]
    assert column_slices(64, 2) == [(0, 64), (64, 0)]
    with pytest.raises(ValueError):
        column_slices(100, 2)
    a = np.arange(3 * 320, dtype=np.uint32).astype(np.uint8).reshape(3, 320)
    assert np.array_equal(join_columns([take_columns(a, r, 3) for r in range(3)]), a)


def _root_worker(rank, world, port, k, m, S, q):
    # The data flow of the RCCL path (rs16_comm.cpp) with gloo point-to-point
    # on CPU: rank 0 packs the column slices (rs16_column_slice, the C ABI's
    # partition) into one staging buffer, sends each rank its slice, every
    # rank runs the codec on its slice (the oracle standing in for the
    # device), the root receives the recovery slices into the staging layout
    # and unpacks them.
    for p in (str(ROOT / "reed-solomon-16_amd"), str(ROOT / "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import oracle_bind as O
    import rs16
    from rs16.util import generate_original

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sl = [rs16.column_slice(S, world, r) for r in range(world)]
        off, w = sl[rank]
        mine = torch.zeros(k * w, dtype=torch.uint8)
        if rank == 0:
            full = generate_original(k, S, 12)
            stage = np.empty(k * S, np.uint8)
            for r, (o, wr) in enumerate(sl):
                stage[k * o:k * (o + wr)] = full[:, o:o + wr].reshape(-1)
            for r, (o, wr) in enumerate(sl):
                part = torch.from_numpy(stage[k * o:k * (o + wr)].copy())
                if r == 0:
                    mine = part
                elif wr:
                    dist.send(part, r)
        elif w:
            dist.recv(mine, 0)
        rec = O.encode(k, m, mine.numpy().reshape(k, w)) if w else np.zeros((m, 0), np.uint8)
        if rank == 0:
            stage = np.empty(m * S, np.uint8)
            for r, (o, wr) in enumerate(sl):
                if r == 0:
                    stage[m * o:m * (o + wr)] = rec.reshape(-1)
                elif wr:
                    t = torch.zeros(m * wr, dtype=torch.uint8)
                    dist.recv(t, r)
                    stage[m * o:m * (o + wr)] = t.numpy()
            out = np.empty((m, S), np.uint8)
            for o, wr in sl:
                out[:, o:o + wr] = stage[m * o:m * (o + wr)].reshape(m, wr)
            q.put(bool(np.array_equal(out, O.encode(k, m, full))))
        elif w:
            dist.send(torch.from_numpy(rec.reshape(-1).copy()), 0)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("S,world", [(64 * 5, 2), (128, 3)])
def test_root_scatter_gather_flow(S, world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_root_worker, args=(r, world, port, 200, 100, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        ok = q.get(timeout=180)
    finally:
        for p in procs:
            p.join(60)
    assert all(p.exitcode == 0 for p in procs)
    assert ok, "root scatter -> per-slice encode -> gather differs from the full-width encode"
