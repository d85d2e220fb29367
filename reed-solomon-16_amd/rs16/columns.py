"""Byte-column partitioning of a stripe across GPUs (BASELINE configs[4]).

Every byte column of the shards is an independent codeword: the FFT/IFFT
butterflies, ``mul``/``mul_add`` (inside one 64-byte block,
src/engine/engine_nosimd.rs:65-119), ``xor`` and the formal derivative all act
elementwise across shards at a fixed byte offset, and a 16-bit element's low
and high bytes sit in the same 64-byte block (src/algorithm.md:18-32).  So any
split of ``shard_bytes`` into multiples of 64 gives bit-identical results per
slice, and N GPUs can each run the whole codec on their own slice with no
exchange in the data path.

This module is the host side of that layout: which slice a rank owns, how to
cut and re-assemble host shard arrays, and the control-plane helpers the
multi-process bench uses (``torch.distributed`` only; no GPU collective).
It loads no native code.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

BLOCK = 64


def column_slices(shard_bytes: int, world: int) -> List[Tuple[int, int]]:
    """(offset, width) of every rank's slice: whole 64-byte blocks, as even as
    possible (the first ``blocks % world`` ranks get one block more).  A rank
    may get width 0 when there are fewer blocks than ranks."""
    if shard_bytes <= 0 or shard_bytes % BLOCK:
        raise ValueError("shard_bytes must be a positive multiple of 64")
    if world <= 0:
        raise ValueError("world must be positive")
    blocks = shard_bytes // BLOCK
    base, extra = divmod(blocks, world)
    out, off = [], 0
    for r in range(world):
        w = (base + (1 if r < extra else 0)) * BLOCK
        out.append((off, w))
        off += w
    return out


def column_slice(shard_bytes: int, rank: int, world: int) -> Tuple[int, int]:
    return column_slices(shard_bytes, world)[rank]


def take_columns(shards: np.ndarray, rank: int, world: int) -> np.ndarray:
    """Rank ``rank``'s slice of a (count, shard_bytes) array, contiguous."""
    off, w = column_slice(shards.shape[1], rank, world)
    return np.ascontiguousarray(shards[:, off:off + w])


def join_columns(parts: List[np.ndarray]) -> np.ndarray:
    """Inverse of take_columns over all ranks (parts in rank order)."""
    return np.ascontiguousarray(np.concatenate([p for p in parts if p.shape[1]], axis=1))


def gather_columns(part: np.ndarray, world: int, group=None) -> np.ndarray:
    """All-gather every rank's (count, width_r) slice over torch.distributed
    and join them (control/verification path; widths may differ by 64)."""
    import torch
    import torch.distributed as dist

    count = part.shape[0]
    ws = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(ws, torch.tensor([part.shape[1]], dtype=torch.int64), group=group)
    widths = torch.cat(ws)
    wmax = int(widths.max())
    buf = torch.zeros((count, wmax), dtype=torch.uint8)
    buf[:, :part.shape[1]] = torch.from_numpy(np.ascontiguousarray(part))
    bufs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    return join_columns([b[:, :int(w)].numpy() for b, w in zip(bufs, widths.tolist())])


def max_over_ranks(seconds: float, group=None) -> float:
    """The bench's job time: the slowest rank's (all_reduce MAX)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return float(seconds)
    t = torch.tensor([float(seconds)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
