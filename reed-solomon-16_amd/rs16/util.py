"""Reference-compatible synthetic shard generation.

The reference generates every test and benchmark input with
``ChaCha8Rng::from_seed([seed; 32])`` followed by ``rng.fill(shard)`` for each
shard in order (``src/test_util.rs:77-88``, ``benches/benchmarks.rs:21-28``;
rand 0.8.4 / rand_chacha 0.3.1).  That stream is DJB ChaCha with 8 rounds,
key = 32 bytes of ``seed``, a 64-bit block counter starting at 0, a zero
64-bit stream id, and the 16 output words of each block emitted
little-endian.  Shards are multiples of 64 bytes, so no partial word is ever
discarded and the shards are simply consecutive slices of one stream.

This module is a vectorised numpy restatement of that generator so that GPU
tests and the bench use exactly the reference's inputs (golden hashes in
``tests/golden`` pin it).  It is input tooling, not the codec.
"""
from __future__ import annotations

import numpy as np

_CONST = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], dtype=np.uint32)


def _rotl(x: np.ndarray, n: int) -> np.ndarray:
    return (x << np.uint32(n)) | (x >> np.uint32(32 - n))


def chacha8_stream(seed: int, nbytes: int) -> np.ndarray:
    """Return the first ``nbytes`` of ChaCha8Rng::from_seed([seed; 32])."""
    if nbytes % 64:
        raise ValueError("nbytes must be a multiple of 64")
    nblocks = nbytes // 64
    key_word = np.uint32((seed & 0xFF) * 0x01010101)
    ctr = np.arange(nblocks, dtype=np.uint64)
    init = np.empty((16, nblocks), dtype=np.uint32)
    init[0:4] = _CONST[:, None]
    init[4:12] = key_word
    init[12] = (ctr & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    init[13] = (ctr >> np.uint64(32)).astype(np.uint32)
    init[14] = 0
    init[15] = 0
    x = [init[i].copy() for i in range(16)]

    def qr(a, b, c, d):
        x[a] += x[b]; x[d] ^= x[a]; x[d] = _rotl(x[d], 16)
        x[c] += x[d]; x[b] ^= x[c]; x[b] = _rotl(x[b], 12)
        x[a] += x[b]; x[d] ^= x[a]; x[d] = _rotl(x[d], 8)
        x[c] += x[d]; x[b] ^= x[c]; x[b] = _rotl(x[b], 7)

    with np.errstate(over="ignore"):
        for _ in range(4):  # 8 rounds = 4 double rounds
            qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
            qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
        out = np.stack([x[i] + init[i] for i in range(16)], axis=1)  # (nblocks, 16)
    return out.astype("<u4").view(np.uint8).reshape(-1)


def generate_original(count: int, shard_bytes: int, seed: int) -> np.ndarray:
    """``test_util::generate_original`` / ``benches::generate_shards``:
    ``count`` shards of ``shard_bytes`` as a (count, shard_bytes) uint8 array."""
    return chacha8_stream(seed, count * shard_bytes).reshape(count, shard_bytes)
