"""Several engines in one process (include/rs16.h "Several GPUs in one
process"): one stripe's byte columns split over n engines, each copying its
column slice in and out with pitched DMA copies (every 64-byte
column block is an independent codeword, src/algorithm.md:18-32).  The GPU
box has one GPU, so the n engines here share device 0: the partition logic,
the per-engine buffers and streams are the same as with one GPU per engine.
Checked against the oracle bit for bit, including n larger than the number
of column blocks (engines with an empty slice)."""
import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.util import generate_original

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engines():
    es = [rs16.Engine(0) for _ in range(4)]
    yield es
    for e in es:
        e.close()


@pytest.mark.parametrize("n", [1, 2, 3, 4])
@pytest.mark.parametrize("k,m,sb", [(1000, 1000, 1024), (4096, 4096, 192), (100, 300, 64), (3000, 1000, 512)])
def test_multi_engine_roundtrip(engines, n, k, m, sb):
    es = engines[:n]
    original = generate_original(k, sb, n + k)
    want = O.encode(k, m, original)
    rec = np.zeros((m, sb), np.uint8)
    rs16.encode_host_multi(k, m, sb, original, rec, es)
    assert np.array_equal(rec, want)
    rng = np.random.default_rng(n * 7 + k)
    for loss in (min(k, m), max(1, min(k, m) // 100)):
        lost = rng.choice(k, loss, replace=False)
        of = np.ones(k, np.uint8)
        of[lost] = 0
        rf = np.zeros(m, np.uint8)
        rf[rng.choice(m, loss, replace=False)] = 1
        holes = original.copy()
        holes[lost] = 0xA5
        rs16.decode_host_multi(k, m, sb, holes, of, rec, rf, es)
        assert np.array_equal(holes, original), loss
