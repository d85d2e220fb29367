"""The general decode's middle pass as a direct product (rs16_pass.hip
mid_direct_kernel): when the lost originals lie in at most
MID_DIRECT_MAX = 4 of the middle pass's output rows per column, those rows
are computed as sums over the live z rows with the pass's matrix
(mid_matrix_entries) instead of DEC_MID's IFFT / derivative / FFT.  Every
decode must restore the originals bit for bit (src/rate/rate_high.rs:168-247),
with RS16_DIAG_NO_MID_DIRECT (DEC_MID only) as the control: the reference
bench's 1 % loss (benches/benchmarks.rs:81-105), lost originals spanning
1..5 last-pass tiles (5: DEC_MID computes it), several transform sizes,
batched stripes with one pattern and with a pattern each (the kernel decides
per stripe), column slices, the low rate."""
import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu
DIAGS = [0, rs16.DIAG_NO_MID_DIRECT]
IDS = ["direct", "dec_mid"]


@pytest.fixture(scope="module")
def eng():
    e = rs16.Engine(0)
    yield e
    e.close()


def tile_rows(k, m):
    """Rows of a last-pass tile of the general decode (2^lo, lo = L // 2)."""
    chunk = 1 << (m - 1).bit_length()
    n = 2 * chunk
    return 1 << (n.bit_length() - 1) // 2


def masks_clustered(k, m, first_lost, nlost):
    """Originals [first_lost, first_lost + nlost) lost; just enough recovery received."""
    om = np.ones(k, bool)
    om[first_lost:first_lost + nlost] = False
    rm = np.zeros(m, bool)
    rm[:nlost] = True
    return om, rm


def run(eng, k, m, sb, om, rm, diag, seed):
    old = eng.set_diagnostics(diag)
    try:
        original = generate_original(k, sb, seed)
        d_o = DeviceArray.from_numpy(eng, original)
        d_r = DeviceArray(eng, m * sb)
        rs16.encode_device(k, m, sb, d_o.ptr, d_r.ptr, engine=eng)
        held = original.copy()
        held[~om] = 0xA5
        d_x = DeviceArray.from_numpy(eng, held)
        d_fo = DeviceArray.from_numpy(eng, om.astype(np.uint8))
        d_fr = DeviceArray.from_numpy(eng, rm.astype(np.uint8))
        rs16.decode_device(k, m, sb, d_x.ptr, d_fo.ptr, d_r.ptr, d_fr.ptr, int(om.sum()), int(rm.sum()), engine=eng,
                           check=True)
        assert np.array_equal(d_x.download(shape=(k, sb)), original)
    finally:
        eng.set_diagnostics(old)


@pytest.mark.parametrize("diag", DIAGS, ids=IDS)
@pytest.mark.parametrize("sb", [1024, 128])
def test_reference_bench_1pct(eng, sb, diag):
    k = m = 32768
    lost = k // 100
    om, rm = masks_clustered(k, m, k - lost, lost)
    run(eng, k, m, sb, om, rm, diag, 1)


@pytest.mark.parametrize("diag", DIAGS, ids=IDS)
@pytest.mark.parametrize("k,m", [(32768, 32768), (10000, 10000), (4096, 4096), (2500, 2500)])
@pytest.mark.parametrize("tiles", [1, 2, 3, 4, 5])
def test_lost_span(eng, k, m, tiles, diag):
    # lost originals spanning `tiles` last-pass tiles (the high rate's
    # originals start at row chunk, a multiple of the tile)
    tr = tile_rows(k, m)
    nlost = min(k, m, (tiles - 1) * tr + 3)
    first = min(k - nlost, tr - 2) if tiles > 1 else min(k - nlost, 5)
    om, rm = masks_clustered(k, m, first, nlost)
    run(eng, k, m, 64, om, rm, diag, tiles)


@pytest.mark.parametrize("diag", DIAGS, ids=IDS)
def test_low_rate(diag):
    # RateDecoder with the low rate: originals are segment A, recovery B
    k, m, sb = 3000, 30000, 64
    original = generate_original(k, sb, 7)
    recovery = O.encode(k, m, original, rate="low")
    lost = list(range(2000, 2040))
    eng = rs16.default_engine()
    old = eng.set_diagnostics(diag)
    try:
        dec = rs16.RateDecoder(k, m, sb, "low")
        for i in range(k):
            if i not in lost:
                dec.add_original_shard(i, original[i])
        for i in range(len(lost)):
            dec.add_recovery_shard(100 + i, recovery[100 + i])
        with dec.decode() as res:
            got = dict(res.restored_original_iter())
        assert sorted(got) == lost
        assert all(got[i] == original[i].tobytes() for i in lost)
    finally:
        eng.set_diagnostics(old)


@pytest.mark.parametrize("diag", DIAGS, ids=IDS)
def test_batched_shared_pattern(eng, diag):
    k = m = 8192
    n, sb = 3, 128
    old = eng.set_diagnostics(diag)
    try:
        stripes = [generate_original(k, sb, 50 + i) for i in range(n)]
        host_o = np.concatenate([s.reshape(-1) for s in stripes])
        d_o = DeviceArray.from_numpy(eng, host_o)
        d_r = DeviceArray(eng, n * m * sb)
        rs16.encode_device_batch(k, m, sb, n, d_o.ptr, k * sb, d_r.ptr, m * sb, engine=eng)
        om, rm = masks_clustered(k, m, k - 100, 100)
        held = host_o.copy().reshape(n, k, sb)
        held[:, ~om] = 0x11
        d_x = DeviceArray.from_numpy(eng, held.reshape(-1))
        d_fo = DeviceArray.from_numpy(eng, om.astype(np.uint8))
        d_fr = DeviceArray.from_numpy(eng, rm.astype(np.uint8))
        rs16.decode_device_batch(k, m, sb, n, d_x.ptr, k * sb, d_fo.ptr, d_r.ptr, m * sb, d_fr.ptr, int(om.sum()),
                                 int(rm.sum()), engine=eng)
        assert np.array_equal(d_x.download(shape=(n * k * sb,)), host_o)
    finally:
        eng.set_diagnostics(old)


@pytest.mark.parametrize("diag", DIAGS, ids=IDS)
def test_batched_varied_patterns(eng, diag):
    # stripe 0 and 2 clustered (direct), stripe 1 spread (DEC_MID), stripe 3 clustered over 5 tiles
    k = m = 4096
    sb = 64
    tr = tile_rows(k, m)
    rng = np.random.default_rng(3)
    pats = []
    for i, kind in enumerate(["cluster", "spread", "cluster", "wide"]):
        if kind == "cluster":
            om, rm = masks_clustered(k, m, 17 * (i + 1), 40)
        elif kind == "wide":
            om, rm = masks_clustered(k, m, 0, 4 * tr + 10)
        else:
            om = np.ones(k, bool)
            om[rng.choice(k, 300, replace=False)] = False
            rm = np.zeros(m, bool)
            rm[rng.choice(m, 300, replace=False)] = True
        pats.append((om, rm))
    n = len(pats)
    old = eng.set_diagnostics(diag)
    try:
        stripes = [generate_original(k, sb, 70 + i) for i in range(n)]
        host_o = np.zeros((n, k, sb), np.uint8)
        host_r = np.zeros((n, m, sb), np.uint8)
        fo = np.zeros((n, k), np.uint8)
        fr = np.zeros((n, m), np.uint8)
        for i, (om, rm) in enumerate(pats):
            host_o[i] = stripes[i]
            host_o[i][~om] = 0x5A
            host_r[i] = O.encode(k, m, stripes[i])
            fo[i], fr[i] = om, rm
        d_o, d_r = DeviceArray.from_numpy(eng, host_o.reshape(-1)), DeviceArray.from_numpy(eng, host_r.reshape(-1))
        d_fo, d_fr = DeviceArray.from_numpy(eng, fo.reshape(-1)), DeviceArray.from_numpy(eng, fr.reshape(-1))
        oc = [int(p[0].sum()) for p in pats]
        rc = [int(p[1].sum()) for p in pats]
        rs16.decode_device_batch_varied(k, m, sb, n, d_o.ptr, k * sb, d_fo.ptr, k, d_r.ptr, m * sb, d_fr.ptr, m, oc, rc,
                                        engine=eng)
        got = d_o.download(shape=(n, k, sb))
        for i in range(n):
            assert np.array_equal(got[i], stripes[i]), i
    finally:
        eng.set_diagnostics(old)


def test_slices(eng):
    k = m = 16384
    sb = 192
    eng.set_slices(3)
    try:
        om, rm = masks_clustered(k, m, 16000, 300)
        run(eng, k, m, sb, om, rm, 0, 9)
    finally:
        eng.set_slices(1)


def masks_span(k, m, span_tiles, nlost, seed, tr=256):
    """nlost originals lost, scattered over the last `span_tiles` 256-row
    tiles of the originals (first and last of them lost); as many random
    recovery shards received."""
    rng = np.random.default_rng(seed)
    lo = max(0, k - span_tiles * tr)
    om = np.ones(k, bool)
    om[rng.choice(np.arange(lo, k), min(nlost, k - lo), replace=False)] = False
    om[lo] = om[k - 1] = False
    rm = np.zeros(m, bool)
    rm[rng.choice(m, int((~om).sum()), replace=False)] = True
    return om, rm


@pytest.mark.parametrize("diag", [0, rs16.DIAG_TILE_LAST, rs16.DIAG_NO_TILE_LAST], ids=["auto", "tile_last", "items"])
@pytest.mark.parametrize("span", [1, 15, 16, 17, 40, 128])
def test_last_pass_choice_by_span(eng, span, diag):
    """The general decode's last pass at 2^16 work rows: tile_last_kernel for
    lost originals spanning <= TILE_LAST_MAX = 16 tiles, the 8-wave DEC_LAST
    items beyond (decided on the device from the lost range: both launch,
    each returns where the other applies).  Scattered losses over 1..128
    tiles, each form forced as the control."""
    k = m = 32768
    om, rm = masks_span(k, m, span, 300, span)
    run(eng, k, m, 128, om, rm, diag, span)


def test_last_pass_choice_batched_varied(eng):
    """Stripes of one call whose lost ranges fall on either side of the cut
    (the kernels decide per stripe)."""
    k = m = 32768
    sb, ns = 64, 3
    spans = [2, 40, 16]
    origs = [generate_original(k, sb, 50 + i) for i in range(ns)]
    recs = [O.encode(k, m, o) for o in origs]
    oms, rms = zip(*[masks_span(k, m, s, 200, 60 + i) for i, s in enumerate(spans)])
    held = np.stack(origs)
    for i in range(ns):
        held[i][~oms[i]] = 0x5C
    d_x = DeviceArray.from_numpy(eng, held.reshape(-1))
    d_r = DeviceArray.from_numpy(eng, np.stack(recs).reshape(-1))
    d_fo = DeviceArray.from_numpy(eng, np.stack(oms).astype(np.uint8).reshape(-1))
    d_fr = DeviceArray.from_numpy(eng, np.stack(rms).astype(np.uint8).reshape(-1))
    rs16.decode_device_batch_varied(k, m, sb, ns, d_x.ptr, k * sb, d_fo.ptr, k, d_r.ptr, m * sb, d_fr.ptr, m,
                                    [int(o.sum()) for o in oms], [int(r.sum()) for r in rms], engine=eng)
    back = d_x.download(shape=(ns, k, sb))
    for i in range(ns):
        assert np.array_equal(back[i], origs[i]), spans[i]
