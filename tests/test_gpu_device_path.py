"""GPU parity of the device-resident one-shot path (the benchmark path) at
BASELINE.json's configurations, against the oracle (same ChaCha8 inputs as
benches/benchmarks.rs:21-28, seed 0) and the oracle-generated SHA-256
fixtures in tests/golden/kib_hashes.json; full-size properties: decode after
erasure restores every lost original bit-exactly, for 100 %, 1 % and random
loss patterns, both rates, single- and multi-chunk.
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu
KIB = {(c["k"], c["m"]): c for c in json.loads((Path(__file__).parent / "golden" / "kib_hashes.json").read_text())["cases"]}


@pytest.fixture(scope="module")
def eng():
    return rs16.default_engine()


def dev_encode(eng, original, m):
    k, sb = original.shape
    d_orig = DeviceArray.from_numpy(eng, original)
    d_rec = DeviceArray(eng, m * sb)
    rs16.encode_device(k, m, sb, d_orig.ptr, d_rec.ptr, engine=eng)
    return d_rec.download(shape=(m, sb))


def dev_decode(eng, original, recovery, orig_mask, rec_mask):
    k, sb = original.shape
    m = recovery.shape[0]
    holes = original.copy()
    holes[~orig_mask] = 0xA5  # garbage in lost slots must not matter
    d_orig = DeviceArray.from_numpy(eng, holes)
    d_rec = DeviceArray.from_numpy(eng, recovery)
    d_of = DeviceArray.from_numpy(eng, orig_mask.astype(np.uint8))
    d_rf = DeviceArray.from_numpy(eng, rec_mask.astype(np.uint8))
    rs16.decode_device(k, m, sb, d_orig.ptr, d_of.ptr, d_rec.ptr, d_rf.ptr, int(orig_mask.sum()),
                       int(rec_mask.sum()), engine=eng)
    return d_orig.download(shape=(k, sb))


@pytest.mark.parametrize("k,m", [(100, 100), (1000, 1000), (32768, 32768)])
def test_baseline_configs_encode_decode(eng, k, m):
    original = generate_original(k, 1024, 0)
    recovery = dev_encode(eng, original, m)
    assert hashlib.sha256(recovery.tobytes()).hexdigest() == KIB[(k, m)]["recovery_sha256"]
    # 100 % original loss: recovery 0..k given (benches/benchmarks.rs:82-87 with loss = min(k, m))
    loss = min(k, m)
    om = np.ones(k, bool)
    om[:loss] = False
    rm = np.zeros(m, bool)
    rm[:loss] = True
    restored = dev_decode(eng, original, recovery, om, rm)
    assert np.array_equal(restored, original)
    # 1 % loss
    loss = min(k, m) // 100
    if loss:
        om = np.ones(k, bool)
        om[k - loss:] = False
        rm = np.zeros(m, bool)
        rm[:loss] = True
        assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


@pytest.mark.parametrize("k,m", [(1, 1), (2, 1), (3, 5), (100, 1000), (1000, 100), (1025, 1024), (1024, 1025),
                                 (2048, 1025), (4096, 61440), (61440, 4096)])
def test_device_path_vs_oracle(eng, k, m):
    sb = 128 if k * m > 10**7 else 1024
    original = generate_original(k, sb, k % 251)
    recovery = dev_encode(eng, original, m)
    want = O.encode(k, m, original)
    assert np.array_equal(recovery, want)
    rng = np.random.default_rng(k * 7 + m)
    # random erasures: keep exactly k of the k+m shards
    keep = rng.permutation(k + m)[:k]
    om = np.zeros(k, bool)
    rm = np.zeros(m, bool)
    om[keep[keep < k]] = True
    rm[keep[keep >= k] - k] = True
    assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


def test_decode_nothing_to_do_and_not_enough(eng):
    original = generate_original(4, 64, 1)
    recovery = dev_encode(eng, original, 2)
    out = dev_decode(eng, original, recovery, np.ones(4, bool), np.zeros(2, bool))
    assert np.array_equal(out, original)
    with pytest.raises(rs16.Error) as e:
        dev_decode(eng, original, recovery, np.array([1, 0, 0, 1], bool), np.array([1, 0], bool))
    assert e.value == rs16.Error("NotEnoughShards", original_count=4, original_received_count=2,
                                 recovery_received_count=1)


@pytest.mark.parametrize("k,m,sb", [(32768, 32768, 64), (1000, 1000, 64 * 3), (300, 300, 64 * 9),
                                    (100, 100, 65536 + 192), (300, 600, 65536 + 192)])
def test_odd_shard_widths(eng, k, m, sb):
    # shard widths that are not a multiple of the 512-byte tile slab; rows
    # wider than the 64 KiB zero page (the lanes past the last partial slab
    # read from it at their in-row offset, masked into the page)
    original = generate_original(k, sb, 5)
    recovery = dev_encode(eng, original, m)
    assert np.array_equal(recovery, O.encode(k, m, original))
    om = np.zeros(k, bool)
    om[::3] = True
    rm = np.zeros(m, bool)
    rm[: k - om.sum()] = True
    assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


def loss_masks(k, m, pattern):
    """Received masks for the zero-tile cases: 'all' = every original lost
    (min(k, m) of them, as benches/benchmarks.rs:82-87 at 100 %); 'blocks' =
    originals lost in aligned 256-shard blocks, every other block."""
    om = np.ones(k, bool)
    if pattern == "all":
        om[:min(k, m)] = False
    else:
        for b in range(0, k, 512):
            om[b:b + 256] = False
    lost = int((~om).sum())
    assert lost <= m
    rm = np.zeros(m, bool)
    rm[:lost] = True
    return om, rm


@pytest.mark.parametrize("k,m,sb,pattern", [
    (32768, 32768, 64, "blocks"),  # 256-row DEC_FIRST tiles: zero tiles between live ones, whole zero 16-tile blocks
    (4096, 4096, 128, "blocks"),   # 64-row DEC_FIRST tiles, T = 7 DEC_MID
    (1000, 3000, 1024, "all"),     # low rate: zero prefix of the decode work
    (3000, 30000, 64, "all"),      # low rate, n = 65536: a whole zero 16-tile block at the start
    (30000, 3000, 64, "all"),      # high rate, k > m: zero tiles from lost originals and from the zero tail
])
def test_decode_zero_tiles(eng, k, m, sb, pattern):
    # DEC_FIRST tiles without a received row are skipped and read back as
    # zero by DEC_MID / DEC_LAST (rs16_pass.hip); restoration must be exact.
    original = generate_original(k, sb, 11)
    recovery = dev_encode(eng, original, m)
    assert np.array_equal(recovery, O.encode(k, m, original))
    om, rm = loss_masks(k, m, pattern)
    assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


def test_rate_decoder_zero_tiles():
    # Same through the work-buffer decoder (src/rate/decoder_work.rs), where the
    # first pass works in place on the work buffer and skipped tiles keep stale rows.
    k = m = 4096
    sb = 128
    original = generate_original(k, sb, 12)
    enc = rs16.RateEncoder(k, m, sb, "high")
    for s in original:
        enc.add_original_shard(s)
    with enc.encode() as r:
        recovery = list(r.recovery_iter())
    dec = rs16.RateDecoder(k, m, sb, "high")
    for rnd in range(2):  # second round reuses the work buffer (stale data in lost slots)
        om, rm = loss_masks(k, m, "blocks" if rnd == 0 else "all")
        for i in np.flatnonzero(om):
            dec.add_original_shard(int(i), original[i])
        for i in np.flatnonzero(rm):
            dec.add_recovery_shard(int(i), recovery[i])
        with dec.decode() as res:
            restored = dict(res.restored_original_iter())
        assert set(restored) == set(np.flatnonzero(~om).tolist())
        for i, v in restored.items():
            assert v == original[i].tobytes(), i


def test_configs4_per_gpu_column_slice(eng):
    # BASELINE configs[4]: 32768:32768 x 64 KiB over 8 GPUs = 8 KiB of every
    # shard per GPU (rs16/columns.py).  Full-size parity by column
    # independence: two 1 KiB column slices of the 8 KiB device encode equal
    # the oracle's encode of those slices alone; 100 % loss decode restores all.
    k = m = 32768
    sb = 64 * 1024 // 8
    original = np.random.default_rng(4).integers(0, 256, (k, sb), dtype=np.uint8)
    recovery = dev_encode(eng, original, m)
    for c0 in (0, sb - 1024):
        want = O.encode(k, m, np.ascontiguousarray(original[:, c0:c0 + 1024]))
        assert np.array_equal(recovery[:, c0:c0 + 1024], want), c0
    om = np.zeros(k, bool)
    rm = np.ones(m, bool)
    assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


@pytest.mark.parametrize("slices", [1, 2, 3, 4])
@pytest.mark.parametrize("k,m,sb", [(1000, 1000, 192), (3000, 3000, 1024), (100, 200, 320)])
def test_column_slices(eng, slices, k, m, sb):
    # the device one-shot codec split into concurrent column slices
    # (rs16_engine_set_slices): identical results for any slice count,
    # including widths that do not divide evenly into 64-byte blocks
    eng.set_slices(slices)
    try:
        original = generate_original(k, sb, slices)
        recovery = dev_encode(eng, original, m)
        assert np.array_equal(recovery, O.encode(k, m, original))
        om = np.zeros(k, bool)
        om[: k // 3] = True
        rm = np.zeros(m, bool)
        rm[: k - k // 3] = True
        assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)
        om[:] = False
        rm[:] = False
        rm[m - k:] = True  # 100 % loss: the half-transform path
        assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)
    finally:
        eng.set_slices(1)


def lost_pattern(k, m, pattern):
    """Received masks whose lost originals sit in one part of the originals'
    segment; recovery 0..lost given."""
    om = np.ones(k, bool)
    if pattern == "tail":      # benches/benchmarks.rs:84-87 (1 %): the last L originals
        om[k - max(1, min(k, m) // 100):] = False
    elif pattern == "head":
        om[:3] = False
    elif pattern == "two":     # the range spans (almost) the whole segment
        om[[1, k - 2]] = False
    elif pattern == "one_mid":
        om[k // 2 + 5] = False
    elif pattern == "edge":    # across a 256-row block boundary
        om[250:262] = False
    lost = int((~om).sum())
    rm = np.zeros(m, bool)
    rm[:lost] = True
    return om, rm


@pytest.mark.parametrize("pattern", ["tail", "head", "two", "one_mid", "edge"])
@pytest.mark.parametrize("k,m,sb", [(32768, 32768, 64), (4096, 4096, 128), (2000, 2000, 64), (1000, 1000, 1024),
                                    (3000, 30000, 64), (30000, 3000, 64), (700, 300, 128)])
def test_decode_lost_range_pruning(eng, k, m, sb, pattern):
    # The general decode prunes DEC_MID's FFT / stores and DEC_LAST's tiles to
    # the lost originals' row range computed on the device by the eval_poly
    # kernels (rs16_misc.hip lost_part_wave / lost_range_wave, eval_small);
    # every lost original must still come back bit-exactly, and received
    # originals must stay untouched.
    original = generate_original(k, sb, 13)
    recovery = dev_encode(eng, original, m)
    om, rm = lost_pattern(k, m, pattern)
    assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)


@pytest.mark.parametrize("path", ["tile", "items"])
@pytest.mark.parametrize("k,m,sb,pattern", [
    (32768, 32768, 1024, "tail"),      # the reference bench's 1 % loss (benches/benchmarks.rs:84-87)
    (32768, 32768, 64 * 5, "two"),     # partial 64-byte blocks of a workgroup's 4 quad columns
    (32768, 32768, 64, "edge"),
    (30000, 3000, 192, "tail"),        # high rate, k > m (a zero tail in the decode work)
    (3000, 30000, 64, "one_mid"),      # low rate: originals are segment A
    (32768, 32768, 128, "blocks"),     # zero DEC_FIRST tiles next to tiles with lost originals
    (32768, 32768, 64, "scatter"),     # every tile holds lost originals
])
def test_decode_last_pass_paths(eng, k, m, sb, pattern, path):
    # The general decode's last pass over 65536 work rows in both forms: one
    # wave per quad column of a tile (tile_last_kernel, the default for few
    # lost originals) and 8-wave items of 32 quad columns -- forced here
    # either way for every pattern; bit-exact restoration, received
    # originals untouched
    original = generate_original(k, sb, 17)
    recovery = dev_encode(eng, original, m)
    if pattern == "blocks":
        om, rm = loss_masks(k, m, "blocks")
    elif pattern == "scatter":
        om = np.ones(k, bool)
        om[np.random.default_rng(5).choice(k, min(k, m) // 2, replace=False)] = False
        rm = np.zeros(m, bool)
        rm[:int((~om).sum())] = True
    else:
        om, rm = lost_pattern(k, m, pattern)
    old = rs16.set_diagnostics(rs16.DIAG_TILE_LAST if path == "tile" else rs16.DIAG_NO_TILE_LAST)
    try:
        assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)
    finally:
        rs16.set_diagnostics(old)


@pytest.mark.parametrize("fd", ["split", "lds"])
@pytest.mark.parametrize("k,m,sb,diag,lost", [
    # DEC_MID T = 8 (65536 work rows): a layout-B register row = 4096 originals
    (32768, 32768, 64, 0, list(range(4090, 4102))),   # across a register-row boundary
    (32768, 32768, 64, 0, [0, 8000]),                 # two adjacent register rows, sparse
    (32768, 32768, 128, 0, [5000, 5001]),
    (32768, 32768, 64, 0, [0, 12288]),                # three register rows: the LDS derivative
    (32768, 32768, 64, 0, list(range(32768 - 327, 32768))),  # benches/benchmarks.rs:84-87, 1 %
    # T = 7 (8192 work rows): register row = 512 originals
    (4096, 4096, 128, 0, list(range(508, 516))),
    (4096, 4096, 64, 0, [0, 1000]),
    (4096, 4096, 64, 0, [0, 1100]),
    # T = 6 (4096 work rows): register row = 256 originals
    (2000, 2000, 64, 0, list(range(250, 261))),
    (2000, 2000, 64, 0, [0, 300]),
    (2000, 2000, 64, 0, [0, 600]),
    # T = 5 through the pass codec (2^10 work rows): register row = 128 originals
    (500, 500, 64, 8, list(range(120, 131))),
    (500, 500, 64, 8, [0, 200]),
    (500, 500, 64, 8, [0, 300]),
    # high / low rate with a zero tail / zero prefix in the work
    (30000, 3000, 64, 0, [10, 20, 4095, 4096]),
    (3000, 30000, 64, 0, list(range(250, 261))),
])
def test_decode_split_formal_derivative(eng, k, m, sb, diag, lost, fd):
    # DEC_MID's in-tile formal derivative split by row bits (fd_regs /
    # fd_image, rs16_pass.hip) when the consumed tile rows lie in two
    # layout-B register rows, else through the LDS image; DIAG_FD_LDS forces
    # the LDS form everywhere.  Both restore the lost originals bit-exactly.
    original = generate_original(k, sb, 19)
    recovery = dev_encode(eng, original, m)
    om = np.ones(k, bool)
    om[lost] = False
    rm = np.zeros(m, bool)
    rm[:len(lost)] = True
    old = rs16.set_diagnostics(diag | (rs16.DIAG_FD_LDS if fd == "lds" else 0))
    try:
        assert np.array_equal(dev_decode(eng, original, recovery, om, rm), original)
    finally:
        rs16.set_diagnostics(old)
