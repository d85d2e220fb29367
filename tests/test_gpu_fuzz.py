"""Random round trips on the GPU, after examples/test-random-roundtrips.rs:72-256,
widened to the engine's size-dependent dispatch.

The reference fuzzer's rules are kept: original / recovery counts
log-uniform up to the GF_ORDER limit (:101-116), loss count =
recovery_count half the time, else uniform in 1..=recovery_count
(:118-123), loss positions sampled over originals + recovery (:125-128),
DefaultRate plus HighRate / LowRate where supported (:137-174) with reused
coders (:144-145, via reset).  Recovery shards must equal the oracle's (the
reference checks Naive == NoSimd), restored originals the inputs.

On top of that every case draws what this engine's path choice depends on:
  * the shard width: 64 .. 8192 bytes in 64-byte steps, non-powers of two
    included (bounded so that one case moves at most a few MiB), which moves
    it across col_ok / col_max_quads (rs16_engine.cpp) and the pass codec's
    slab count;
  * the entry point: the Rate API, the device one-shot codec with 1-4 column
    slices (rs16_engine_set_slices), the batched codec with one shared loss
    pattern, and the batched decode with a loss pattern per stripe, with
    random stripe counts;
  * the engine's diagnostic switches (rs16_engine_set_diagnostics), each on
    with probability 0.15: forced column / pass codec, radix-4 column form,
    64-bit lane offsets, the eval_poly forms, the last-pass forms, the
    formal derivative through LDS, the evaluated erasure logs of whole-half erasures.
Every case's parameters are in the assertion message.
"""
import os

import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray

pytestmark = pytest.mark.gpu
GF_ORDER = 65536
DIAGS = (rs16.DIAG_FORCE_VOFF64, rs16.DIAG_EVAL_TWO_KERNEL, rs16.DIAG_EVAL_FULL, rs16.DIAG_NO_COLUMN,
         rs16.DIAG_FORCE_COLUMN, rs16.DIAG_TILE_LAST, rs16.DIAG_NO_TILE_LAST, rs16.DIAG_FD_LDS,
         rs16.DIAG_COL_RADIX4, rs16.DIAG_NO_IDENTITY, rs16.DIAG_NO_MID_DIRECT)
BUDGET = 3 << 20  # bytes of originals + recovery per case (all stripes)
# soak runs (not the default suite): RS16_FUZZ_SEED shifts every test's seed,
# RS16_FUZZ_MULT multiplies its case count
SEED = int(os.environ.get("RS16_FUZZ_SEED", "0"))
MULT = max(1, int(os.environ.get("RS16_FUZZ_MULT", "1")))


def next_pow2(x):
    return 1 << (x - 1).bit_length()


def random_counts(rng):
    while True:
        k = int(2.0 ** rng.uniform(0.0, 16.0))
        m = int(2.0 ** rng.uniform(0.0, 16.0))
        if next_pow2(min(k, m)) + max(k, m) <= GF_ORDER:
            return k, m


def random_width(rng, rows):
    """64 .. 8192 bytes in 64-byte steps, at most BUDGET / rows."""
    most = max(1, min(128, BUDGET // (64 * rows)))
    return 64 * int(rng.integers(1, most + 1))


def random_loss(rng, k, m):
    """Lost positions over originals + recovery (:118-128): (orig_lost, rec_lost) masks."""
    loss = m if rng.random() < 0.5 else int(rng.integers(1, m + 1))
    lost = np.zeros(k + m, bool)
    lost[rng.choice(k + m, size=loss, replace=False)] = True
    return lost[:k], lost[k:]


def random_diag(rng):
    flags = 0
    for f in DIAGS:
        if rng.random() < 0.15:
            flags |= f
    return flags


def random_data(rng, rows, sb):
    return rng.integers(0, 256, (rows, sb), dtype=np.uint8)


@pytest.fixture(scope="module")
def eng():
    e = rs16.Engine(0)
    yield e
    e.close()


def test_random_rate_api(eng):
    """The Rate API (ReedSolomonEncoder / Decoder and the forced rates) with
    coders reused across cases, random widths and switches: 60 cases."""
    rng = np.random.default_rng(20240611 + SEED)
    coders = {}
    for case in range(60 * MULT):
        k, m = random_counts(rng)
        sb = random_width(rng, k + m)
        diag = random_diag(rng)
        eng.set_diagnostics(diag)
        original = random_data(rng, k, sb)
        o_lost, r_lost = random_loss(rng, k, m)
        for rate in ("default", "high", "low"):
            if rate != "default" and not rs16.supports(k, m, rate):
                continue
            why = (case, rate, k, m, sb, hex(diag))
            if rate not in coders:
                coders[rate] = (rs16.RateEncoder(1, 1, 64, rate, engine=eng), rs16.RateDecoder(1, 1, 64, rate, engine=eng))
            enc, dec = coders[rate]
            enc.reset(k, m, sb)
            for s in original:
                enc.add_original_shard(s)
            with enc.encode() as res:
                recovery = list(res.recovery_iter())
            want = O.encode(k, m, original, rate=rate)
            assert b"".join(recovery) == want.tobytes(), why
            dec.reset(k, m, sb)
            for i in np.flatnonzero(~o_lost):
                dec.add_original_shard(int(i), original[i])
            for i in np.flatnonzero(~r_lost):
                dec.add_recovery_shard(int(i), recovery[i])
            with dec.decode() as res:
                restored = dict(res.restored_original_iter())
            assert set(restored) == set(np.flatnonzero(o_lost).tolist()), why
            for i, v in restored.items():
                assert v == original[i].tobytes(), why + (i,)
    eng.set_diagnostics(0)


def _decode_masks(eng, k, m, o_lost, r_lost):
    return (DeviceArray.from_numpy(eng, (~o_lost).astype(np.uint8)),
            DeviceArray.from_numpy(eng, (~r_lost).astype(np.uint8)))


def test_random_device_oneshot(eng):
    """rs16_encode_device / rs16_decode_device with 1-4 column slices:
    80 cases, lost slots holding garbage."""
    rng = np.random.default_rng(7_000_001 + SEED)
    for case in range(80 * MULT):
        k, m = random_counts(rng)
        sb = random_width(rng, k + m)
        diag = random_diag(rng)
        slices = int(rng.integers(1, 5))
        eng.set_diagnostics(diag)
        eng.set_slices(slices)
        why = (case, k, m, sb, hex(diag), slices)
        original = random_data(rng, k, sb)
        d_o = DeviceArray.from_numpy(eng, original)
        d_r = DeviceArray.from_numpy(eng, np.full((m, sb), 0x5A, np.uint8))
        rs16.encode_device(k, m, sb, d_o.ptr, d_r.ptr, engine=eng)
        rec = d_r.download(shape=(m, sb))
        assert np.array_equal(rec, O.encode(k, m, original)), why
        o_lost, r_lost = random_loss(rng, k, m)
        held = original.copy()
        held[o_lost] = 0xA5
        rec_held = rec.copy()
        rec_held[r_lost] = 0x3C
        d_x, d_rr = DeviceArray.from_numpy(eng, held), DeviceArray.from_numpy(eng, rec_held)
        d_fo, d_fr = _decode_masks(eng, k, m, o_lost, r_lost)
        rs16.decode_device(k, m, sb, d_x.ptr, d_fo.ptr, d_rr.ptr, d_fr.ptr, int((~o_lost).sum()),
                           int((~r_lost).sum()), engine=eng, check=True)
        assert np.array_equal(d_x.download(shape=(k, sb)), original), why
        assert np.array_equal(d_rr.download(shape=(m, sb)), rec_held), why  # recovery untouched
    eng.set_slices(1)
    eng.set_diagnostics(0)


def test_random_batches(eng):
    """rs16_encode_device_batch + rs16_decode_device_batch (one shared loss
    pattern): 2-12 stripes with gaps between them, 40 cases."""
    rng = np.random.default_rng(31_337 + SEED)
    for case in range(40 * MULT):
        k, m = random_counts(rng)
        n = int(rng.integers(2, 13))
        sb = 64 * int(rng.integers(1, max(1, min(128, BUDGET // (64 * (k + m) * n))) + 1))
        diag = random_diag(rng)
        eng.set_diagnostics(diag)
        why = (case, k, m, sb, n, hex(diag))
        pad = 64 * int(rng.integers(0, 3))
        so, sr = k * sb + pad, m * sb + pad
        stripes = [random_data(rng, k, sb) for _ in range(n)]
        host_o = np.full(n * so, 0xEE, np.uint8)
        for i, o in enumerate(stripes):
            host_o[i * so:i * so + k * sb] = o.reshape(-1)
        d_o = DeviceArray.from_numpy(eng, host_o)
        d_r = DeviceArray.from_numpy(eng, np.full(n * sr, 0x77, np.uint8))
        rs16.encode_device_batch(k, m, sb, n, d_o.ptr, so, d_r.ptr, sr, engine=eng)
        got = d_r.download(shape=(n * sr,))
        recs = []
        for i, o in enumerate(stripes):
            r = got[i * sr:i * sr + m * sb].reshape(m, sb)
            assert np.array_equal(r, O.encode(k, m, o)), why + (i,)
            assert (got[i * sr + m * sb:(i + 1) * sr] == 0x77).all(), why + (i,)
            recs.append(r.copy())
        o_lost, r_lost = random_loss(rng, k, m)
        for i in range(n):
            host_o[i * so:i * so + k * sb].reshape(k, sb)[o_lost] = 0xA5
        d_x = DeviceArray.from_numpy(eng, host_o)
        d_fo, d_fr = _decode_masks(eng, k, m, o_lost, r_lost)
        rs16.decode_device_batch(k, m, sb, n, d_x.ptr, so, d_fo.ptr, d_r.ptr, sr, d_fr.ptr, int((~o_lost).sum()),
                                 int((~r_lost).sum()), engine=eng)
        back = d_x.download(shape=(n * so,))
        for i, o in enumerate(stripes):
            assert np.array_equal(back[i * so:i * so + k * sb].reshape(k, sb), o), why + (i,)
            assert (back[i * so + k * sb:(i + 1) * so] == 0xEE).all(), why + (i,)
    eng.set_diagnostics(0)


def test_random_batches_varied(eng):
    """rs16_decode_device_batch_varied: every stripe its own loss set drawn
    by the reference's rules, 2-12 stripes, 40 cases."""
    rng = np.random.default_rng(4_242_424 + SEED)
    for case in range(40 * MULT):
        k, m = random_counts(rng)
        n = int(rng.integers(2, 13))
        sb = 64 * int(rng.integers(1, max(1, min(128, BUDGET // (64 * (k + m) * n))) + 1))
        diag = random_diag(rng)
        eng.set_diagnostics(diag)
        why = (case, k, m, sb, n, hex(diag))
        so, sr = k * sb + 64, m * sb
        fso, fsr = k + int(rng.integers(0, 9)), m + int(rng.integers(0, 9))
        stripes = [random_data(rng, k, sb) for _ in range(n)]
        host_o = np.full(n * so, 0x3C, np.uint8)
        host_r = np.zeros(n * sr, np.uint8)
        fo = np.full(n * fso, 0xFF, np.uint8)
        fr = np.full(n * fsr, 0xFF, np.uint8)
        oc, rc = [], []
        for i, o in enumerate(stripes):
            o_lost, r_lost = random_loss(rng, k, m)
            held = o.copy()
            held[o_lost] = 0xA5
            host_o[i * so:i * so + k * sb] = held.reshape(-1)
            rec = O.encode(k, m, o)
            rec[r_lost] = 0x5A
            host_r[i * sr:(i + 1) * sr] = rec.reshape(-1)
            fo[i * fso:i * fso + k] = ~o_lost
            fr[i * fsr:i * fsr + m] = ~r_lost
            oc.append(int((~o_lost).sum()))
            rc.append(int((~r_lost).sum()))
        d_o, d_r = DeviceArray.from_numpy(eng, host_o), DeviceArray.from_numpy(eng, host_r)
        d_fo, d_fr = DeviceArray.from_numpy(eng, fo), DeviceArray.from_numpy(eng, fr)
        rs16.decode_device_batch_varied(k, m, sb, n, d_o.ptr, so, d_fo.ptr, fso, d_r.ptr, sr, d_fr.ptr, fsr, oc, rc,
                                        engine=eng)
        got = d_o.download(shape=(n * so,))
        for i, o in enumerate(stripes):
            assert np.array_equal(got[i * so:i * so + k * sb].reshape(k, sb), o), why + (i,)
            assert (got[i * so + k * sb:(i + 1) * so] == 0x3C).all(), why + (i,)
        assert np.array_equal(d_r.download(shape=(n * sr,)), host_r), why
    eng.set_diagnostics(0)
