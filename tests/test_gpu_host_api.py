"""The Rate-level API with shards in host memory:
ReedSolomonEncoder / ReedSolomonDecoder add_*_shard copy host shards into a
page-locked image of the work buffer (rs16_api.cpp "Host staging"), stream
runs of consecutive rows to HBM while the caller keeps adding, and bring the
results back in one DMA copy.  Checked against the oracle (tests/oracle_bind)
bit for bit:

- several rounds on one encoder / decoder, with results dropped unread (the
  reference bench's pattern, benches/benchmarks.rs:71-76, 98-106) so that a
  round's adds run while the previous round's copies may still be in flight;
- large rounds (several 1 MiB streaming copies per round), random add orders,
  scattered receive patterns (the decoder's run / span copy paths);
- host and device shards mixed in one round;
- stale Python results (a result kept across reset()) do not disturb a newer
  round.
"""
import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16.device import DeviceArray
from rs16.util import generate_original

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,m,sb", [(4096, 4096, 1024), (3000, 1000, 512), (1000, 3000, 256), (60000, 3000, 64)])
def test_encoder_rounds_unread(k, m, sb):
    enc = rs16.ReedSolomonEncoder(k, m, sb)
    for rnd in range(4):
        original = generate_original(k, sb, 40 + rnd)
        for s in original:
            enc.add_original_shard(s)
        res = enc.encode()
        if rnd in (1, 2):
            res.drop()  # unread: the next round's adds overlap this round's copies
            continue
        got = b"".join(res.recovery_iter())
        res.drop()
        assert got == O.encode(k, m, original).tobytes(), rnd


@pytest.mark.parametrize("k,m,sb", [(4096, 4096, 1024), (1000, 3000, 256), (3000, 1000, 512)])
def test_decoder_rounds_random_orders(k, m, sb):
    rng = np.random.default_rng(k + m)
    dec = rs16.ReedSolomonDecoder(k, m, sb)
    for rnd in range(4):
        original = generate_original(k, sb, 50 + rnd)
        recovery = O.encode(k, m, original)
        loss = int(rng.integers(1, min(k, m) + 1))
        lost = rng.choice(k, loss, replace=False)
        keep = np.setdiff1d(np.arange(k), lost)
        rec = rng.choice(m, loss, replace=False)
        adds = [(True, int(i)) for i in keep] + [(False, int(i)) for i in rec]
        if rnd % 2:
            rng.shuffle(adds)  # random order: runs, pending rows, span copies
        for is_orig, i in adds:
            if is_orig:
                dec.add_original_shard(i, original[i])
            else:
                dec.add_recovery_shard(i, recovery[i])
        res = dec.decode()
        if rnd == 2:
            res.drop()
            continue
        got = dict(res.restored_original_iter())
        res.drop()
        assert set(got) == set(int(i) for i in lost)
        for i, s in got.items():
            assert s == original[i].tobytes(), (rnd, i)


def test_decoder_sequential_tail_loss_large():
    # the reference bench's 1 % pattern at 32768:32768 x 1 KiB: two long
    # sequential runs (originals 0..k-L, recovery 0..L) streamed while adding
    k = m = 32768
    sb = 1024
    original = generate_original(k, sb, 0)
    recovery = O.encode(k, m, original)
    L = k // 100
    dec = rs16.ReedSolomonDecoder(k, m, sb)
    for _ in range(2):
        for i in range(k - L):
            dec.add_original_shard(i, original[i])
        for i in range(L):
            dec.add_recovery_shard(i, recovery[i])
        with dec.decode() as res:
            got = dict(res.restored_original_iter())
        assert sorted(got) == list(range(k - L, k))
        for i, s in got.items():
            assert s == original[i].tobytes(), i


def test_mixed_host_and_device_shards():
    eng = rs16.Engine(0)
    k, m, sb = 2048, 2048, 256
    original = generate_original(k, sb, 7)
    recovery = O.encode(k, m, original)
    d_orig = DeviceArray.from_numpy(eng, original)
    d_rec = DeviceArray.from_numpy(eng, recovery)
    enc = rs16.ReedSolomonEncoder(k, m, sb, engine=eng)
    for i in range(k):
        if (i // 37) % 2:
            enc.add_original_shard_device(d_orig.ptr + i * sb, sb)
        else:
            enc.add_original_shard(original[i])
    with enc.encode() as res:
        assert b"".join(res.recovery_iter()) == recovery.tobytes()
    # decoder: scattered host rows (more than 32 runs) with device rows in
    # between, so the span copy must not be used; then the same pattern all
    # from host memory (span copy)
    rng = np.random.default_rng(3)
    lost = np.sort(rng.choice(k, 700, replace=False))
    keep = np.setdiff1d(np.arange(k), lost)
    dec = rs16.ReedSolomonDecoder(k, m, sb, engine=eng)
    for device_rows in (True, False):
        for j, i in enumerate(keep):
            if device_rows and j % 3 == 1:
                dec.add_original_shard_device(int(i), d_orig.ptr + int(i) * sb, sb)
            else:
                dec.add_original_shard(int(i), original[i])
        for j, i in enumerate(range(0, 2 * 700, 2)):
            if device_rows and j % 5 == 2:
                dec.add_recovery_shard_device(i, d_rec.ptr + i * sb, sb)
            else:
                dec.add_recovery_shard(i, recovery[i])
        with dec.decode() as res:
            got = dict(res.restored_original_iter())
        assert sorted(got) == [int(i) for i in lost]
        for i, s in got.items():
            assert s == original[i].tobytes(), (device_rows, i)
    del enc, dec
    eng.close()


def test_stale_result_does_not_disturb_newer_round():
    k, m, sb = 16, 16, 64
    a = generate_original(k, sb, 1)
    b = generate_original(k, sb, 2)
    enc = rs16.ReedSolomonEncoder(k, m, sb)
    for s in a:
        enc.add_original_shard(s)
    old = enc.encode()
    enc.reset(k, m, sb)  # the reference needs &mut here: `old` is stale
    for s in b:
        enc.add_original_shard(s)
    new = enc.encode()
    old.drop()  # no-op: must not end the newer round
    assert b"".join(new.recovery_iter()) == O.encode(k, m, b).tobytes()
    with pytest.raises(ValueError):
        old.recovery(0)
    new.drop()
    dec = rs16.ReedSolomonDecoder(k, m, sb)
    rb = O.encode(k, m, b)
    for i in range(k):
        dec.add_recovery_shard(i, rb[i])
    old_d = dec.decode()
    dec.reset(k, m, sb)
    for i in range(k // 2):
        dec.add_original_shard(i, b[i])
    old_d.drop()  # must not wipe the received set of the round being built
    for i in range(k // 2):
        dec.add_recovery_shard(i, rb[i])
    with dec.decode() as res:
        got = dict(res.restored_original_iter())
    assert got == {i: b[i].tobytes() for i in range(k // 2, k)}
