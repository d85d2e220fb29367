"""CPU-only checks of the C-ABI library (no GPU calls).

- librs16.so loads and exports every symbol include/rs16.h declares, and the
  Python binding covers exactly that set.
- Host-side logic mirrors the reference: supports / validate / use_high_rate /
  work_count tables from src/rate/rate_{high,low,default}.rs tests and
  src/reed_solomon.rs:274-283, Error Display texts (src/lib.rs:130-222).
- The v_perm multiply-table format (evaluated on the host through the same
  mul_xor code the kernels use) equals the oracle's NoSimd::mul for random
  data and random/edge log_m values.
"""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as O
import rs16
from rs16._lib import LIB_PATH, SIGNATURES, lib

ROOT = Path(__file__).resolve().parents[1]
HEADER = (ROOT / "include" / "rs16.h").read_text()
USIZE_MAX = 2**64 - 1


def declared_functions():
    body = re.sub(r"/\*.*?\*/", "", HEADER, flags=re.S)
    return set(re.findall(r"\b(rs16_[a-z0-9_]+)\s*\(", body))


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB_PATH)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\b(rs16_[a-z0-9_]+)\b", out))
    declared = declared_functions()
    assert declared, "no declarations parsed"
    missing = declared - exported
    assert not missing, missing
    assert set(SIGNATURES) == declared
    lib()  # every signature resolves


def test_version():
    assert b"gfx950" in lib().rs16_version()


# ---- src/rate/rate_high.rs:458-605, rate_low.rs:458-605 ----
def test_high_low_supports():
    H, Lo = "high", "low"
    assert not rs16.supports(0, 1, H) and not rs16.supports(1, 0, H)
    assert not rs16.supports(4096, 61440, H)
    assert rs16.supports(61440, 4096, H)
    assert not rs16.supports(61440, 4097, H) and not rs16.supports(61441, 4096, H)
    assert not rs16.supports(USIZE_MAX, USIZE_MAX, H)
    assert not rs16.supports(0, 1, Lo) and not rs16.supports(1, 0, Lo)
    assert rs16.supports(4096, 61440, Lo)
    assert not rs16.supports(61440, 4096, Lo)
    assert not rs16.supports(4097, 61440, Lo) and not rs16.supports(4096, 61441, Lo)
    assert not rs16.supports(USIZE_MAX, USIZE_MAX, Lo)


def test_validate():
    for rate in ("high", "low"):
        with pytest.raises(rs16.Error) as e:
            rs16.validate(1, 1, 123, rate)
        assert e.value == rs16.Error("InvalidShardSize", shard_bytes=123)
    with pytest.raises(rs16.Error) as e:
        rs16.validate(4096, 61440, 64, "high")
    assert e.value == rs16.Error("UnsupportedShardCount", original_count=4096, recovery_count=61440)
    rs16.validate(61440, 4096, 64, "high")
    rs16.validate(4096, 61440, 64, "low")


def test_work_counts():
    # rate_high.rs:521-528, 583-592 ; rate_low.rs same tables mirrored
    assert rs16.encoder_work_count(True, 1, 1) == 1
    assert rs16.encoder_work_count(True, 4096, 1024) == 4096
    assert rs16.encoder_work_count(True, 4097, 1024) == 5120
    assert rs16.encoder_work_count(True, 4097, 1025) == 6144
    assert rs16.encoder_work_count(True, 32768, 32768) == 32768
    assert rs16.decoder_work_count(True, 1, 1) == 2
    assert rs16.decoder_work_count(True, 2048, 1025) == 4096
    assert rs16.decoder_work_count(True, 2049, 1025) == 8192
    assert rs16.decoder_work_count(True, 3072, 1024) == 4096
    assert rs16.decoder_work_count(True, 3073, 1024) == 8192
    assert rs16.decoder_work_count(True, 32768, 32768) == 65536
    assert rs16.encoder_work_count(False, 1024, 4096) == 4096
    assert rs16.encoder_work_count(False, 1024, 4097) == 5120
    assert rs16.encoder_work_count(False, 1025, 4097) == 6144
    assert rs16.decoder_work_count(False, 1025, 2048) == 4096
    assert rs16.decoder_work_count(False, 1025, 2049) == 8192


def test_use_high_rate_table():
    # src/rate/rate_default.rs:444-478
    cases = [(0, 1, None), (1, 0, None), (3, 3, True), (3, 4, True), (3, 5, False), (4, 3, False), (5, 3, True),
             (4096, 61440, False), (4096, 61441, None), (4097, 61440, None), (61440, 4096, True),
             (61440, 4097, None), (61441, 4096, None), (USIZE_MAX, USIZE_MAX, None)]
    for k, m, want in cases:
        if want is None:
            with pytest.raises(rs16.Error) as e:
                rs16.use_high_rate(k, m)
            assert e.value == rs16.Error("UnsupportedShardCount", original_count=k, recovery_count=m)
        else:
            assert rs16.use_high_rate(k, m) is want


def test_reed_solomon_supports():
    # src/reed_solomon.rs:76-81, 174-179, 274-283
    assert rs16.ReedSolomonEncoder.supports(60000, 4000)
    assert not rs16.ReedSolomonEncoder.supports(60000, 5000)
    assert rs16.ReedSolomonDecoder.supports(60000, 4000)
    assert not rs16.ReedSolomonDecoder.supports(60000, 5000)
    for cls in (rs16.ReedSolomonEncoder, rs16.ReedSolomonDecoder):
        assert cls.supports(4096, 61440) and cls.supports(61440, 4096)


def test_error_display_texts():
    E = rs16.Error
    assert str(E("DifferentShardSize", shard_bytes=64, got=128)) == "different shard size: expected 64 bytes, got 128 bytes"
    assert str(E("DuplicateOriginalShardIndex", index=3)) == "duplicate original shard index: 3"
    assert str(E("DuplicateRecoveryShardIndex", index=4)) == "duplicate recovery shard index: 4"
    assert str(E("InvalidOriginalShardIndex", original_count=1, index=2)) == "invalid original shard index: 2 >= original_count 1"
    assert str(E("InvalidRecoveryShardIndex", recovery_count=1, index=2)) == "invalid recovery shard index: 2 >= recovery_count 1"
    assert str(E("InvalidShardSize", shard_bytes=0)) == "invalid shard size: 0 bytes (must non-zero and multiple of 64)"
    assert str(E("NotEnoughShards", original_count=5, original_received_count=1, recovery_received_count=2)) == \
        "not enough shards: 1 original + 2 recovery < 5 original_count"
    assert str(E("TooFewOriginalShards", original_count=3, original_received_count=1)) == \
        "too few original shards: got 1 shards while original_count is 3"
    assert str(E("TooManyOriginalShards", original_count=1)) == "too many original shards: got more than original_count (1) shards"
    assert str(E("UnsupportedShardCount", original_count=0, recovery_count=1)) == \
        "unsupported shard count: 0 original shards with 1 recovery shards"


def test_one_shot_errors_before_any_device_work():
    # src/lib.rs:406-430 : these are raised before an encoder is created
    with pytest.raises(rs16.Error) as e:
        rs16.encode(0, 1, [])
    assert e.value == rs16.Error("UnsupportedShardCount", original_count=0, recovery_count=1)
    with pytest.raises(rs16.Error) as e:
        rs16.encode(1, 0, [bytes(64)])
    assert e.value == rs16.Error("UnsupportedShardCount", original_count=1, recovery_count=0)
    with pytest.raises(rs16.Error) as e:
        rs16.encode(1, 1, [])
    assert e.value == rs16.Error("TooFewOriginalShards", original_count=1, original_received_count=0)
    # src/lib.rs:441-444, 539-548, 562-580
    assert rs16.decode(1, 1, [(0, bytes(64))], []) == {}
    with pytest.raises(rs16.Error) as e:
        rs16.decode(1, 1, [], [])
    assert e.value == rs16.Error("NotEnoughShards", original_count=1, original_received_count=0, recovery_received_count=0)
    with pytest.raises(rs16.Error) as e:
        rs16.decode(0, 1, [], [])
    assert e.value == rs16.Error("UnsupportedShardCount", original_count=0, recovery_count=1)
    with pytest.raises(rs16.Error) as e:
        rs16.decode(1, 0, [], [])
    assert e.value == rs16.Error("UnsupportedShardCount", original_count=1, recovery_count=0)


@pytest.mark.parametrize("log_m", [0, 1, 2, 12345, 32768, 65534, 65535])
def test_host_mul_table_format_matches_oracle(log_m):
    rng = np.random.default_rng(log_m)
    x = rng.integers(0, 256, 64 * 64, dtype=np.uint8)
    want = x.copy()
    O.mul(want, log_m, "nosimd")
    got = np.empty_like(x)
    lib().rs16_host_mul(x.ctypes.data_as(C.c_void_p), got.ctypes.data_as(C.c_void_p), x.size, log_m)
    assert np.array_equal(got, want)


def test_host_mul_all_logs_one_block():
    rng = np.random.default_rng(7)
    x = rng.integers(0, 256, 64, dtype=np.uint8)
    got = np.empty_like(x)
    for log_m in range(0, 65536, 97):
        want = x.copy()
        O.mul(want, log_m, "nosimd")
        lib().rs16_host_mul(x.ctypes.data_as(C.c_void_p), got.ctypes.data_as(C.c_void_p), 64, log_m)
        assert np.array_equal(got, want), log_m


def test_column_slice_partition_matches_python():
    # rs16_column_slice (the RCCL scatter / gather and multi-engine split) and
    # rs16/columns.py (the bench's per-rank split) partition alike: every
    # 64-byte block once, in order (src/algorithm.md:18-32)
    from rs16.columns import column_slices
    for S in (64, 192, 1024, 64 * 1024, 64 * 5):
        for n in (1, 2, 3, 4, 8):
            got = [rs16.column_slice(S, n, r) for r in range(n)]
            assert sum(w for _, w in got) == S
            assert all(o % 64 == 0 and w % 64 == 0 for o, w in got)
            assert [o for o, _ in got] == sorted(o for o, _ in got)
            assert got == column_slices(S, n)
    with pytest.raises(rs16.Error):
        rs16.column_slice(100, 2, 0)


def test_deprecated_process_diagnostics_default():
    """rs16_set_diagnostics (the round-4 process-wide ABI, kept as a
    deprecated wrapper): it sets the flags new engines start with
    and returns the previous default; unknown bits are dropped.  No device
    call is made."""
    from rs16._lib import lib

    L = lib()
    prev = L.rs16_set_diagnostics(512 | (1 << 30))
    try:
        assert L.rs16_set_diagnostics(0) == 512
        assert L.rs16_set_diagnostics(prev) == 0
    finally:
        L.rs16_set_diagnostics(prev)
