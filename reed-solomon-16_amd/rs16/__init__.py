"""rs16 -- Python mirror of the reed_solomon_16 API over the MI355X C ABI.

Reference API (malaire/reed-solomon-16 v0.1.0) -> here:
  reed_solomon_16::encode / decode        (src/lib.rs:242-344)    -> encode(), decode()
  ReedSolomonEncoder / ReedSolomonDecoder (src/reed_solomon.rs)   -> same names
  EncoderResult / DecoderResult + Drop    (src/{encoder,decoder}_result.rs)
  rate::{Default,High,Low}Rate{Encoder,Decoder} (src/rate/*.rs)  -> RateEncoder/RateDecoder(rate=...)
  Error (src/lib.rs:31-222)                                       -> Error
  engine::Engine ops (src/engine.rs:140-260) on device arrays     -> Engine methods
plus the device-resident one-shot path (encode_device / decode_device).

Every call runs through reed-solomon-16_amd/build/librs16.so (HIP, gfx950).
There is no CPU fallback.
"""
from __future__ import annotations

import atexit
import ctypes as C
import weakref
from typing import Iterable, Iterator, Optional, Tuple

import numpy as np

from ._lib import RS16Error, lib

__all__ = [
    "Error", "Engine", "default_engine", "ReedSolomonEncoder", "ReedSolomonDecoder", "RateEncoder",
    "RateDecoder", "EncoderResult", "DecoderResult", "encode", "decode", "encode_device", "decode_device",
    "supports", "validate", "use_high_rate", "encode_device_batch", "decode_device_batch", "encoder_work_count", "decoder_work_count",
    "RATE_DEFAULT", "RATE_HIGH", "RATE_LOW", "GF_ORDER", "GF_MODULUS", "set_diagnostics",
    "DIAG_FORCE_VOFF64", "DIAG_EVAL_TWO_KERNEL", "DIAG_EVAL_FULL", "DIAG_NO_COLUMN", "DIAG_FORCE_COLUMN",
    "DIAG_TILE_LAST", "DIAG_NO_TILE_LAST", "DIAG_FD_LDS", "DIAG_COL_RADIX4", "DIAG_NO_IDENTITY", "DIAG_NO_MID_DIRECT", "encode_host", "decode_host",
    "encode_host_batch", "decode_host_batch", "decode_prepare", "decode_device_prepared",
    "encode_host_multi", "decode_host_multi", "Comm", "column_slice", "scatter_columns", "gather_columns",
]

GF_ORDER = 65536
GF_MODULUS = 65535
# rs16_engine_set_diagnostics flags (include/rs16.h): alternative code paths for tests
DIAG_FORCE_VOFF64, DIAG_EVAL_TWO_KERNEL, DIAG_EVAL_FULL, DIAG_NO_COLUMN, DIAG_FORCE_COLUMN = 1, 2, 4, 8, 16
DIAG_TILE_LAST, DIAG_NO_TILE_LAST, DIAG_FD_LDS, DIAG_COL_RADIX4, DIAG_NO_IDENTITY = 32, 64, 128, 256, 512
DIAG_NO_MID_DIRECT = 1024
# Test convenience only: the flags set_diagnostics() without an engine gave
# every live engine, and that engines created later in this Python process
# start with.  The library itself keeps the switches per engine.
_diag_default = 0


def set_diagnostics(flags: int, engine: Optional["Engine"] = None) -> int:
    """Diagnostic switches (identical results); returns the previous flags.

    With an engine: that engine's switches (rs16_engine_set_diagnostics).
    Without: every live engine's, and those of engines created afterwards
    in this process (a test helper; returns the previous default)."""
    global _diag_default
    if engine is not None:
        return engine.set_diagnostics(flags)
    old, _diag_default = _diag_default, flags
    for e in list(_live_engines):
        if getattr(e, "h", None):
            e.set_diagnostics(flags)
    return old
RATE_DEFAULT, RATE_HIGH, RATE_LOW = 0, 1, 2
_RATES = {"default": 0, "high": 1, "low": 2, 0: 0, 1: 1, 2: 2}

# Error variants in the order of src/lib.rs:31-125 and their payload fields.
_VARIANTS = {
    1: ("DifferentShardSize", ("shard_bytes", "got")),
    2: ("DuplicateOriginalShardIndex", ("index",)),
    3: ("DuplicateRecoveryShardIndex", ("index",)),
    4: ("InvalidOriginalShardIndex", ("original_count", "index")),
    5: ("InvalidRecoveryShardIndex", ("recovery_count", "index")),
    6: ("InvalidShardSize", ("shard_bytes",)),
    7: ("NotEnoughShards", ("original_count", "original_received_count", "recovery_received_count")),
    8: ("TooFewOriginalShards", ("original_count", "original_received_count")),
    9: ("TooManyOriginalShards", ("original_count",)),
    10: ("UnsupportedShardCount", ("original_count", "recovery_count")),
    100: ("DeviceError", ("hip_error",)),
    101: ("InvalidArgument", ()),
}
_CODES = {name: code for code, (name, _) in _VARIANTS.items()}


class Error(Exception):
    """reed_solomon_16::Error.  ``Error("UnsupportedShardCount", original_count=0,
    recovery_count=1)`` compares equal to the error the library returns."""

    def __init__(self, kind: str, **fields):
        if kind not in _CODES:
            raise ValueError(kind)
        self.kind, self.fields = kind, fields
        self.code = _CODES[kind]
        super().__init__(self._message())

    @classmethod
    def _from_c(cls, e: RS16Error) -> "Error":
        name, fnames = _VARIANTS.get(e.code, ("InvalidArgument", ()))
        vals = (e.v0, e.v1, e.v2)
        err = cls(name, **{f: int(v) for f, v in zip(fnames, vals)})
        return err

    def _message(self) -> str:
        e = RS16Error(self.code, 0, 0, 0)
        vals = list(self.fields.values()) + [0, 0, 0]
        e.v0, e.v1, e.v2 = vals[0], vals[1], vals[2]
        buf = C.create_string_buffer(256)
        lib().rs16_error_message(C.byref(e), buf, 256)
        return buf.value.decode()

    def __eq__(self, other):
        return isinstance(other, Error) and (self.kind, self.fields) == (other.kind, other.fields)

    def __hash__(self):
        return hash((self.kind, tuple(sorted(self.fields.items()))))

    def __repr__(self):
        return f"Error.{self.kind}({', '.join(f'{k}={v}' for k, v in self.fields.items())})"


def _check(rc: int, err: RS16Error):
    if rc != 0:
        raise Error._from_c(err)


# ---------------------------------------------------------------------------
# Shard buffers: host (bytes / bytearray / memoryview / numpy) or device
# (any object with .is_cuda/.data_ptr(), e.g. a torch tensor on ROCm).
# ---------------------------------------------------------------------------
def _is_device(x) -> bool:
    return bool(getattr(x, "is_cuda", False))


def _device_ptr_len(x) -> Tuple[int, int]:
    if not x.is_contiguous():
        raise ValueError("device shard must be contiguous")
    return x.data_ptr(), x.numel() * x.element_size()


def _host_buf(x):
    """Returns (ctypes pointer, length, keepalive)."""
    if isinstance(x, np.ndarray):
        a = np.ascontiguousarray(x).view(np.uint8).reshape(-1)
        return a.ctypes.data_as(C.c_void_p), a.size, a
    if isinstance(x, str):
        x = x.encode()
    mv = memoryview(x).cast("B")
    n = mv.nbytes
    if n == 0:
        return None, 0, None
    if mv.readonly:
        buf = (C.c_char * n).from_buffer_copy(mv)
    else:
        buf = (C.c_char * n).from_buffer(mv)
    return C.cast(buf, C.c_void_p), n, buf


def _shard_len(x) -> int:
    if _is_device(x):
        return _device_ptr_len(x)[1]
    if isinstance(x, np.ndarray):
        return x.nbytes
    return memoryview(x.encode() if isinstance(x, str) else x).nbytes


# ---------------------------------------------------------------------------
# Engine
# ---------------------------------------------------------------------------
class Engine:
    """The MI355X engine: GF tables resident in HBM of ``device`` (NoSimd::new
    analogue, src/engine/engine_nosimd.rs:27-35) plus the Engine trait ops on
    device shard arrays (src/engine.rs:140-260).  Device arrays are passed as
    raw device pointers (int) or torch tensors."""

    OWN_QUEUE = 1  # RS16_ENGINE_OWN_QUEUE: the engine's stream on a hardware queue of its own

    def __init__(self, device: int = 0, flags: int = 0):
        self._err = RS16Error()
        self.h = lib().rs16_engine_new_ex(device, flags, C.byref(self._err))
        if not self.h:
            raise Error._from_c(self._err)
        self.device = device
        _live_engines.add(self)
        if _diag_default:
            self.set_diagnostics(_diag_default)

    def set_diagnostics(self, flags: int) -> int:
        """This engine's diagnostic switches (include/rs16.h); returns the previous ones."""
        return lib().rs16_engine_set_diagnostics(self.h, flags)

    def close(self):
        if getattr(self, "h", None):
            lib().rs16_engine_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return lib().rs16_engine_stream(self.h) or 0

    def synchronize(self, stream=None):
        _check(lib().rs16_engine_synchronize(self.h, stream, C.byref(self._err)), self._err)

    def set_slices(self, n: int):
        """Concurrent column slices of the device one-shot codec (1..4)."""
        _check(lib().rs16_engine_set_slices(self.h, n, C.byref(self._err)), self._err)

    def create_stream(self) -> int:
        """A new non-blocking hipStream_t on this engine's device (raw handle)."""
        p = lib().rs16_stream_create(self.h, C.byref(self._err))
        if not p:
            raise Error._from_c(self._err)
        return p

    def destroy_stream(self, stream: int):
        if self.h and stream:
            lib().rs16_stream_destroy(self.h, stream)

    # per-pass hipEvent timing (include/rs16.h "Diagnostics")
    def set_profiling(self, enable: bool):
        _check(lib().rs16_engine_set_profiling(self.h, int(enable), C.byref(self._err)), self._err)

    def profile_reset(self):
        lib().rs16_engine_profile_reset(self.h)

    def profile(self) -> dict:
        """{program name: (total_ms, launches)} since the last reset."""
        out = {}
        for p in range(lib().rs16_prog_count()):
            ms, n = C.c_double(), C.c_uint64()
            _check(lib().rs16_engine_profile_read(self.h, p, C.byref(ms), C.byref(n), C.byref(self._err)), self._err)
            if n.value:
                out[lib().rs16_prog_name(p).decode()] = (ms.value, n.value)
        return out

    @staticmethod
    def _ptr(x) -> int:
        return x.data_ptr() if hasattr(x, "data_ptr") else int(x)

    # Engine trait (device arrays; see include/rs16.h)
    def fft(self, data, shard_count, shard_bytes, pos, size, truncated_size, skew_delta, stream=None):
        _check(lib().rs16_engine_fft(self.h, self._ptr(data), shard_count, shard_bytes, pos, size, truncated_size,
                                     skew_delta, stream, C.byref(self._err)), self._err)

    def ifft(self, data, shard_count, shard_bytes, pos, size, truncated_size, skew_delta, stream=None):
        _check(lib().rs16_engine_ifft(self.h, self._ptr(data), shard_count, shard_bytes, pos, size, truncated_size,
                                      skew_delta, stream, C.byref(self._err)), self._err)

    def fft_skew_end(self, data, shard_count, shard_bytes, pos, size, truncated_size, stream=None):
        _check(lib().rs16_engine_fft_skew_end(self.h, self._ptr(data), shard_count, shard_bytes, pos, size,
                                              truncated_size, stream, C.byref(self._err)), self._err)

    def ifft_skew_end(self, data, shard_count, shard_bytes, pos, size, truncated_size, stream=None):
        _check(lib().rs16_engine_ifft_skew_end(self.h, self._ptr(data), shard_count, shard_bytes, pos, size,
                                               truncated_size, stream, C.byref(self._err)), self._err)

    def fwht(self, data_u16, truncated_size, stream=None):
        _check(lib().rs16_engine_fwht(self.h, self._ptr(data_u16), truncated_size, stream, C.byref(self._err)),
               self._err)

    def eval_poly(self, erasures_u16, truncated_size, stream=None):
        _check(lib().rs16_engine_eval_poly(self.h, self._ptr(erasures_u16), truncated_size, stream,
                                           C.byref(self._err)), self._err)

    def mul(self, x, nbytes, log_m, stream=None):
        _check(lib().rs16_engine_mul(self.h, self._ptr(x), nbytes, log_m, stream, C.byref(self._err)), self._err)

    def xor(self, x, y, nbytes, stream=None):
        _check(lib().rs16_engine_xor(self.h, self._ptr(x), self._ptr(y), nbytes, stream, C.byref(self._err)),
               self._err)

    def xor_within(self, data, shard_count, shard_bytes, x, y, count, stream=None):
        _check(lib().rs16_engine_xor_within(self.h, self._ptr(data), shard_count, shard_bytes, x, y, count, stream,
                                            C.byref(self._err)), self._err)

    def formal_derivative(self, data, shard_count, shard_bytes, stream=None):
        _check(lib().rs16_engine_formal_derivative(self.h, self._ptr(data), shard_count, shard_bytes, stream,
                                                   C.byref(self._err)), self._err)


_default_engines = {}
_live_engines = weakref.WeakSet()


@atexit.register
def _close_engines():
    # Close engines while the HIP runtime is still up, in a defined order
    # (module globals are torn down in arbitrary order at interpreter exit);
    # device arrays still alive after this see engine.h None and are left
    # to the runtime.
    for e in list(_live_engines):
        e.close()


def default_engine(device: Optional[int] = None) -> Engine:
    if device is None:
        device = 0
    if device not in _default_engines:
        _default_engines[device] = Engine(device)
    return _default_engines[device]


# ---------------------------------------------------------------------------
# Rate helpers
# ---------------------------------------------------------------------------
def supports(original_count, recovery_count, rate="default") -> bool:
    if not (0 <= original_count < 2**64 and 0 <= recovery_count < 2**64):
        return False
    return bool(lib().rs16_supports(_RATES[rate], original_count, recovery_count))


def validate(original_count, recovery_count, shard_bytes, rate="default"):
    err = RS16Error()
    _check(lib().rs16_validate(_RATES[rate], original_count, recovery_count, shard_bytes, C.byref(err)), err)


def use_high_rate(original_count, recovery_count) -> bool:
    err = RS16Error()
    r = lib().rs16_use_high_rate(original_count, recovery_count, C.byref(err))
    if r < 0:
        raise Error._from_c(err)
    return bool(r)


def encoder_work_count(high: bool, original_count, recovery_count) -> int:
    return lib().rs16_encoder_work_count(int(high), original_count, recovery_count)


def decoder_work_count(high: bool, original_count, recovery_count) -> int:
    return lib().rs16_decoder_work_count(int(high), original_count, recovery_count)


# ---------------------------------------------------------------------------
# Results
# ---------------------------------------------------------------------------
class EncoderResult:
    """EncoderResult (src/encoder_result.rs).  Dropping it (``del``, ``with``,
    or ``drop()``) resets the encoder for a new round, like Drop.  A result
    that outlives a later round of its encoder (reset, or a new encode after
    an explicit drop) is stale: its drop is a no-op, as the reference's borrow
    rules make that state unreachable there."""

    def __init__(self, enc: "RateEncoder"):
        self._enc = enc
        self._gen = enc._gen

    def _live(self) -> "RateEncoder":
        e = self._enc
        if e is None or e._gen != self._gen:
            raise ValueError("EncoderResult used after it was dropped")
        return e

    def recovery(self, index: int) -> Optional[bytes]:
        e = self._live()
        p = lib().rs16_encoder_recovery(e.h, index, C.byref(e._err))
        if not p:
            if e._err.code != 0:
                raise Error._from_c(e._err)
            return None
        return C.string_at(p, e.shard_bytes)

    def recovery_device(self, index: int) -> Optional[int]:
        return lib().rs16_encoder_recovery_device(self._live().h, index)

    def recovery_iter(self) -> Iterator[bytes]:
        i = 0
        while True:
            r = self.recovery(i)
            if r is None:
                return
            yield r
            i += 1

    def drop(self):
        enc, self._enc = self._enc, None
        if enc is not None and enc.h and enc._gen == self._gen:
            enc._gen += 1
            lib().rs16_encoder_result_drop(enc.h)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.drop()

    def __del__(self):
        try:
            self.drop()
        except Exception:
            pass


class DecoderResult:
    """DecoderResult (src/decoder_result.rs); stale results as EncoderResult."""

    def __init__(self, dec: "RateDecoder"):
        self._dec = dec
        self._gen = dec._gen

    def _live(self) -> "RateDecoder":
        d = self._dec
        if d is None or d._gen != self._gen:
            raise ValueError("DecoderResult used after it was dropped")
        return d

    def restored_original(self, index: int) -> Optional[bytes]:
        d = self._live()
        p = lib().rs16_decoder_restored_original(d.h, index, C.byref(d._err))
        if not p:
            if d._err.code != 0:
                raise Error._from_c(d._err)
            return None
        return C.string_at(p, d.shard_bytes)

    def restored_original_device(self, index: int) -> Optional[int]:
        return lib().rs16_decoder_restored_original_device(self._live().h, index)

    def restored_original_iter(self) -> Iterator[Tuple[int, bytes]]:
        for i in range(self._live().original_count):
            r = self.restored_original(i)
            if r is not None:
                yield i, r

    def drop(self):
        dec, self._dec = self._dec, None
        if dec is not None and dec.h and dec._gen == self._gen:
            dec._gen += 1
            lib().rs16_decoder_result_drop(dec.h)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.drop()

    def __del__(self):
        try:
            self.drop()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# Encoders / decoders
# ---------------------------------------------------------------------------
class RateEncoder:
    """RateEncoder<E = MI355X engine> (src/rate.rs:113-173) for rate
    "default" (DefaultRateEncoder), "high" or "low"."""

    def __init__(self, original_count, recovery_count, shard_bytes, rate="default", engine: Optional[Engine] = None):
        self.engine = engine or default_engine()
        self._err = RS16Error()
        self._gen = 0  # bumped by reset() and by a result's drop: older results go stale
        self.h = lib().rs16_encoder_new(self.engine.h, _RATES[rate], original_count, recovery_count, shard_bytes,
                                        C.byref(self._err))
        if not self.h:
            raise Error._from_c(self._err)
        self.original_count, self.recovery_count, self.shard_bytes = original_count, recovery_count, shard_bytes

    def __del__(self):
        # Safe after the engine is gone: rs16_engine_free detaches its
        # encoders, and freeing a detached one only frees host memory.
        try:
            if getattr(self, "h", None):
                lib().rs16_encoder_free(self.h)
                self.h = None
        except Exception:
            pass

    @staticmethod
    def supports(original_count, recovery_count) -> bool:
        return supports(original_count, recovery_count)

    @property
    def is_high_rate(self) -> bool:
        return bool(lib().rs16_encoder_is_high_rate(self.h))

    def reset(self, original_count, recovery_count, shard_bytes):
        self._gen += 1
        _check(lib().rs16_encoder_reset(self.h, original_count, recovery_count, shard_bytes, C.byref(self._err)),
               self._err)
        self.original_count, self.recovery_count, self.shard_bytes = original_count, recovery_count, shard_bytes

    def add_original_shard(self, shard):
        if _is_device(shard):
            p, n = _device_ptr_len(shard)
            rc = lib().rs16_encoder_add_original_shard_device(self.h, p, n, C.byref(self._err))
        else:
            p, n, keep = _host_buf(shard)
            rc = lib().rs16_encoder_add_original_shard(self.h, p, n, C.byref(self._err))
        _check(rc, self._err)

    def add_original_shard_device(self, d_shard: int, nbytes: int):
        """add_original_shard with the shard in HBM (raw device pointer)."""
        _check(lib().rs16_encoder_add_original_shard_device(self.h, d_shard, nbytes, C.byref(self._err)), self._err)

    def encode(self) -> EncoderResult:
        _check(lib().rs16_encoder_encode(self.h, C.byref(self._err)), self._err)
        return EncoderResult(self)


class RateDecoder:
    """RateDecoder<E = MI355X engine> (src/rate.rs:179-250)."""

    def __init__(self, original_count, recovery_count, shard_bytes, rate="default", engine: Optional[Engine] = None):
        self.engine = engine or default_engine()
        self._err = RS16Error()
        self._gen = 0
        self.h = lib().rs16_decoder_new(self.engine.h, _RATES[rate], original_count, recovery_count, shard_bytes,
                                        C.byref(self._err))
        if not self.h:
            raise Error._from_c(self._err)
        self.original_count, self.recovery_count, self.shard_bytes = original_count, recovery_count, shard_bytes

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().rs16_decoder_free(self.h)
                self.h = None
        except Exception:
            pass

    @staticmethod
    def supports(original_count, recovery_count) -> bool:
        return supports(original_count, recovery_count)

    @property
    def is_high_rate(self) -> bool:
        return bool(lib().rs16_decoder_is_high_rate(self.h))

    def reset(self, original_count, recovery_count, shard_bytes):
        self._gen += 1
        _check(lib().rs16_decoder_reset(self.h, original_count, recovery_count, shard_bytes, C.byref(self._err)),
               self._err)
        self.original_count, self.recovery_count, self.shard_bytes = original_count, recovery_count, shard_bytes

    def _add(self, original: bool, index, shard):
        if _is_device(shard):
            p, n = _device_ptr_len(shard)
            f = lib().rs16_decoder_add_original_shard_device if original else lib().rs16_decoder_add_recovery_shard_device
            rc = f(self.h, index, p, n, C.byref(self._err))
        else:
            p, n, keep = _host_buf(shard)
            f = lib().rs16_decoder_add_original_shard if original else lib().rs16_decoder_add_recovery_shard
            rc = f(self.h, index, p, n, C.byref(self._err))
        _check(rc, self._err)

    def add_original_shard(self, index, shard):
        self._add(True, index, shard)

    def add_recovery_shard(self, index, shard):
        self._add(False, index, shard)

    def add_original_shard_device(self, index, d_shard: int, nbytes: int):
        """add_original_shard with the shard in HBM (raw device pointer)."""
        _check(lib().rs16_decoder_add_original_shard_device(self.h, index, d_shard, nbytes, C.byref(self._err)),
               self._err)

    def add_recovery_shard_device(self, index, d_shard: int, nbytes: int):
        _check(lib().rs16_decoder_add_recovery_shard_device(self.h, index, d_shard, nbytes, C.byref(self._err)),
               self._err)

    def decode(self) -> DecoderResult:
        _check(lib().rs16_decoder_decode(self.h, C.byref(self._err)), self._err)
        return DecoderResult(self)


class ReedSolomonEncoder(RateEncoder):
    """ReedSolomonEncoder (src/reed_solomon.rs:13-85): DefaultRate + MI355X engine."""

    def __init__(self, original_count, recovery_count, shard_bytes, engine: Optional[Engine] = None):
        super().__init__(original_count, recovery_count, shard_bytes, "default", engine)


class ReedSolomonDecoder(RateDecoder):
    """ReedSolomonDecoder (src/reed_solomon.rs:93-183)."""

    def __init__(self, original_count, recovery_count, shard_bytes, engine: Optional[Engine] = None):
        super().__init__(original_count, recovery_count, shard_bytes, "default", engine)


# ---------------------------------------------------------------------------
# One-shot API (src/lib.rs:242-344)
# ---------------------------------------------------------------------------
def encode(original_count: int, recovery_count: int, original: Iterable, engine: Optional[Engine] = None):
    """reed_solomon_16::encode -> list of recovery shards (bytes)."""
    if not ReedSolomonEncoder.supports(original_count, recovery_count):
        raise Error("UnsupportedShardCount", original_count=original_count, recovery_count=recovery_count)
    it = iter(original)
    first = next(it, None)
    if first is None:
        raise Error("TooFewOriginalShards", original_count=original_count, original_received_count=0)
    enc = ReedSolomonEncoder(original_count, recovery_count, _shard_len(first), engine)
    enc.add_original_shard(first)
    for o in it:
        enc.add_original_shard(o)
    with enc.encode() as result:
        return list(result.recovery_iter())


def decode(original_count: int, recovery_count: int, original: Iterable, recovery: Iterable,
           engine: Optional[Engine] = None):
    """reed_solomon_16::decode -> {index: restored original shard (bytes)}."""
    if not ReedSolomonDecoder.supports(original_count, recovery_count):
        raise Error("UnsupportedShardCount", original_count=original_count, recovery_count=recovery_count)
    original = iter(original)
    recovery = iter(recovery)
    first = next(recovery, None)
    if first is None:
        n = sum(1 for _ in original)
        if n == original_count:
            return {}
        raise Error("NotEnoughShards", original_count=original_count, original_received_count=n,
                    recovery_received_count=0)
    dec = ReedSolomonDecoder(original_count, recovery_count, _shard_len(first[1]), engine)
    for i, o in original:
        dec.add_original_shard(i, o)
    dec.add_recovery_shard(first[0], first[1])
    for i, r in recovery:
        dec.add_recovery_shard(i, r)
    with dec.decode() as result:
        return dict(result.restored_original_iter())


# ---------------------------------------------------------------------------
# Device-resident one-shot path (the metric path; include/rs16.h)
# ---------------------------------------------------------------------------
def encode_device(original_count, recovery_count, shard_bytes, d_original, d_recovery, stream=None,
                  engine: Optional[Engine] = None):
    eng = engine or default_engine()
    err = RS16Error()
    _check(lib().rs16_encode_device(eng.h, original_count, recovery_count, shard_bytes, Engine._ptr(d_original),
                                    Engine._ptr(d_recovery), stream, C.byref(err)), err)


def encode_device_batch(original_count, recovery_count, shard_bytes, nstripes, d_original, original_stride,
                        d_recovery, recovery_stride, stream=None, engine: Optional[Engine] = None):
    """rs16_encode_device_batch: nstripes independent stripes, stripe i at
    d_original + i * original_stride / d_recovery + i * recovery_stride (bytes)."""
    eng = engine or default_engine()
    err = RS16Error()
    _check(lib().rs16_encode_device_batch(eng.h, original_count, recovery_count, shard_bytes, nstripes,
                                          Engine._ptr(d_original), original_stride, Engine._ptr(d_recovery),
                                          recovery_stride, stream, C.byref(err)), err)


def decode_device_batch(original_count, recovery_count, shard_bytes, nstripes, d_original, original_stride,
                        d_original_received, d_recovery, recovery_stride, d_recovery_received,
                        original_received_count, recovery_received_count, stream=None,
                        engine: Optional[Engine] = None):
    """rs16_decode_device_batch: nstripes stripes with one shared erasure pattern."""
    eng = engine or default_engine()
    err = RS16Error()
    _check(lib().rs16_decode_device_batch(eng.h, original_count, recovery_count, shard_bytes, nstripes,
                                          Engine._ptr(d_original), original_stride, Engine._ptr(d_original_received),
                                          Engine._ptr(d_recovery), recovery_stride, Engine._ptr(d_recovery_received),
                                          original_received_count, recovery_received_count, stream, C.byref(err)), err)


def decode_device_batch_varied(original_count, recovery_count, shard_bytes, nstripes, d_original, original_stride,
                               d_original_received, original_received_stride, d_recovery, recovery_stride,
                               d_recovery_received, recovery_received_stride, original_received_counts,
                               recovery_received_counts, stream=None, engine: Optional[Engine] = None):
    """rs16_decode_device_batch_varied: nstripes stripes, each with its own
    received flags (stripe i's at d_*_received + i * *_received_stride) and
    counts (host sequences of nstripes ints)."""
    eng = engine or default_engine()
    err = RS16Error()
    oc = (C.c_size_t * nstripes)(*[int(x) for x in original_received_counts])
    rc = (C.c_size_t * nstripes)(*[int(x) for x in recovery_received_counts])
    _check(lib().rs16_decode_device_batch_varied(
        eng.h, original_count, recovery_count, shard_bytes, nstripes, Engine._ptr(d_original), original_stride,
        Engine._ptr(d_original_received), original_received_stride, Engine._ptr(d_recovery), recovery_stride,
        Engine._ptr(d_recovery_received), recovery_received_stride, oc, rc, stream, C.byref(err)), err)


def decode_device(original_count, recovery_count, shard_bytes, d_original, d_original_received, d_recovery,
                  d_recovery_received, original_received_count, recovery_received_count, stream=None,
                  engine: Optional[Engine] = None, check: bool = False):
    """rs16_decode_device.  The received counts must equal the device flags'
    counts; check=True waits for the decode and verifies that
    (rs16_decode_check), raising InvalidArgument on a mismatch."""
    eng = engine or default_engine()
    err = RS16Error()
    _check(lib().rs16_decode_device(eng.h, original_count, recovery_count, shard_bytes, Engine._ptr(d_original),
                                    Engine._ptr(d_original_received), Engine._ptr(d_recovery),
                                    Engine._ptr(d_recovery_received), original_received_count,
                                    recovery_received_count, stream, C.byref(err)), err)
    if check:
        _check(lib().rs16_decode_check(eng.h, stream, C.byref(err)), err)


def decode_prepare(original_count, recovery_count, shard_bytes, d_original_received, d_recovery_received,
                   original_received_count, recovery_received_count, stream=None, engine: Optional[Engine] = None):
    """rs16_decode_prepare: the erasure locator of a received pattern on
    `stream`, ahead of the shards (see decode_device_prepared)."""
    eng = engine or default_engine()
    err = RS16Error()
    _check(lib().rs16_decode_prepare(eng.h, original_count, recovery_count, shard_bytes,
                                     Engine._ptr(d_original_received), Engine._ptr(d_recovery_received),
                                     original_received_count, recovery_received_count, stream, C.byref(err)), err)


def decode_device_prepared(original_count, recovery_count, shard_bytes, d_original, d_recovery, stream=None,
                           engine: Optional[Engine] = None, check: bool = False):
    """rs16_decode_device_prepared: the rest of the decode prepared last on this
    engine (same results as decode_device)."""
    eng = engine or default_engine()
    err = RS16Error()
    _check(lib().rs16_decode_device_prepared(eng.h, original_count, recovery_count, shard_bytes,
                                             Engine._ptr(d_original), Engine._ptr(d_recovery), stream, C.byref(err)),
           err)
    if check:
        _check(lib().rs16_decode_check(eng.h, stream, C.byref(err)), err)


def _host_ptr(x) -> int:
    """Address of a host buffer: an int (e.g. PinnedArray.ptr) or a C-contiguous numpy array."""
    if isinstance(x, int):
        return x
    if not x.flags["C_CONTIGUOUS"]:
        raise ValueError("host buffers must be C-contiguous")
    return x.ctypes.data


def encode_host(original_count, recovery_count, shard_bytes, h_original, h_recovery, slice_bytes=0,
                engine: Optional[Engine] = None):
    """reed_solomon_16::encode (src/lib.rs:242-279) with shards in host memory
    (rs16_encode_host: column slices pipelined over two streams)."""
    eng = engine or default_engine()
    err = RS16Error()
    _check(lib().rs16_encode_host(eng.h, original_count, recovery_count, shard_bytes, _host_ptr(h_original),
                                  _host_ptr(h_recovery), slice_bytes, C.byref(err)), err)


def decode_host(original_count, recovery_count, shard_bytes, h_original, original_received, h_recovery,
                recovery_received, slice_bytes=0, engine: Optional[Engine] = None):
    """reed_solomon_16::decode (src/lib.rs:287-344) with shards in host memory;
    lost originals are restored in place into h_original (rs16_decode_host)."""
    eng = engine or default_engine()
    err = RS16Error()
    _check(lib().rs16_decode_host(eng.h, original_count, recovery_count, shard_bytes, _host_ptr(h_original),
                                  _host_ptr(original_received), _host_ptr(h_recovery),
                                  _host_ptr(recovery_received), slice_bytes, C.byref(err)), err)


def encode_host_batch(original_count, recovery_count, shard_bytes, nstripes, h_original, original_stride,
                      h_recovery, recovery_stride, engine: Optional[Engine] = None):
    """nstripes host-resident stripes, two in flight (rs16_encode_host_batch):
    stripe i + 1's host->device copy and stripe i - 1's device->host copy
    overlap stripe i's codec."""
    eng = engine or default_engine()
    err = RS16Error()
    _check(lib().rs16_encode_host_batch(eng.h, original_count, recovery_count, shard_bytes, nstripes,
                                        _host_ptr(h_original), original_stride, _host_ptr(h_recovery),
                                        recovery_stride, C.byref(err)), err)


def decode_host_batch(original_count, recovery_count, shard_bytes, nstripes, h_original, original_stride,
                      original_received, original_received_stride, h_recovery, recovery_stride, recovery_received,
                      recovery_received_stride, engine: Optional[Engine] = None):
    """rs16_decode_host_batch: every stripe with its own host flag bytes; lost
    originals restored in place into h_original."""
    eng = engine or default_engine()
    err = RS16Error()
    _check(lib().rs16_decode_host_batch(eng.h, original_count, recovery_count, shard_bytes, nstripes,
                                        _host_ptr(h_original), original_stride, _host_ptr(original_received),
                                        original_received_stride, _host_ptr(h_recovery), recovery_stride,
                                        _host_ptr(recovery_received), recovery_received_stride, C.byref(err)), err)


def _engine_array(engines):
    arr = (C.c_void_p * len(engines))(*[e.h for e in engines])
    return arr


def encode_host_multi(original_count, recovery_count, shard_bytes, h_original, h_recovery, engines):
    """One stripe with host-resident shards, byte columns split over several
    engines (one per GPU) that run concurrently (rs16_encode_host_multi)."""
    err = RS16Error()
    _check(lib().rs16_encode_host_multi(_engine_array(engines), len(engines), original_count, recovery_count,
                                        shard_bytes, _host_ptr(h_original), _host_ptr(h_recovery), C.byref(err)), err)


def decode_host_multi(original_count, recovery_count, shard_bytes, h_original, original_received, h_recovery,
                      recovery_received, engines):
    """rs16_decode_host_multi: lost originals restored in place into h_original."""
    err = RS16Error()
    _check(lib().rs16_decode_host_multi(_engine_array(engines), len(engines), original_count, recovery_count,
                                        shard_bytes, _host_ptr(h_original), _host_ptr(original_received),
                                        _host_ptr(h_recovery), _host_ptr(recovery_received), C.byref(err)), err)


# ---------------------------------------------------------------------------
# RCCL over xGMI: byte-column scatter / gather of a stripe held by one GPU
# (include/rs16.h "RCCL over xGMI"; SURVEY.md 8(e), BASELINE configs[4])
# ---------------------------------------------------------------------------
def column_slice(shard_bytes: int, nranks: int, rank: int) -> Tuple[int, int]:
    """(byte offset, width) of rank's column slice: whole 64-byte blocks, the
    first (B mod n) ranks one block more (as rs16/columns.py)."""
    off, w = C.c_size_t(), C.c_size_t()
    if lib().rs16_column_slice(shard_bytes, nranks, rank, C.byref(off), C.byref(w)) != 0:
        raise Error("InvalidArgument")
    return off.value, w.value


class Comm:
    """One rank's RCCL communicator bound to an engine (rs16_comm)."""

    def __init__(self, engine: Engine, nranks: int = 0, rank: int = 0, unique_id: bytes = b"", _h=None):
        self.engine = engine
        self._err = RS16Error()
        if _h is not None:
            self.h = _h
        else:
            buf = C.create_string_buffer(bytes(unique_id), 128)
            self.h = lib().rs16_comm_new(engine.h, nranks, rank, buf, C.byref(self._err))
            if not self.h:
                raise Error._from_c(self._err)

    @staticmethod
    def unique_id() -> bytes:
        """The root's ncclUniqueId (128 bytes), to be shared with every rank."""
        buf = C.create_string_buffer(128)
        err = RS16Error()
        _check(lib().rs16_comm_unique_id(buf, C.byref(err)), err)
        return buf.raw

    @classmethod
    def init_all(cls, engines) -> list:
        """One communicator per engine of this process (ncclCommInitAll)."""
        arr = (C.c_void_p * len(engines))()
        err = RS16Error()
        _check(lib().rs16_comm_init_all(_engine_array(engines), len(engines), arr, C.byref(err)), err)
        return [cls(e, _h=arr[i]) for i, e in enumerate(engines)]

    @property
    def rank(self) -> int:
        return lib().rs16_comm_rank(self.h)

    @property
    def size(self) -> int:
        return lib().rs16_comm_size(self.h)

    def close(self):
        if getattr(self, "h", None):
            lib().rs16_comm_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _ptrs(xs):
    return (C.c_void_p * len(xs))(*[int(x or 0) for x in xs])


def scatter_columns(comms, root, rows, shard_bytes, d_full, d_slice, stream=None):
    """Root's rows x shard_bytes array (d_full[i] of the root's comm) -> every
    rank's contiguous rows x width column slice (d_slice[i])."""
    err = RS16Error()
    _check(lib().rs16_scatter_columns((C.c_void_p * len(comms))(*[c.h for c in comms]), len(comms), root, rows,
                                      shard_bytes, _ptrs(d_full), _ptrs(d_slice), stream, C.byref(err)), err)


def gather_columns(comms, root, rows, shard_bytes, d_slice, d_full, stream=None):
    """Every rank's column slice -> the root's rows x shard_bytes array."""
    err = RS16Error()
    _check(lib().rs16_gather_columns((C.c_void_p * len(comms))(*[c.h for c in comms]), len(comms), root, rows,
                                     shard_bytes, _ptrs(d_slice), _ptrs(d_full), stream, C.byref(err)), err)


def scatter_columns_virtual(comm, vslices, rows, shard_bytes, d_full, d_slices, stream=None):
    """Diagnostics: the multi-rank scatter on one rank -- `vslices` column
    slices all owned by comm's only rank, every slice but slice 0 through the
    staging pack and a grouped ncclSend / ncclRecv to the rank itself."""
    err = RS16Error()
    _check(lib().rs16_scatter_columns_virtual(comm.h, vslices, rows, shard_bytes, int(d_full), _ptrs(d_slices),
                                              stream, C.byref(err)), err)


def gather_columns_virtual(comm, vslices, rows, shard_bytes, d_slices, d_full, stream=None):
    """Diagnostics: the mirror image of scatter_columns_virtual (slices -> d_full)."""
    err = RS16Error()
    _check(lib().rs16_gather_columns_virtual(comm.h, vslices, rows, shard_bytes, _ptrs(d_slices), int(d_full),
                                             stream, C.byref(err)), err)
