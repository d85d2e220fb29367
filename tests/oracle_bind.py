"""ctypes binding of the CPU oracle (oracle/rs16_oracle.c).

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module.  The product (reed-solomon-16_amd/)
never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE_DIR = ROOT / "oracle"
LIB_PATH = ORACLE_DIR / "build" / "librs16_oracle.so"

RATE = {"default": 0, "high": 1, "low": 2}
ENGINE = {"naive": 0, "nosimd": 1}


class OracleError(C.Structure):
    _fields_ = [("code", C.c_int32), ("a", C.c_uint64), ("b", C.c_uint64), ("c", C.c_uint64)]


def build():
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        sz, p, e = C.c_size_t, C.c_void_p, C.POINTER(OracleError)
        sig = {
            "oracle_init": (None, []),
            "oracle_use_high_rate": (C.c_int, [sz, sz, e]),
            "oracle_supports": (C.c_int, [C.c_int, sz, sz]),
            "oracle_validate": (C.c_int, [C.c_int, sz, sz, sz, e]),
            "oracle_encoder_work_count": (sz, [C.c_int, sz, sz]),
            "oracle_decoder_work_count": (sz, [C.c_int, sz, sz]),
            "oracle_encoder_new": (p, [C.c_int, C.c_int, sz, sz, sz, e]),
            "oracle_encoder_reset": (C.c_int, [p, sz, sz, sz, e]),
            "oracle_encoder_free": (None, [p]),
            "oracle_encoder_add_original_shard": (C.c_int, [p, p, sz, e]),
            "oracle_encoder_encode": (C.c_int, [p, e]),
            "oracle_encoder_recovery": (p, [p, sz]),
            "oracle_encoder_reset_received": (None, [p]),
            "oracle_decoder_new": (p, [C.c_int, C.c_int, sz, sz, sz, e]),
            "oracle_decoder_reset": (C.c_int, [p, sz, sz, sz, e]),
            "oracle_decoder_free": (None, [p]),
            "oracle_decoder_add_original_shard": (C.c_int, [p, sz, p, sz, e]),
            "oracle_decoder_add_recovery_shard": (C.c_int, [p, sz, p, sz, e]),
            "oracle_decoder_decode": (C.c_int, [p, e]),
            "oracle_decoder_restored_original": (p, [p, sz]),
            "oracle_decoder_reset_received": (None, [p]),
            "oracle_fft": (None, [C.c_int, p, sz, sz, sz, sz, sz]),
            "oracle_ifft": (None, [C.c_int, p, sz, sz, sz, sz, sz]),
            "oracle_fwht": (None, [C.c_int, p, sz]),
            "oracle_eval_poly": (None, [C.c_int, p, sz]),
            "oracle_mul": (None, [C.c_int, p, sz, C.c_uint16]),
            "oracle_formal_derivative": (None, [C.c_int, p, sz, sz]),
            "oracle_table": (C.POINTER(C.c_uint16), [C.c_int]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        L.oracle_init()
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Error(Exception):
    def __init__(self, e: OracleError):
        self.code, self.vals = e.code, (e.a, e.b, e.c)
        super().__init__(f"oracle error {e.code} {self.vals}")


def _check(rc, err):
    if rc != 0:
        raise Error(err)


class Encoder:
    """Oracle RateEncoder (src/rate.rs:113-173)."""

    def __init__(self, rate, engine, k, m, sb):
        self.err = OracleError()
        self.h = lib().oracle_encoder_new(RATE[rate], ENGINE[engine], k, m, sb, C.byref(self.err))
        if not self.h:
            raise Error(self.err)
        self.m, self.sb = m, sb

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_encoder_free(self.h)

    def reset(self, k, m, sb):
        _check(lib().oracle_encoder_reset(self.h, k, m, sb, C.byref(self.err)), self.err)
        self.m, self.sb = m, sb

    def add_original_shard(self, shard):
        a = np.ascontiguousarray(np.frombuffer(bytes(shard), np.uint8)) if not isinstance(shard, np.ndarray) else np.ascontiguousarray(shard)
        _check(lib().oracle_encoder_add_original_shard(self.h, _ptr(a), a.size, C.byref(self.err)), self.err)

    def encode(self):
        _check(lib().oracle_encoder_encode(self.h, C.byref(self.err)), self.err)
        out = np.empty((self.m, self.sb), np.uint8)
        for i in range(self.m):
            p = lib().oracle_encoder_recovery(self.h, i)
            C.memmove(out[i].ctypes.data, p, self.sb)
        lib().oracle_encoder_reset_received(self.h)  # EncoderResult dropped
        return out


class Decoder:
    """Oracle RateDecoder (src/rate.rs:179-250)."""

    def __init__(self, rate, engine, k, m, sb):
        self.err = OracleError()
        self.h = lib().oracle_decoder_new(RATE[rate], ENGINE[engine], k, m, sb, C.byref(self.err))
        if not self.h:
            raise Error(self.err)
        self.k, self.sb = k, sb

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_decoder_free(self.h)

    def reset(self, k, m, sb):
        _check(lib().oracle_decoder_reset(self.h, k, m, sb, C.byref(self.err)), self.err)
        self.k, self.sb = k, sb

    def add_original_shard(self, i, shard):
        a = np.ascontiguousarray(shard, dtype=np.uint8)
        _check(lib().oracle_decoder_add_original_shard(self.h, i, _ptr(a), a.size, C.byref(self.err)), self.err)

    def add_recovery_shard(self, i, shard):
        a = np.ascontiguousarray(shard, dtype=np.uint8)
        _check(lib().oracle_decoder_add_recovery_shard(self.h, i, _ptr(a), a.size, C.byref(self.err)), self.err)

    def decode(self):
        """Returns {index: restored original shard}, then drops the result."""
        _check(lib().oracle_decoder_decode(self.h, C.byref(self.err)), self.err)
        out = {}
        for i in range(self.k):
            p = lib().oracle_decoder_restored_original(self.h, i)
            if p:
                buf = np.empty(self.sb, np.uint8)
                C.memmove(buf.ctypes.data, p, self.sb)
                out[i] = buf
        lib().oracle_decoder_reset_received(self.h)
        return out


def encode(k, m, original, rate="default", engine="nosimd"):
    enc = Encoder(rate, engine, k, m, original.shape[1])
    for s in original:
        enc.add_original_shard(s)
    return enc.encode()


# ---- engine-level ops (in place on numpy arrays) ----
def fft(data, pos, size, trunc, skew_delta, engine="nosimd"):
    lib().oracle_fft(ENGINE[engine], _ptr(data), data.shape[1], pos, size, trunc, skew_delta)


def ifft(data, pos, size, trunc, skew_delta, engine="nosimd"):
    lib().oracle_ifft(ENGINE[engine], _ptr(data), data.shape[1], pos, size, trunc, skew_delta)


def fwht(data_u16, trunc, engine="nosimd"):
    lib().oracle_fwht(ENGINE[engine], _ptr(data_u16), trunc)


def eval_poly(e_u16, trunc, engine="nosimd"):
    lib().oracle_eval_poly(ENGINE[engine], _ptr(e_u16), trunc)


def mul(x, log_m, engine="nosimd"):
    lib().oracle_mul(ENGINE[engine], _ptr(x), x.size, log_m)


def formal_derivative(data, engine="nosimd"):
    lib().oracle_formal_derivative(ENGINE[engine], _ptr(data), data.shape[1], data.shape[0])


def table(name):
    idx = {"exp": 0, "log": 1, "skew": 2, "log_walsh": 3}[name]
    n = 65535 if name == "skew" else 65536
    return np.ctypeslib.as_array(lib().oracle_table(idx), shape=(n,)).copy()
