"""Loader for the C-ABI library reed-solomon-16_amd/build/librs16.so.

There is no CPU fallback: if the library is missing or fails to load, every
entry point raises.  Build it with ``make -C reed-solomon-16_amd/csrc`` (or
``python -c "import __graft_entry__ as g; g.build()"``).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parents[1]
LIB_PATH = Path(os.environ.get("RS16_LIB", PKG_ROOT / "build" / "librs16.so"))


class RS16Error(C.Structure):
    _fields_ = [("code", C.c_int32), ("v0", C.c_uint64), ("v1", C.c_uint64), ("v2", C.c_uint64)]


_sz, _p, _i, _e = C.c_size_t, C.c_void_p, C.c_int, C.POINTER(RS16Error)

# name -> (restype, argtypes).  Must list every symbol of include/rs16.h
# (tests/test_cabi.py checks both directions).
SIGNATURES = {
    "rs16_error_message": (_sz, [_e, C.c_char_p, _sz]),
    "rs16_version": (C.c_char_p, []),
    "rs16_host_mul": (None, [_p, _p, _sz, C.c_uint16]),
    "rs16_engine_set_profiling": (_i, [_p, _i, _e]),
    "rs16_engine_profile_read": (_i, [_p, _i, C.POINTER(C.c_double), C.POINTER(C.c_uint64), _e]),
    "rs16_engine_profile_reset": (None, [_p]),
    "rs16_prog_count": (_i, []),
    "rs16_engine_set_diagnostics": (_i, [_p, _i]),
    "rs16_prog_name": (C.c_char_p, [_i]),
    "rs16_engine_set_stamps": (_i, [_p, _p, _i, _e]),
    "rs16_engine_set_slices": (_i, [_p, _i, _e]),
    "rs16_engine_new": (_p, [_i, _e]),
    "rs16_engine_new_ex": (_p, [_i, _i, _e]),
    "rs16_set_diagnostics": (_i, [_i]),
    "rs16_engine_free": (None, [_p]),
    "rs16_engine_device": (_i, [_p]),
    "rs16_engine_stream": (_p, [_p]),
    "rs16_engine_synchronize": (_i, [_p, _p, _e]),
    "rs16_engine_fft": (_i, [_p, _p, _sz, _sz, _sz, _sz, _sz, _sz, _p, _e]),
    "rs16_engine_fft_skew_end": (_i, [_p, _p, _sz, _sz, _sz, _sz, _sz, _p, _e]),
    "rs16_engine_ifft": (_i, [_p, _p, _sz, _sz, _sz, _sz, _sz, _sz, _p, _e]),
    "rs16_engine_ifft_skew_end": (_i, [_p, _p, _sz, _sz, _sz, _sz, _sz, _p, _e]),
    "rs16_engine_fwht": (_i, [_p, _p, _sz, _p, _e]),
    "rs16_engine_eval_poly": (_i, [_p, _p, _sz, _p, _e]),
    "rs16_engine_mul": (_i, [_p, _p, _sz, C.c_uint16, _p, _e]),
    "rs16_engine_xor": (_i, [_p, _p, _p, _sz, _p, _e]),
    "rs16_engine_xor_within": (_i, [_p, _p, _sz, _sz, _sz, _sz, _sz, _p, _e]),
    "rs16_engine_formal_derivative": (_i, [_p, _p, _sz, _sz, _p, _e]),
    "rs16_supports": (_i, [_i, _sz, _sz]),
    "rs16_validate": (_i, [_i, _sz, _sz, _sz, _e]),
    "rs16_use_high_rate": (_i, [_sz, _sz, _e]),
    "rs16_encoder_work_count": (_sz, [_i, _sz, _sz]),
    "rs16_decoder_work_count": (_sz, [_i, _sz, _sz]),
    "rs16_encoder_new": (_p, [_p, _i, _sz, _sz, _sz, _e]),
    "rs16_encoder_free": (None, [_p]),
    "rs16_encoder_reset": (_i, [_p, _sz, _sz, _sz, _e]),
    "rs16_encoder_add_original_shard": (_i, [_p, _p, _sz, _e]),
    "rs16_encoder_add_original_shard_device": (_i, [_p, _p, _sz, _e]),
    "rs16_encoder_encode": (_i, [_p, _e]),
    "rs16_encoder_recovery": (_p, [_p, _sz, _e]),
    "rs16_encoder_recovery_device": (_p, [_p, _sz]),
    "rs16_encoder_recovery_copy": (_i, [_p, _sz, _p, _sz, _e]),
    "rs16_encoder_result_drop": (None, [_p]),
    "rs16_encoder_is_high_rate": (_i, [_p]),
    "rs16_decoder_new": (_p, [_p, _i, _sz, _sz, _sz, _e]),
    "rs16_decoder_free": (None, [_p]),
    "rs16_decoder_reset": (_i, [_p, _sz, _sz, _sz, _e]),
    "rs16_decoder_add_original_shard": (_i, [_p, _sz, _p, _sz, _e]),
    "rs16_decoder_add_recovery_shard": (_i, [_p, _sz, _p, _sz, _e]),
    "rs16_decoder_add_original_shard_device": (_i, [_p, _sz, _p, _sz, _e]),
    "rs16_decoder_add_recovery_shard_device": (_i, [_p, _sz, _p, _sz, _e]),
    "rs16_decoder_decode": (_i, [_p, _e]),
    "rs16_decoder_restored_original": (_p, [_p, _sz, _e]),
    "rs16_decoder_restored_original_device": (_p, [_p, _sz]),
    "rs16_decoder_restored_original_copy": (_i, [_p, _sz, _p, _sz, _e]),
    "rs16_decoder_result_drop": (None, [_p]),
    "rs16_decoder_is_high_rate": (_i, [_p]),
    "rs16_encode_device": (_i, [_p, _sz, _sz, _sz, _p, _p, _p, _e]),
    "rs16_encode_device_batch": (_i, [_p, _sz, _sz, _sz, _sz, _p, _sz, _p, _sz, _p, _e]),
    "rs16_decode_device_batch": (_i, [_p, _sz, _sz, _sz, _sz, _p, _sz, _p, _p, _sz, _p, _sz, _sz, _p, _e]),
    "rs16_decode_device_batch_varied": (_i, [_p, _sz, _sz, _sz, _sz, _p, _sz, _p, _sz, _p, _sz, _p, _sz, _p, _p, _p,
                                             _e]),
    "rs16_decode_device": (_i, [_p, _sz, _sz, _sz, _p, _p, _p, _p, _sz, _sz, _p, _e]),
    "rs16_decode_check": (_i, [_p, _p, _e]),
    "rs16_device_alloc": (_p, [_p, _sz, _e]),
    "rs16_device_free": (None, [_p, _p]),
    "rs16_memcpy_htod": (_i, [_p, _p, _p, _sz, _p, _e]),
    "rs16_memcpy_dtoh": (_i, [_p, _p, _p, _sz, _p, _e]),
    "rs16_memset_device": (_i, [_p, _p, _i, _sz, _p, _e]),
    "rs16_encode_host": (_i, [_p, _sz, _sz, _sz, _p, _p, _sz, _e]),
    "rs16_decode_host": (_i, [_p, _sz, _sz, _sz, _p, _p, _p, _p, _sz, _e]),
    "rs16_host_alloc": (_p, [_p, _sz, _e]),
    "rs16_comm_unique_id": (_i, [_p, _e]),
    "rs16_comm_new": (_p, [_p, _i, _i, _p, _e]),
    "rs16_comm_init_all": (_i, [_p, _i, _p, _e]),
    "rs16_comm_free": (None, [_p]),
    "rs16_comm_rank": (_i, [_p]),
    "rs16_comm_size": (_i, [_p]),
    "rs16_column_slice": (_i, [_sz, _i, _i, C.POINTER(_sz), C.POINTER(_sz)]),
    "rs16_scatter_columns": (_i, [_p, _i, _i, _sz, _sz, _p, _p, _p, _e]),
    "rs16_gather_columns": (_i, [_p, _i, _i, _sz, _sz, _p, _p, _p, _e]),
    "rs16_scatter_columns_virtual": (_i, [_p, _i, _sz, _sz, _p, _p, _p, _e]),
    "rs16_gather_columns_virtual": (_i, [_p, _i, _sz, _sz, _p, _p, _p, _e]),
    "rs16_encode_host_multi": (_i, [_p, _i, _sz, _sz, _sz, _p, _p, _e]),
    "rs16_decode_prepare": (_i, [_p, _sz, _sz, _sz, _p, _p, _sz, _sz, _p, _e]),
    "rs16_decode_device_prepared": (_i, [_p, _sz, _sz, _sz, _p, _p, _p, _e]),
    "rs16_encode_host_batch": (_i, [_p, _sz, _sz, _sz, _sz, _p, _sz, _p, _sz, _e]),
    "rs16_decode_host_batch": (_i, [_p, _sz, _sz, _sz, _sz, _p, _sz, _p, _sz, _p, _sz, _p, _sz, _e]),
    "rs16_decode_host_multi": (_i, [_p, _i, _sz, _sz, _sz, _p, _p, _p, _p, _e]),
    "rs16_stream_create": (_p, [_p, _e]),
    "rs16_stream_destroy": (None, [_p, _p]),
    "rs16_host_free": (None, [_p, _p]),
}

_lib = None


def lib():
    """Load librs16.so (raises OSError if it is missing: no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise OSError(f"rs16: native library not built: {LIB_PATH} (run make -C reed-solomon-16_amd/csrc)")
        L = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


def hip_runtime():
    """The HIP runtime librs16.so runs on, for the few direct HIP calls of the
    diagnostics (events in bench.py).  A process that imported torch holds a
    second libamdhip64 (torch's bundled copy, soname libamdhip64.so): loading
    "libamdhip64.so" by name resolves to that one, which does not share
    librs16's device context (hipGetDevice there fails with 100).  This
    returns the mapped copy that is not torch's."""
    lib()
    with open("/proc/self/maps") as maps:
        for line in maps:
            path = line.split()[-1] if "/" in line else ""
            if "libamdhip64" in path and "/torch/" not in path:
                return C.CDLL(path)
    return C.CDLL("libamdhip64.so")
