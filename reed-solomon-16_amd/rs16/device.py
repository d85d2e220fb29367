"""Device buffers through the rs16 C ABI (so callers need neither torch nor HIP headers)."""
import ctypes as C

import numpy as np

from . import Engine, Error
from ._lib import RS16Error, lib


class DeviceArray:
    def __init__(self, engine: Engine, nbytes: int):
        self.engine, self.nbytes = engine, nbytes
        err = RS16Error()
        self.ptr = lib().rs16_device_alloc(engine.h, max(nbytes, 1), C.byref(err))
        if not self.ptr:
            raise Error._from_c(err)

    @classmethod
    def from_numpy(cls, engine, a: np.ndarray):
        a = np.ascontiguousarray(a)
        d = cls(engine, a.nbytes)
        d.upload(a)
        return d

    def upload(self, a: np.ndarray):
        a = np.ascontiguousarray(a)
        err = RS16Error()
        if lib().rs16_memcpy_htod(self.engine.h, self.ptr, a.ctypes.data_as(C.c_void_p), a.nbytes, None, C.byref(err)):
            raise Error._from_c(err)

    def download(self, dtype=np.uint8, shape=None) -> np.ndarray:
        self.engine.synchronize()
        out = np.empty(self.nbytes, np.uint8)
        err = RS16Error()
        if lib().rs16_memcpy_dtoh(self.engine.h, out.ctypes.data_as(C.c_void_p), self.ptr, self.nbytes, None, C.byref(err)):
            raise Error._from_c(err)
        out = out.view(dtype)
        return out.reshape(shape) if shape is not None else out

    def offset(self, nbytes: int) -> int:
        return self.ptr + nbytes

    def __del__(self):
        try:
            if self.ptr and self.engine.h:  # engine closed first (interpreter exit): leave it to the runtime
                lib().rs16_device_free(self.engine.h, self.ptr)
        except Exception:
            pass


class PinnedArray:
    """Page-locked host buffer (rs16_host_alloc) viewed as a numpy uint8 array."""

    def __init__(self, engine: Engine, nbytes: int):
        self.engine, self.nbytes = engine, nbytes
        err = RS16Error()
        self.ptr = lib().rs16_host_alloc(engine.h, max(nbytes, 1), C.byref(err))
        if not self.ptr:
            raise Error._from_c(err)
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(nbytes, 1)).from_address(self.ptr))[:nbytes]

    def to_device(self, d: "DeviceArray", nbytes: int = None):
        err = RS16Error()
        if lib().rs16_memcpy_htod(self.engine.h, d.ptr, self.ptr, self.nbytes if nbytes is None else nbytes, None,
                                  C.byref(err)):
            raise Error._from_c(err)

    def from_device(self, d: "DeviceArray", nbytes: int = None):
        err = RS16Error()
        if lib().rs16_memcpy_dtoh(self.engine.h, self.ptr, d.ptr, self.nbytes if nbytes is None else nbytes, None,
                                  C.byref(err)):
            raise Error._from_c(err)

    def __del__(self):
        try:
            if self.ptr and self.engine.h:
                self.array = None
                lib().rs16_host_free(self.engine.h, self.ptr)
        except Exception:
            pass
