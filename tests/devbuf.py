"""Minimal device buffers for tests that drive the device-pointer entry points of the C ABI
without torch (hipMalloc / hipMemcpy through ctypes on the HIP runtime)."""
import ctypes as C

import numpy as np

_hip = C.CDLL("libamdhip64.so")
_hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
_hip.hipFree.argtypes = [C.c_void_p]
_hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
_hip.hipDeviceSynchronize.argtypes = []
H2D, D2H = 1, 2


class DeviceArray:
    def __init__(self, n):
        self.n = int(n)
        self.p = C.c_void_p()
        rc = _hip.hipMalloc(C.byref(self.p), max(self.n, 1) * 8)
        if rc != 0:
            raise RuntimeError(f"hipMalloc failed ({rc})")

    @classmethod
    def of(cls, a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        d = cls(a.size)
        if a.size and _hip.hipMemcpy(d.p, a.ctypes.data, a.size * 8, H2D) != 0:
            raise RuntimeError("hipMemcpy H2D failed")
        return d

    def numpy(self):
        _hip.hipDeviceSynchronize()
        out = np.empty(self.n)
        if self.n and _hip.hipMemcpy(out.ctypes.data, self.p, self.n * 8, D2H) != 0:
            raise RuntimeError("hipMemcpy D2H failed")
        return out

    def __del__(self):
        if getattr(self, "p", None):
            _hip.hipFree(self.p)
            self.p = None
