"""ctypes binding of the C++/OpenMP fp32 CPU baseline (voxcpu.cpp).  Oracle
side: bench.py's cpu_baseline leg and tests only."""
import ctypes as C
import os

from .build import LIB

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run oracle/cpu/build.py (or __graft_entry__.build())")
        h = C.CDLL(LIB)
        h.voxcpu_load.restype = C.c_int
        h.voxcpu_load.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]
        h.voxcpu_embed.restype = C.c_int
        h.voxcpu_embed.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                   C.c_int]
        h.voxcpu_dim.restype = C.c_int
        h.voxcpu_dim.argtypes = [C.c_void_p]
        h.voxcpu_free.argtypes = [C.c_void_p]
        h.voxcpu_last_error.restype = C.c_char_p
        h.voxcpu_max_threads.restype = C.c_int
        _lib = h
    return _lib


class CpuModel:
    def __init__(self, blob):
        import numpy as np  # noqa: F401
        self._buf = C.create_string_buffer(bytes(blob), len(blob))
        h = C.c_void_p()
        if lib().voxcpu_load(self._buf, len(blob), C.byref(h)) != 0:
            raise RuntimeError(lib().voxcpu_last_error().decode())
        self._h = h
        self.dim = lib().voxcpu_dim(h)

    def run(self, x, threads=0):
        import numpy as np
        x = np.ascontiguousarray(x, np.float32)
        n, t, f = x.shape
        out = np.empty((n, self.dim), np.float32)
        if lib().voxcpu_embed(self._h, x.ctypes.data, n, t, f, out.ctypes.data, int(threads)) != 0:
            raise RuntimeError(lib().voxcpu_last_error().decode())
        return out

    def close(self):
        if getattr(self, "_h", None):
            lib().voxcpu_free(self._h)
            self._h = None

    def __del__(self):
        self.close()
