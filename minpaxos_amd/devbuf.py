"""Device buffers, streams and events through the engine's own HIP runtime (mpx_dev_alloc & co).

The bench and the device-pointer tests stage their HBM-resident inputs with these helpers, so the
engine, its kernels, its RCCL communicator and the caller's buffers all live in the one HIP
runtime libmpx.so is bound to (reported by `_lib.runtime_info()`), whatever else the process
has loaded (torch brings a HIP runtime of its own; it is never used for device work here).
"""
import ctypes as C

import numpy as np

H2D, D2H, D2D = 1, 2, 3


class DevArray:
    """a device allocation with the numpy dtype / shape it holds"""

    def __init__(self, ptr, nbytes, dtype, shape):
        self.ptr, self.nbytes, self.dtype, self.shape = ptr, nbytes, np.dtype(dtype), shape

    def at(self, index):
        """device pointer of element `index` (for sub-ranges of the buffer)"""
        return self.ptr + int(index) * self.dtype.itemsize

    @property
    def size(self):
        return int(np.prod(self.shape)) if self.shape else 1


class Arena:
    """allocations of one engine, freed together (close / context manager)"""

    def __init__(self, eng):
        self.eng = eng
        self.live = []

    def empty(self, shape, dtype):
        shape = (shape,) if np.isscalar(shape) else tuple(shape)
        dt = np.dtype(dtype)
        nbytes = int(np.prod(shape)) * dt.itemsize
        p = self.eng.dev_alloc(max(nbytes, 16))
        self.live.append(p)
        return DevArray(p, nbytes, dt, shape)

    def put(self, a, stream=None):
        """copy a host array to a new device buffer (synchronous on `stream`)"""
        a = np.ascontiguousarray(a)
        d = self.empty(a.shape, a.dtype)
        if a.nbytes:
            self.eng.memcpy(d.ptr, a.ctypes.data_as(C.c_void_p), a.nbytes, H2D, stream)
            self.eng.stream_synchronize(stream)
        return d

    def full(self, shape, dtype, byte_value, stream=None):
        d = self.empty(shape, dtype)
        self.eng.memset(d.ptr, byte_value, d.nbytes, stream)
        return d

    def get(self, d, count=None, offset=0, stream=None):
        """device buffer (or `count` elements from `offset`) back to a new host array"""
        n = d.size if count is None else int(count)
        out = np.empty(n, d.dtype)
        if out.nbytes:
            self.eng.memcpy(out.ctypes.data_as(C.c_void_p), d.at(offset), out.nbytes, D2H, stream)
            self.eng.stream_synchronize(stream)
        if count is None and len(d.shape) > 1:
            out = out.reshape(d.shape)
        return out

    def close(self):
        for p in self.live:
            self.eng.dev_free(p)
        self.live = []

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
