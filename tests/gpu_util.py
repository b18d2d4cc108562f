"""Device buffers for GPU tests, through the C ABI's own allocator (no torch)."""
import ctypes as C

import numpy as np

from immustore_amd import _native as N


class DevBuf:
    def __init__(self, ctx, nbytes):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        N.check(N.load().mh_dev_alloc(ctx.handle, max(self.nbytes, 1), C.byref(p)))
        self.ptr = p.value

    @classmethod
    def from_host(cls, ctx, arr):
        a = np.ascontiguousarray(arr)
        b = cls(ctx, a.nbytes)
        if a.nbytes:
            N.check(N.load().mh_memcpy_h2d(ctx.handle, b.ptr, a.ctypes.data, a.nbytes))
            ctx.synchronize()
        return b

    def to_host(self, dtype=np.uint8, count=None):
        count = self.nbytes // np.dtype(dtype).itemsize if count is None else count
        out = np.zeros(max(count, 1), dtype)
        nb = count * np.dtype(dtype).itemsize
        if nb:
            N.check(N.load().mh_memcpy_d2h(self.ctx.handle, out.ctypes.data, self.ptr, nb))
            self.ctx.synchronize()
        return out[:count]

    def free(self):
        if self.ptr:
            N.load().mh_dev_free(self.ctx.handle, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
