"""ctypes binding of include/tfs_ec.h -- the GPU erasure code.

Mirrors tfs::dataserver::ErasureCode (src/dataserver/erasure_code.h): config(dn,
pn, erased) then encode(size) / decode(size) over dn + pn member buffers.  The
region work runs in libtfs_crc.so's gfx950 kernels; no CPU fallback.
"""
import ctypes


from . import crc as _crc

TFS_EXIT_NO_MEMORY = -16000
TFS_EXIT_DATA_INVALID = -16001
TFS_EXIT_SIZE_INVALID = -16002
TFS_EXIT_MATRIX_INVALID = -16003
TFS_EXIT_NO_ENOUGH_DATA = -16004
UNIT = 1024  # ws_ * ps_ (erasure_code.cpp:33-34)
EXPORTED = ["tfs_ec_config", "tfs_ec_free", "tfs_ec_encode_device", "tfs_ec_encode", "tfs_ec_decode_device",
            "tfs_ec_decode"]
_SIG = set()


def lib(L=None):
    """The library of a context (ctx.L: the product, or the measurement build
    for the TFS_EC_VARIANT forms), with the tfs_ec_* signatures set."""
    L = L or _crc.lib()
    if id(L) not in _SIG:
        vp, i32 = ctypes.c_void_p, ctypes.c_int
        for name, res, args in [
                ("tfs_ec_config", i32, [vp, i32, i32, vp, ctypes.POINTER(vp)]),
                ("tfs_ec_free", i32, [vp]),
                ("tfs_ec_encode_device", i32, [vp, vp, vp, i32, vp]),
                ("tfs_ec_encode", i32, [vp, vp, vp, i32]),
                ("tfs_ec_decode_device", i32, [vp, vp, vp, i32, vp]),
                ("tfs_ec_decode", i32, [vp, vp, vp, i32])]:
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _SIG.add(id(L))
    return L


class ErasureCode:
    """ErasureCode::config + encode/decode.  `rc` holds config's status."""

    def __init__(self, ctx, dn, pn, erased=None):
        self.ctx, self.dn, self.pn = ctx, dn, pn
        h = ctypes.c_void_p()
        e = None if erased is None else (ctypes.c_int * (dn + pn))(*erased)
        self.L = lib(ctx.L)
        self.rc = self.L.tfs_ec_config(ctx.handle, dn, pn, e, ctypes.byref(h))
        self.h = h

    @staticmethod
    def _ptrs(members):
        return (ctypes.c_void_p * len(members))(*[m if isinstance(m, int) or m is None else m.ctypes.data
                                                  for m in members])

    @staticmethod
    def _size(size):
        if not -(1 << 31) <= int(size) < (1 << 31):
            raise ValueError("ErasureCode sizes are C int (erasure_code.h): %d" % size)
        return int(size)

    @staticmethod
    def _sizes(sizes, n):
        return None if sizes is None else (ctypes.c_int * n)(*sizes)

    def encode(self, members, size, sizes=None):
        """Host members (numpy uint8 arrays, written in place for parity)."""
        return self.L.tfs_ec_encode(self.h, self._ptrs(members), self._sizes(sizes, len(members)), self._size(size))

    def decode(self, members, size, sizes=None):
        return self.L.tfs_ec_decode(self.h, self._ptrs(members), self._sizes(sizes, len(members)), self._size(size))

    def encode_device(self, d_members, size, sizes=None, stream=None):
        p = (ctypes.c_void_p * len(d_members))(*[d if isinstance(d, int) or d is None else d.ptr for d in d_members])
        return self.L.tfs_ec_encode_device(self.h, p, self._sizes(sizes, len(d_members)), self._size(size), stream)

    def decode_device(self, d_members, size, sizes=None, stream=None):
        p = (ctypes.c_void_p * len(d_members))(*[d if isinstance(d, int) or d is None else d.ptr for d in d_members])
        return self.L.tfs_ec_decode_device(self.h, p, self._sizes(sizes, len(d_members)), self._size(size), stream)

    def free(self):
        # after the context is closed its device memory is gone with it: only drop the handle
        if self.h is not None and self.h.value and self.ctx.handle is not None and self.ctx.handle.value:
            self.L.tfs_ec_free(self.h)
        self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
