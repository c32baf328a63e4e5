"""tfs_amd -- MI355X-native per-file CRC32 integrity path of TFS's dataserver.

Product: libtfs_crc.so (C ABI, include/tfs_crc.h) = hand-written gfx950 HIP
kernels (csrc/tfs_crc_kernels.hip) + host runtime (csrc/tfs_crc_abi.cpp).
`tfs_amd.crc` is its ctypes binding; it raises if the library is missing.
"""
__all__ = ["crc", "synth"]
