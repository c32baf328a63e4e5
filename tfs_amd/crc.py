"""ctypes binding of the C ABI in include/tfs_crc.h (libtfs_crc.so, built in-tree).

The native library is the product: every function here calls into the gfx950
kernels through the C ABI.  There is no Python or CPU fallback -- if the
library is missing this module raises on import, and if no gfx950 device is
present the calls return TFS_CRC_EXIT_NO_DEVICE and raise TfsCrcError.

Names mirror the reference interface they replace:
  func_crc(seed, data)        tfs::common::Func::crc   src/common/func.h:90, func.cpp:426-435
  Context.batch / verify      the per-file call sites   data_file.cpp:190, sync_backup.cpp:383/429
  Context.block_verify        verify-on-read of a block sync_backup.cpp:345-435, block_console.cpp:543-577
  Context.block_compact       CompactTask::real_compact task.cpp:713-836 (+ re-CRC verify)
  Context.packet_verify/seal  BasePacket::decode / copy+reply  base_packet.cpp:74,141,208
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libtfs_crc.so")  # the product: one form of each kernel
# The measurement build (-DTFS_CRC_MEASURE): the A/B kernel forms selected by
# TFS_CRC_VARIANT / TFS_EC_VARIANT and the calibration kernels.  Loaded only
# for a Context(measure=True) or when TFS_CRC_VARIANT / TFS_EC_VARIANT is set
# (A/B tools, variant parity tests); TFS_CRC_LIB points it at another build
# (an old commit) for an A/B.  The product library never reads those variables.
MEASURE_LIB_PATH = os.environ.get("TFS_CRC_LIB") or os.path.join(HERE, "libtfs_crc_measure.so")

TFS_SUCCESS = 0
TFS_EXIT_CHECK_CRC_ERROR = -1010
TFS_EXIT_PARAMETER_ERROR = -1016
TFS_EXIT_DATA_FILE_ERROR = -8013
TFS_EXIT_FILE_INFO_ERROR = -8016
TFS_EXIT_READ_FILE_SIZE_ERROR = -8034
TFS_EXIT_SYNC_FILE_ERROR = -8038
TFS_CRC_EXIT_DEVICE_ERROR = -20001
TFS_CRC_EXIT_NO_DEVICE = -20002

TFS_ERROR = -1
TFS_PACKET_INCOMPLETE = 1
TFS_PACKET_FLAG_V0 = 0x4D534654
TFS_PACKET_FLAG_V1 = 0x4E534654
PACKET_HEADER_V0_SIZE, PACKET_HEADER_V1_SIZE = 12, 24

FI_DELETED, FI_INVALID, FI_CONCEAL = 1, 2, 4
FILEINFO_SIZE = 36

DESC_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("aux", "<u4")])  # tfs_crc_desc / tfs_crc_vdesc
PACKET_DESC_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("reserved", "<u4")])  # tfs_packet_desc
COMPACT_JOB_DTYPE = np.dtype([("src_offset", "<u8"), ("dest_offset", "<u8"), ("file_id", "<u8"), ("size", "<i4"),
                              ("flag", "<i4"), ("new_offset", "<i4"), ("reserved", "<i4")])  # tfs_compact_job
META_DTYPE = np.dtype([("file_id", "<u8"), ("offset", "<i4"), ("size", "<i4")])  # tfs_raw_meta
FILEINFO_DTYPE = np.dtype([("id_", "<u8"), ("offset_", "<i4"), ("size_", "<i4"), ("usize_", "<i4"),
                           ("modify_time_", "<i4"), ("create_time_", "<i4"), ("flag_", "<i4"),
                           ("crc_", "<u4")], align=False)
assert DESC_DTYPE.itemsize == 16 and META_DTYPE.itemsize == 16 and FILEINFO_DTYPE.itemsize == 36

# Every symbol include/tfs_crc.h and include/tfs_crc_testing.h declare (checked by
# tests/test_abi.py).
EXPORTED = [
    "tfs_crc32_ctx_create", "tfs_crc32_ctx_destroy", "tfs_crc32_last_error", "tfs_crc32_device_count",
    "tfs_crc32_device_numa_node",
    "tfs_crc32", "tfs_crc32_e", "tfs_datafile_get_crc", "tfs_crc32_batch", "tfs_crc32_verify",
    "tfs_crc32_batch_device", "tfs_crc32_verify_device", "tfs_crc32_submit_verify", "tfs_crc32_wait",
    "tfs_block_verify", "tfs_block_verify_device", "tfs_block_compact", "tfs_blocks_compact",
    "tfs_crc32_synth_fill_device", "tfs_crc32_write_headers_device", "tfs_crc32_membench_device",
    "tfs_crc32_dev_malloc", "tfs_crc32_dev_free", "tfs_crc32_host_malloc_pinned", "tfs_crc32_host_free_pinned",
    "tfs_crc32_host_device_ptr",
    "tfs_crc32_memcpy", "tfs_crc32_memset_device", "tfs_crc32_event_create", "tfs_crc32_event_record",
    "tfs_crc32_event_elapsed_ms", "tfs_crc32_event_destroy",
    "tfs_crc32_stream", "tfs_crc32_sync", "tfs_crc32_stream_create", "tfs_crc32_stream_sync",
    "tfs_crc32_stream_destroy", "tfs_crc32_inject_device_error", "tfs_crc32_set_resident",
    "tfs_crc32_resident_stats", "tfs_crc32_resident_ring_in_device_memory", "tfs_crc32_stats", "tfs_crc32_res_trace", "tfs_crc32_res_trace_last", "tfs_crc32_error_count", "tfs_crc32_set_default_ctx", "tfs_crc32_bind_thread",
    "tfs_crc32_default_ctx", "tfs_crc32_set_cu_reserve", "tfs_crc32_throughput_grid", "tfs_crc32_sched_stats", "tfs_crc32_plan_stats",
    "tfs_crc32_debug_state", "tfs_crc32_debug_poison_resident",
    "tfs_crc32_set_split", "tfs_crc32_split_stats", "tfs_crc32_set_compact_segment",
    "tfs_crc_group_create", "tfs_crc_group_destroy", "tfs_crc_group_last_error", "tfs_crc_group_size",
    "tfs_crc_group_ctx", "tfs_crc_group_member_of", "tfs_crc_group_ctx_for_block", "tfs_crc_group_numa_node",
    "tfs_crc_group_member_bound", "tfs_crc_group_host_malloc", "tfs_crc_group_host_free",
    "tfs_crc_group_blocks_verify", "tfs_crc_group_blocks_compact", "tfs_blocks_verify_device",
    "tfs_packet_verify", "tfs_packet_verify_device", "tfs_packet_seal", "tfs_packet_seal_device",
    "tfs_crc32_write_packet_headers_device", "tfs_block_compact_device", "tfs_compact_jobs_device",
]


class BlockJob(ctypes.Structure):
    """tfs_block_job (include/tfs_crc.h)."""
    _fields_ = [("src_image", ctypes.c_void_p), ("src_len", ctypes.c_uint64), ("metas", ctypes.c_void_p),
                ("flags", ctypes.c_void_p), ("n", ctypes.c_uint32), ("dest_image", ctypes.c_void_p),
                ("dest_cap", ctypes.c_uint64), ("dest_metas", ctypes.c_void_p), ("crc_ok", ctypes.c_void_p),
                ("dest_len", ctypes.c_uint64), ("n_live", ctypes.c_uint32), ("status", ctypes.c_int)]


class CrcStats(ctypes.Structure):
    """tfs_crc_stats (include/tfs_crc.h)."""
    _fields_ = [(k, ctypes.c_uint64) for k in (
        "host_calls", "host_files", "lone_calls", "lone_small_calls", "lone_small_bytes", "resident_launches",
        "resident_files", "resident_ring_full")]


LONE_CROSSOVER = 3500  # TFS_CRC_LONE_CROSSOVER


class TfsCrcError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (code %d)" % (msg, code))
        self.code = code


_LIBS = {}


def measuring():
    """True when this process asked for a measurement kernel form."""
    return os.environ.get("TFS_CRC_VARIANT", "0") not in ("", "0") or \
        os.environ.get("TFS_EC_VARIANT", "0") not in ("", "0")


def lib(measure=False):
    """Load libtfs_crc.so (or the measurement build); raise loudly when it is
    missing (no fallback)."""
    path = MEASURE_LIB_PATH if measure else LIB_PATH
    if path not in _LIBS:
        if not os.path.exists(path):
            raise ImportError("tfs_amd native library not built: %s (run __graft_entry__.build())" % path)
        L = ctypes.CDLL(path)
        vp, u32, i32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64
        sig = {
            "tfs_crc32_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
            "tfs_crc32_ctx_destroy": (ctypes.c_int, [vp]),
            "tfs_crc32_last_error": (ctypes.c_char_p, [vp]),
            "tfs_crc32_device_count": (ctypes.c_int, []),
            "tfs_crc32_device_numa_node": (ctypes.c_int, [ctypes.c_int]),
            "tfs_crc32": (u32, [u32, ctypes.c_char_p, i32]),
            "tfs_crc32_e": (u32, [u32, ctypes.c_char_p, i32, ctypes.POINTER(ctypes.c_int)]),
            "tfs_datafile_get_crc": (ctypes.c_int, [vp, ctypes.c_char_p, i32, ctypes.POINTER(u32)]),
            "tfs_crc32_batch": (ctypes.c_int, [vp, vp, u32, vp, u64, vp]),
            "tfs_crc32_verify": (ctypes.c_int, [vp, vp, u32, vp, u64, vp, vp, vp]),
            "tfs_crc32_batch_device": (ctypes.c_int, [vp, vp, u32, vp, vp, vp]),
            "tfs_crc32_verify_device": (ctypes.c_int, [vp, vp, u32, vp, vp, vp, vp, vp]),
            "tfs_crc32_submit_verify": (ctypes.c_int, [vp, vp, u32, vp, u64, vp, vp, vp, vp]),
            "tfs_crc32_wait": (ctypes.c_int, [vp, u64]),
            "tfs_block_verify": (ctypes.c_int, [vp, vp, u64, vp, u32, vp, vp, vp]),
            "tfs_block_verify_device": (ctypes.c_int, [vp, vp, u64, vp, u32, vp, vp, vp, vp]),
            "tfs_block_compact": (ctypes.c_int, [vp, vp, u64, vp, vp, u32, vp, u64, vp, vp, vp, vp]),
            "tfs_blocks_compact": (ctypes.c_int, [vp, vp, u32]),
            "tfs_block_compact_device": (ctypes.c_int, [vp, vp, u64, vp, vp, vp, u32, vp, vp, vp, vp, vp]),
            "tfs_compact_jobs_device": (ctypes.c_int, [vp, vp, u64, vp, u32, vp, vp, vp, vp, vp]),
            "tfs_blocks_verify_device": (ctypes.c_int, [vp, vp, u64, vp, u32, vp, vp, vp, vp]),
            "tfs_crc32_synth_fill_device": (ctypes.c_int, [vp, vp, u64, u64, u64, vp]),
            "tfs_crc32_write_headers_device": (ctypes.c_int, [vp, vp, vp, vp, vp, u64, u32, vp]),
            "tfs_crc32_membench_device": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, u32, u64, vp, ctypes.c_uint, vp]),
            "tfs_crc32_dev_malloc": (ctypes.c_int, [vp, u64, ctypes.POINTER(vp)]),
            "tfs_crc32_dev_free": (ctypes.c_int, [vp, vp]),
            "tfs_crc32_host_malloc_pinned": (ctypes.c_int, [vp, u64, ctypes.POINTER(vp)]),
            "tfs_crc32_host_free_pinned": (ctypes.c_int, [vp, vp]),
            "tfs_crc32_host_device_ptr": (ctypes.c_int, [vp, vp, ctypes.POINTER(vp)]),
            "tfs_crc32_memcpy": (ctypes.c_int, [vp, vp, vp, u64, vp]),
            "tfs_crc32_memset_device": (ctypes.c_int, [vp, vp, ctypes.c_int, u64, vp]),
            "tfs_crc32_event_create": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
            "tfs_crc32_event_record": (ctypes.c_int, [vp, vp, vp]),
            "tfs_crc32_event_elapsed_ms": (ctypes.c_int, [vp, vp, vp, ctypes.POINTER(ctypes.c_float)]),
            "tfs_crc32_event_destroy": (ctypes.c_int, [vp, vp]),
            "tfs_crc32_stream": (vp, [vp]),
            "tfs_crc32_sync": (ctypes.c_int, [vp]),
            "tfs_crc32_stream_create": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
            "tfs_crc32_stream_sync": (ctypes.c_int, [vp, vp]),
            "tfs_crc32_stream_destroy": (ctypes.c_int, [vp, vp]),
            "tfs_crc32_inject_device_error": (ctypes.c_int, [vp, u32, u32]),
            "tfs_crc32_set_resident": (ctypes.c_int, [vp, ctypes.c_int]),
            "tfs_crc32_resident_stats": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64),
                                                        ctypes.POINTER(ctypes.c_uint64)]),
            "tfs_crc32_resident_ring_in_device_memory": (ctypes.c_int, [vp]),
            "tfs_crc32_stats": (ctypes.c_int, [vp, vp]),
            "tfs_crc32_res_trace": (ctypes.c_int, [vp, vp]),
            "tfs_crc32_res_trace_last": (ctypes.c_int, [vp, vp]),
            "tfs_crc32_error_count": (ctypes.c_uint64, []),
            "tfs_crc32_set_default_ctx": (ctypes.c_int, [vp]),
            "tfs_crc32_bind_thread": (ctypes.c_int, [vp]),
            "tfs_crc32_default_ctx": (vp, []),
            "tfs_crc32_set_cu_reserve": (ctypes.c_int, [vp, ctypes.c_int]),
            "tfs_crc32_set_split": (ctypes.c_int, [vp, ctypes.c_int]),
            "tfs_crc32_set_compact_segment": (ctypes.c_int, [vp, u32]),
            "tfs_crc32_split_stats": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64),
                                                     ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32),
                                                     ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
            "tfs_crc32_throughput_grid": (ctypes.c_int, [vp]),
            "tfs_crc32_sched_stats": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint32),
                                                     ctypes.POINTER(ctypes.c_uint64)]),
            "tfs_crc32_plan_stats": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint32),
                                                    ctypes.POINTER(ctypes.c_uint64)]),
            "tfs_crc32_debug_state": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_uint64),
                                                     ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_uint64)]),
            "tfs_crc32_debug_poison_resident": (ctypes.c_int, [vp, u32]),
            "tfs_crc_group_create": (ctypes.c_int, [vp, u32, ctypes.POINTER(vp)]),
            "tfs_crc_group_destroy": (ctypes.c_int, [vp]),
            "tfs_crc_group_last_error": (ctypes.c_char_p, [vp]),
            "tfs_crc_group_size": (u32, [vp]),
            "tfs_crc_group_ctx": (vp, [vp, u32]),
            "tfs_crc_group_member_of": (u32, [vp, u32]),
            "tfs_crc_group_ctx_for_block": (vp, [vp, u32]),
            "tfs_crc_group_numa_node": (ctypes.c_int, [vp, u32]),
            "tfs_crc_group_member_bound": (ctypes.c_int, [vp, u32]),
            "tfs_crc_group_host_malloc": (ctypes.c_int, [vp, u32, u64, ctypes.POINTER(vp)]),
            "tfs_crc_group_host_free": (ctypes.c_int, [vp, u32, vp]),
            "tfs_crc_group_blocks_verify": (ctypes.c_int, [vp, vp, u32]),
            "tfs_crc_group_blocks_compact": (ctypes.c_int, [vp, vp, vp, u32]),
            "tfs_packet_verify": (ctypes.c_int, [vp, vp, u32, vp, u64, vp, vp, vp]),
            "tfs_packet_verify_device": (ctypes.c_int, [vp, vp, u32, vp, vp, vp, vp, vp]),
            "tfs_packet_seal": (ctypes.c_int, [vp, vp, u32, vp, u64, vp, vp]),
            "tfs_packet_seal_device": (ctypes.c_int, [vp, vp, u32, vp, vp, vp, vp]),
            "tfs_crc32_write_packet_headers_device": (ctypes.c_int, [vp, vp, vp, vp, u32, i32, i32, u64, vp]),
        }
        for name, (res, args) in sig.items():
            try:
                f = getattr(L, name)
            except AttributeError:
                if measure and os.environ.get("TFS_CRC_LIB"):  # an older build under A/B lacks newer entry points
                    continue
                raise
            f.restype = res
            f.argtypes = args
        _LIBS[path] = L
    return _LIBS[path]


def device_count():
    return lib().tfs_crc32_device_count()


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if isinstance(a, int):
        return a
    if isinstance(a, (DeviceBuffer, PinnedBuffer)):
        return a.ptr
    if isinstance(a, (bytes, bytearray, memoryview)):
        return ctypes.cast(ctypes.c_char_p(bytes(a)), ctypes.c_void_p).value
    raise TypeError("unsupported buffer %r" % type(a))


def _as_u8(data):
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(data), dtype=np.uint8)


class Context:
    """One per GPU: wraps tfs_crc_ctx (device tables, stream, staging pools)."""

    @classmethod
    def wrap(cls, handle, device, L=None):
        """A non-owning view of a context owned elsewhere (a Group member)."""
        c = cls.__new__(cls)
        c.handle, c.device, c._owned = ctypes.c_void_p(handle), device, False
        c.L = L or lib()
        return c

    def __init__(self, device=0, measure=None):
        """measure: use the measurement build (A/B kernel forms); None = when
        TFS_CRC_VARIANT / TFS_EC_VARIANT asks for one."""
        self._owned = True
        self.L = lib(measuring() if measure is None else measure)
        h = ctypes.c_void_p()
        rc = self.L.tfs_crc32_ctx_create(device, ctypes.byref(h))
        if rc != TFS_SUCCESS:
            msg = self.L.tfs_crc32_last_error(h).decode() if h.value else "ctx_create failed"
            if h.value:
                self.L.tfs_crc32_ctx_destroy(h)
            raise TfsCrcError(rc, "tfs_crc32_ctx_create(%d): %s" % (device, msg))
        self.handle = h
        self.device = device

    def close(self):
        if getattr(self, "_owned", True) and self.handle is not None and self.handle.value:
            self.L.tfs_crc32_ctx_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc, what, ok=(TFS_SUCCESS,)):
        if rc not in ok:
            raise TfsCrcError(rc, "%s: %s" % (what, self.L.tfs_crc32_last_error(self.handle).decode()))
        return rc

    @property
    def stream(self):
        return self.L.tfs_crc32_stream(self.handle)

    def sync(self):
        self._check(self.L.tfs_crc32_sync(self.handle), "sync")

    def inject_device_error(self, skip=0, count=1):
        """Fault injection: the next `count` host submissions after `skip` fail with -20001."""
        self._check(self.L.tfs_crc32_inject_device_error(self.handle, skip, count), "inject_device_error")

    def set_resident(self, on):
        """Small synchronous batches through the resident kernel (on) or a launch each (off)."""
        self._check(self.L.tfs_crc32_set_resident(self.handle, 1 if on else 0), "set_resident")

    def resident_stats(self):
        """(launches of the resident kernel, files taken through its ring) so far."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.L.tfs_crc32_resident_stats(self.handle, ctypes.byref(a), ctypes.byref(b)), "resident_stats")
        return a.value, b.value

    def resident_ring_in_device_memory(self):
        """1: the resident ring is in device memory written through the BAR; 0: in
        page-locked host memory; -1: not set up yet."""
        return int(self.L.tfs_crc32_resident_ring_in_device_memory(self.handle))

    def stats(self):
        """tfs_crc32_stats as a dict: host calls, lone (one-body) calls and those under
        TFS_CRC_LONE_CROSSOVER, resident kernel launches / files / ring-full launches."""
        st = CrcStats()
        self._check(self.L.tfs_crc32_stats(self.handle, ctypes.byref(st)), "stats")
        return {k: getattr(st, k) for k, _ in CrcStats._fields_}

    def set_cu_reserve(self, on):
        """Leave live resident kernels' CUs out of throughput launches (on, the default) or not."""
        self._check(self.L.tfs_crc32_set_cu_reserve(self.handle, 1 if on else 0), "set_cu_reserve")

    def set_split(self, on):
        """Split files > 128 KiB of throughput launches over several waves: 0/False whole files,
        1/True segments appended after the files, 2 every unit in address order."""
        self._check(self.L.tfs_crc32_set_split(self.handle, int(on)), "set_split")

    def set_compact_segment(self, seg_bytes):
        """Segmented device compaction: records longer than seg_bytes (8/16/32 KiB) are cut
        into segments on separate waves; 0 keeps every record on one wave."""
        self._check(self.L.tfs_crc32_set_compact_segment(self.handle, int(seg_bytes)), "set_compact_segment")

    def split_stats(self):
        """The latest split throughput launch: {launches, used, files, cap, grid, units} (waits for it)."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        c, d, e = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self.L.tfs_crc32_split_stats(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c),
                                                 ctypes.byref(d), ctypes.byref(e)), "split_stats")
        return {"launches": a.value, "used": b.value, "files": c.value, "cap": d.value, "grid": e.value,
                "units": c.value + min(b.value, d.value)}

    def throughput_grid(self):
        """Workgroups the next throughput launch of this context would use."""
        g = self.L.tfs_crc32_throughput_grid(self.handle)
        if g < 0:
            self._check(g, "throughput_grid")
        return g

    def sched_stats(self):
        """(ctx-owned streams bound, launches so far on streams the ctx does not own)."""
        a, b = ctypes.c_uint32(), ctypes.c_uint64()
        self._check(self.L.tfs_crc32_sched_stats(self.handle, ctypes.byref(a), ctypes.byref(b)), "sched_stats")
        return a.value, b.value

    def plan_stats(self):
        """(split / segment plans held, their device bytes) -- test hook."""
        a, b = ctypes.c_uint32(), ctypes.c_uint64()
        self._check(self.L.tfs_crc32_plan_stats(self.handle, ctypes.byref(a), ctypes.byref(b)), "plan_stats")
        return a.value, b.value

    def debug_state(self):
        """{sched, sched_bytes, res_state, res_state_bytes}: device addresses of the scheduler slots and
        resident-kernel state (test hook)."""
        a, b, c, d = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_void_p(), ctypes.c_uint64()
        self._check(self.L.tfs_crc32_debug_state(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c),
                                                 ctypes.byref(d)), "debug_state")
        return {"sched": a.value, "sched_bytes": b.value, "res_state": c.value, "res_state_bytes": d.value}

    def debug_poison_resident(self, done):
        """Test hook: set every resident workgroup's count of units done to `done`."""
        self._check(self.L.tfs_crc32_debug_poison_resident(self.handle, done), "debug_poison_resident")

    def stream_create(self):
        p = ctypes.c_void_p()
        self._check(self.L.tfs_crc32_stream_create(self.handle, ctypes.byref(p)), "stream_create")
        return p.value

    def stream_sync(self, stream):
        self._check(self.L.tfs_crc32_stream_sync(self.handle, stream), "stream_sync")

    def stream_destroy(self, stream):
        self._check(self.L.tfs_crc32_stream_destroy(self.handle, stream), "stream_destroy")

    # ---- host-memory batches -------------------------------------------------
    def batch(self, base, offsets, lens, seeds=0):
        """out[i] = Func::crc(seeds[i], base+offsets[i], lens[i]) for a host buffer."""
        buf = _as_u8(base)
        n = len(offsets)
        d = np.zeros(n, DESC_DTYPE)
        d["offset"] = offsets
        d["len"] = lens
        d["aux"] = seeds
        out = np.zeros(n, np.uint32)
        self._check(self.L.tfs_crc32_batch(self.handle, _ptr(d), n, _ptr(buf), buf.size, _ptr(out)), "batch")
        return out

    def verify(self, base, offsets, lens, expected):
        """Verify-on-read: returns (crc, ok, n_bad, rc) with rc TFS_SUCCESS or TFS_EXIT_CHECK_CRC_ERROR."""
        buf = _as_u8(base)
        n = len(offsets)
        d = np.zeros(n, DESC_DTYPE)
        d["offset"] = offsets
        d["len"] = lens
        d["aux"] = expected
        crc = np.zeros(n, np.uint32)
        ok = np.zeros(n, np.uint8)
        nbad = np.zeros(1, np.uint32)
        rc = self.L.tfs_crc32_verify(self.handle, _ptr(d), n, _ptr(buf), buf.size, _ptr(crc), _ptr(ok), _ptr(nbad))
        self._check(rc, "verify", ok=(TFS_SUCCESS, TFS_EXIT_CHECK_CRC_ERROR))
        return crc, ok, int(nbad[0]), rc

    def submit_verify(self, base, offsets, lens, expected):
        """Async verify; returns a handle to pass to wait()."""
        buf = _as_u8(base)
        n = len(offsets)
        d = np.zeros(n, DESC_DTYPE)
        d["offset"] = offsets
        d["len"] = lens
        d["aux"] = expected
        crc = np.zeros(n, np.uint32)
        ok = np.zeros(n, np.uint8)
        nbad = np.zeros(1, np.uint32)
        t = ctypes.c_uint64()
        rc = self.L.tfs_crc32_submit_verify(self.handle, _ptr(d), n, _ptr(buf), buf.size, _ptr(crc), _ptr(ok),
                                           _ptr(nbad), ctypes.byref(t))
        self._check(rc, "submit_verify")
        return {"ticket": t.value, "keep": (buf, d), "crc": crc, "ok": ok, "nbad": nbad}

    def wait(self, h):
        rc = self.L.tfs_crc32_wait(self.handle, h["ticket"])
        self._check(rc, "wait", ok=(TFS_SUCCESS, TFS_EXIT_CHECK_CRC_ERROR))
        return h["crc"], h["ok"], int(h["nbad"][0]), rc

    def datafile_get_crc(self, data):
        b = bytes(data)
        out = ctypes.c_uint32()
        self._check(self.L.tfs_datafile_get_crc(self.handle, b, len(b), ctypes.byref(out)), "datafile_get_crc")
        return out.value

    # ---- device-resident (pointers are device addresses: DeviceBuffer or int) ---
    def batch_device(self, d_desc, n, d_base, d_out, stream=None):
        self._check(self.L.tfs_crc32_batch_device(self.handle, _ptr(d_desc), n, _ptr(d_base), _ptr(d_out), stream),
                    "batch_device")

    def verify_device(self, d_desc, n, d_base, d_crc=None, d_ok=None, d_nbad=None, stream=None):
        self._check(self.L.tfs_crc32_verify_device(self.handle, _ptr(d_desc), n, _ptr(d_base), _ptr(d_crc),
                                                  _ptr(d_ok), _ptr(d_nbad), stream), "verify_device")

    def synth_fill_device(self, d_dst, nbytes, seed, first_word=0, stream=None):
        self._check(self.L.tfs_crc32_synth_fill_device(self.handle, _ptr(d_dst), nbytes, seed, first_word, stream),
                    "synth_fill_device")

    def write_headers_device(self, d_image, d_rec_off, d_len, d_crc, first_id, n, stream=None):
        self._check(self.L.tfs_crc32_write_headers_device(self.handle, _ptr(d_image), _ptr(d_rec_off), _ptr(d_len),
                                                         _ptr(d_crc), first_id, n, stream), "write_headers_device")

    def membench_device(self, pattern, d_base, d_desc, n, nbytes, d_out, grid=0, stream=None):
        self._check(self.L.tfs_crc32_membench_device(self.handle, pattern, _ptr(d_base), _ptr(d_desc), n, nbytes,
                                                    _ptr(d_out), grid, stream), "membench_device")

    def block_verify_device(self, d_image, image_len, d_metas, n, d_crc=None, d_status=None, d_nbad=None,
                            stream=None):
        self._check(self.L.tfs_block_verify_device(self.handle, _ptr(d_image), image_len, _ptr(d_metas), n,
                                                  _ptr(d_crc), _ptr(d_status), _ptr(d_nbad), stream),
                    "block_verify_device")

    def block_compact_device(self, d_src, src_len, d_live_metas, d_flags, d_dest_off, n, d_dest, d_crc=None,
                             d_status=None, d_nbad=None, stream=None):
        self._check(self.L.tfs_block_compact_device(self.handle, _ptr(d_src), src_len, _ptr(d_live_metas),
                                                   _ptr(d_flags), _ptr(d_dest_off), n, _ptr(d_dest), _ptr(d_crc),
                                                   _ptr(d_status), _ptr(d_nbad), stream), "block_compact_device")

    def host_device_ptr(self, h_ptr):
        """Device address of page-locked host memory (zero-copy operand of the *_device calls)."""
        p = ctypes.c_void_p()
        self._check(self.L.tfs_crc32_host_device_ptr(self.handle, _ptr(h_ptr), ctypes.byref(p)), "host_device_ptr")
        return p.value

    def compact_jobs_device(self, d_src, src_len, d_jobs, n, d_dest, d_crc=None, d_status=None, d_nbad=None,
                            stream=None):
        self._check(self.L.tfs_compact_jobs_device(self.handle, _ptr(d_src), src_len, _ptr(d_jobs), n, _ptr(d_dest),
                                                  _ptr(d_crc), _ptr(d_status), _ptr(d_nbad), stream),
                    "compact_jobs_device")

    def blocks_verify_device(self, d_src, src_len, d_jobs, n, d_crc=None, d_status=None, d_nbad=None, stream=None):
        """Verify-on-read of records of many device-resident blocks (tfs_compact_job layout)."""
        self._check(self.L.tfs_blocks_verify_device(self.handle, _ptr(d_src), src_len, _ptr(d_jobs), n, _ptr(d_crc),
                                                   _ptr(d_status), _ptr(d_nbad), stream), "blocks_verify_device")

    def blocks_compact(self, jobs):
        """Pipelined compaction of many blocks; `jobs` is a ctypes array of BlockJob."""
        rc = self.L.tfs_blocks_compact(self.handle, ctypes.cast(jobs, ctypes.c_void_p), len(jobs))
        self._check(rc, "blocks_compact", ok=(TFS_SUCCESS, TFS_EXIT_CHECK_CRC_ERROR))
        return rc

    # ---- packet frames (BasePacket) ------------------------------------------
    @staticmethod
    def _packet_desc(offsets, lens):
        d = np.zeros(len(offsets), PACKET_DESC_DTYPE)
        d["offset"] = offsets
        d["len"] = lens
        return d

    def packet_verify(self, base, offsets, lens):
        """Receive side (BasePacket::decode): returns (crc, status, n_bad, rc)."""
        buf = _as_u8(base)
        d = self._packet_desc(offsets, lens)
        n = len(d)
        crc = np.zeros(n, np.uint32)
        st = np.zeros(n, np.int32)
        nbad = np.zeros(1, np.uint32)
        rc = self.L.tfs_packet_verify(self.handle, _ptr(d), n, _ptr(buf), buf.size, _ptr(crc), _ptr(st), _ptr(nbad))
        self._check(rc, "packet_verify", ok=(TFS_SUCCESS, TFS_EXIT_CHECK_CRC_ERROR))
        return crc, st, int(nbad[0]), rc

    def packet_seal(self, buf, offsets, lens):
        """Send side: writes the body CRC into each V1 header of `buf` (a writable uint8 array)."""
        assert isinstance(buf, np.ndarray) and buf.dtype == np.uint8 and buf.flags.c_contiguous
        d = self._packet_desc(offsets, lens)
        n = len(d)
        crc = np.zeros(n, np.uint32)
        st = np.zeros(n, np.int32)
        self._check(self.L.tfs_packet_seal(self.handle, _ptr(d), n, _ptr(buf), buf.size, _ptr(crc), _ptr(st)),
                    "packet_seal")
        return crc, st

    def write_packet_headers_device(self, d_base, d_frame_off, d_body_len, n, pcode=9, version=2, first_id=1,
                                    stream=None):
        self._check(self.L.tfs_crc32_write_packet_headers_device(self.handle, _ptr(d_base), _ptr(d_frame_off),
                                                                _ptr(d_body_len), n, pcode, version, first_id,
                                                                stream), "write_packet_headers_device")

    def packet_verify_device(self, d_desc, n, d_base, d_crc, d_status, d_nbad=None, stream=None):
        self._check(self.L.tfs_packet_verify_device(self.handle, _ptr(d_desc), n, _ptr(d_base), _ptr(d_crc),
                                                   _ptr(d_status), _ptr(d_nbad), stream), "packet_verify_device")

    def packet_seal_device(self, d_desc, n, d_base, d_crc, d_status, stream=None):
        self._check(self.L.tfs_packet_seal_device(self.handle, _ptr(d_desc), n, _ptr(d_base), _ptr(d_crc),
                                                 _ptr(d_status), stream), "packet_seal_device")

    # ---- block images (host) -------------------------------------------------
    def block_verify(self, image, metas):
        img = _as_u8(image)
        m = np.ascontiguousarray(metas, dtype=META_DTYPE)
        n = len(m)
        crc = np.zeros(n, np.uint32)
        st = np.zeros(n, np.int32)
        nbad = np.zeros(1, np.uint32)
        rc = self.L.tfs_block_verify(self.handle, _ptr(img), img.size, _ptr(m), n, _ptr(crc), _ptr(st), _ptr(nbad))
        self._check(rc, "block_verify", ok=(TFS_SUCCESS, TFS_EXIT_CHECK_CRC_ERROR))
        return crc, st, int(nbad[0]), rc

    def block_compact(self, image, metas, flags):
        img = _as_u8(image)
        m = np.ascontiguousarray(metas, dtype=META_DTYPE)
        fl = np.ascontiguousarray(flags, dtype=np.int32)
        n = len(m)
        cap = int(m["size"].astype(np.int64).sum()) + 16
        dest = np.zeros(cap, np.uint8)
        dmetas = np.zeros(n, META_DTYPE)
        ok = np.zeros(n, np.uint8)
        dlen = ctypes.c_uint64()
        nlive = ctypes.c_uint32()
        rc = self.L.tfs_block_compact(self.handle, _ptr(img), img.size, _ptr(m), _ptr(fl), n, _ptr(dest), cap,
                                     _ptr(dmetas), _ptr(ok), ctypes.byref(dlen), ctypes.byref(nlive))
        self._check(rc, "block_compact", ok=(TFS_SUCCESS, TFS_EXIT_CHECK_CRC_ERROR))
        return dest[:dlen.value], dmetas[:nlive.value], ok, rc


class BlockVerifyJob(ctypes.Structure):
    """tfs_block_verify_job (include/tfs_crc.h)."""
    _fields_ = [("block_id", ctypes.c_uint32), ("image", ctypes.c_void_p), ("image_len", ctypes.c_uint64),
                ("metas", ctypes.c_void_p), ("n", ctypes.c_uint32), ("out_crc", ctypes.c_void_p),
                ("out_status", ctypes.c_void_p), ("n_bad", ctypes.c_uint32), ("status", ctypes.c_int)]


class Group:
    """tfs_crc_group: one context per GPU, blocks routed by block id (block_id % size)."""

    def __init__(self, devices=None):
        h = ctypes.c_void_p()
        arr = (ctypes.c_int * len(devices))(*devices) if devices else None
        rc = lib().tfs_crc_group_create(arr, len(devices) if devices else 0, ctypes.byref(h))
        if rc != TFS_SUCCESS:
            msg = lib().tfs_crc_group_last_error(h).decode() if h.value else "group_create failed"
            if h.value:
                lib().tfs_crc_group_destroy(h)
            raise TfsCrcError(rc, "tfs_crc_group_create: %s" % msg)
        self.handle = h
        self.devices = list(devices) if devices else list(range(lib().tfs_crc_group_size(h)))

    def close(self):
        if self.handle is not None and self.handle.value:
            lib().tfs_crc_group_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what, ok=(TFS_SUCCESS,)):
        if rc not in ok:
            raise TfsCrcError(rc, "%s: %s" % (what, lib().tfs_crc_group_last_error(self.handle).decode()))
        return rc

    def size(self):
        return lib().tfs_crc_group_size(self.handle)

    def ctx(self, i):
        return Context.wrap(lib().tfs_crc_group_ctx(self.handle, i), self.devices[i])

    def member_of(self, block_id):
        return lib().tfs_crc_group_member_of(self.handle, block_id)

    def ctx_for_block(self, block_id):
        return self.ctx(self.member_of(block_id))

    def numa_node(self, i):
        return lib().tfs_crc_group_numa_node(self.handle, i)

    def member_bound(self, i):
        return bool(lib().tfs_crc_group_member_bound(self.handle, i))

    def host_malloc(self, i, nbytes):
        """Page-locked memory on member i's NUMA node, as a PinnedBuffer."""
        p = ctypes.c_void_p()
        self._check(lib().tfs_crc_group_host_malloc(self.handle, i, nbytes, ctypes.byref(p)), "group_host_malloc")
        return PinnedBuffer.adopt(self.ctx(i), p.value, nbytes,
                                  lambda ptr, g=self.handle, m=i: lib().tfs_crc_group_host_free(g, m, ptr))

    def blocks_verify(self, jobs):
        rc = lib().tfs_crc_group_blocks_verify(self.handle, ctypes.cast(jobs, ctypes.c_void_p), len(jobs))
        return self._check(rc, "group_blocks_verify", ok=(TFS_SUCCESS, TFS_EXIT_CHECK_CRC_ERROR))

    def blocks_compact(self, block_ids, jobs):
        ids = np.ascontiguousarray(block_ids, np.uint32)
        rc = lib().tfs_crc_group_blocks_compact(self.handle, ids.ctypes.data, ctypes.cast(jobs, ctypes.c_void_p),
                                                len(jobs))
        return self._check(rc, "group_blocks_compact", ok=(TFS_SUCCESS, TFS_EXIT_CHECK_CRC_ERROR))


class DeviceBuffer:
    """Device memory owned through the C ABI (tfs_crc32_dev_malloc)."""

    def __init__(self, ctx, nbytes):
        p = ctypes.c_void_p()
        ctx._check(ctx.L.tfs_crc32_dev_malloc(ctx.handle, nbytes, ctypes.byref(p)), "dev_malloc(%d)" % nbytes)
        self.ctx, self.ptr, self.nbytes = ctx, p.value, nbytes

    def free(self):
        if self.ptr:
            self.ctx.L.tfs_crc32_dev_free(self.ctx.handle, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def upload(self, arr, offset=0):
        a = np.ascontiguousarray(arr)
        self.ctx._check(self.ctx.L.tfs_crc32_memcpy(self.ctx.handle, self.ptr + offset, a.ctypes.data, a.nbytes, None),
                        "memcpy h2d")
        return self

    def download(self, dtype=np.uint8, count=None, offset=0):
        dt = np.dtype(dtype)
        if count is None:
            count = (self.nbytes - offset) // dt.itemsize
        out = np.empty(count, dt)
        self.ctx._check(self.ctx.L.tfs_crc32_memcpy(self.ctx.handle, out.ctypes.data, self.ptr + offset, out.nbytes,
                                               None), "memcpy d2h")
        return out

    def zero(self, stream=None):
        self.ctx._check(self.ctx.L.tfs_crc32_memset_device(self.ctx.handle, self.ptr, 0, self.nbytes, stream), "memset")


class PinnedBuffer:
    """Page-locked host memory (hipHostMalloc) viewed as a numpy uint8 array."""

    def __init__(self, ctx, nbytes):
        p = ctypes.c_void_p()
        ctx._check(ctx.L.tfs_crc32_host_malloc_pinned(ctx.handle, nbytes, ctypes.byref(p)), "host_malloc_pinned")
        self.ctx, self.ptr, self.nbytes = ctx, p.value, nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p.value))
        self._free = lambda ptr: self.ctx.L.tfs_crc32_host_free_pinned(self.ctx.handle, ptr)

    @classmethod
    def adopt(cls, ctx, ptr, nbytes, free_fn):
        b = cls.__new__(cls)
        b.ctx, b.ptr, b.nbytes, b._free = ctx, ptr, nbytes, free_fn
        b.array = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(ptr))
        return b

    def free(self):
        if self.ptr:
            self.array = None
            self._free(self.ptr)
            self.ptr = None


class Event:
    def __init__(self, ctx):
        p = ctypes.c_void_p()
        ctx._check(ctx.L.tfs_crc32_event_create(ctx.handle, ctypes.byref(p)), "event_create")
        self.ctx, self.ptr = ctx, p.value

    def record(self, stream=None):
        self.ctx._check(self.ctx.L.tfs_crc32_event_record(self.ctx.handle, self.ptr, stream), "event_record")

    def elapsed_ms(self, end):
        ms = ctypes.c_float()
        self.ctx._check(self.ctx.L.tfs_crc32_event_elapsed_ms(self.ctx.handle, self.ptr, end.ptr, ctypes.byref(ms)),
                        "event_elapsed")
        return ms.value

    def __del__(self):
        try:
            self.ctx.L.tfs_crc32_event_destroy(self.ctx.handle, self.ptr)
        except Exception:
            pass


def func_crc(crc, data, length=None):
    """Drop-in for Func::crc(uint32_t crc, const char* data, const int32_t len) (GPU, default context)."""
    b = bytes(data)
    n = len(b) if length is None else int(length)
    if n > len(b):
        raise ValueError("length exceeds buffer")
    err = ctypes.c_int(0)
    v = lib().tfs_crc32_e(crc & 0xFFFFFFFF, b, n, ctypes.byref(err))
    if err.value != TFS_SUCCESS:
        raise TfsCrcError(err.value, "tfs_crc32: %s" % lib().tfs_crc32_last_error(None).decode())
    return v
