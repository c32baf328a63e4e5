"""ctypes binding of the dataserver-shaped C++ harness (tfs_amd/ds/, libtfs_ds.so).

The harness is plain host C++ that reaches the CRC only through the C ABI of
include/tfs_crc.h -- the shape of TFS's own dataserver after the drop-in:
DataFile (data_file.cpp), close_write_file (data_management.cpp:173-236),
LogicBlock records (logic_block.cpp:156-372), verify-on-read
(sync_backup.cpp:315-472), BlockChecker CRC-error accounting
(block_checker.cpp:58-182) and compaction (task.cpp:713-836).
"""
import ctypes
import os

import numpy as np

from . import crc as _crc

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "ds", "libtfs_ds.so")
_LIB = None


def _ctx(ctx):
    """The tfs_crc_ctx handle of a product-library context: libtfs_ds.so links
    libtfs_crc.so, so a measurement-build context (another struct layout) is
    refused here."""
    if getattr(ctx, "L", None) is not _crc.lib():
        raise ValueError("the dataserver harness takes contexts of the product library (libtfs_crc.so)")
    return ctx.handle


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("dataserver harness not built: %s (run __graft_entry__.build())" % LIB_PATH)
        _crc.lib()  # load libtfs_crc.so first (same process-wide instance)
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, i32, u64, i64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int64
        sig = {
            "tfs_ds_datafile_new": (vp, [vp, u64, ctypes.c_char_p]),
            "tfs_ds_datafile_new2": (vp, [vp, u64, ctypes.c_char_p, vp]),
            "tfs_ds_datafile_pooled": (ctypes.c_int, [vp]),
            "tfs_ds_datafile_free": (None, [vp]),
            "tfs_ds_datafile_set_data": (ctypes.c_int, [vp, vp, i32, i32]),
            "tfs_ds_datafile_length": (i32, [vp]),
            "tfs_ds_datafile_get_crc": (u32, [vp, ctypes.POINTER(ctypes.c_int)]),
            "tfs_ds_block_new": (vp, [u32, i64]),
            "tfs_ds_pool_new": (vp, [vp, u32, u64]),
            "tfs_ds_pool_free": (None, [vp]),
            "tfs_ds_pool_size": (u32, [vp]),
            "tfs_ds_pool_in_use": (u32, [vp]),
            "tfs_ds_block_new_in": (vp, [vp, u32, i64]),
            "tfs_ds_block_free": (None, [vp]),
            "tfs_ds_block_size": (i64, [vp]),
            "tfs_ds_block_data": (vp, [vp]),
            "tfs_ds_block_set_flag": (ctypes.c_int, [vp, u64, i32]),
            "tfs_ds_block_corrupt": (ctypes.c_int, [vp, i64, ctypes.c_uint8]),
            "tfs_ds_block_metas": (ctypes.c_int, [vp, vp, vp, u32]),
            "tfs_ds_close_write_file": (ctypes.c_int, [vp, u64, u32, vp]),
            "tfs_ds_batcher_new": (vp, [vp, u32, ctypes.c_int]),
            "tfs_ds_batcher_new2": (vp, [vp, u32, ctypes.c_int, ctypes.c_int]),
            "tfs_ds_batcher_new3": (vp, [vp, u32, ctypes.c_int, ctypes.c_int, vp]),
            "tfs_ds_lease_pool_new": (vp, [vp, u32]),
            "tfs_ds_lease_pool_free": (None, [vp]),
            "tfs_ds_lease_pool_in_use": (u32, [vp]),
            "tfs_ds_batcher_free": (None, [vp]),
            "tfs_ds_batcher_batches": (u64, [vp]),
            "tfs_ds_batcher_close": (ctypes.c_int, [vp, vp, u64, u32, vp]),
            "tfs_ds_checker_new": (vp, [ctypes.c_int]),
            "tfs_ds_checker_free": (None, [vp]),
            "tfs_ds_checker_errors": (ctypes.c_int, [vp, u32]),
            "tfs_ds_checker_needs_repair": (ctypes.c_int, [vp, u32]),
            "tfs_ds_verify_block": (ctypes.c_int, [vp, vp, vp, u32, vp]),
            "tfs_ds_compact_block": (ctypes.c_int, [vp, vp, vp, vp, u32]),
            "tfs_ds_loopback_block": (ctypes.c_int, [vp, vp, u32, i32, vp, ctypes.c_int, vp]),
            "tfs_ds_loopback_block_with": (ctypes.c_int, [vp, vp, vp, u32, i32, vp, ctypes.c_int, vp]),
            "tfs_ds_block_read_file": (ctypes.c_int, [vp, u64, vp, ctypes.POINTER(i32), i32, ctypes.c_int]),
            "tfs_ds_recombine_block": (ctypes.c_int, [vp, vp, vp, ctypes.POINTER(ctypes.c_int)]),
            "tfs_ds_read_file_verified": (ctypes.c_int, [vp, vp, u64, vp, i32, ctypes.POINTER(i32), vp]),
            "tfs_ds_encoder_new": (vp, [vp]),
            "tfs_ds_encoder_free": (None, [vp]),
            "tfs_ds_encoder_add": (None, [vp, ctypes.c_int16, ctypes.c_int16, u64, ctypes.c_char_p, i32]),
            "tfs_ds_encoder_flush": (ctypes.c_int, [vp]),
            "tfs_ds_encoder_size": (i64, [vp]),
            "tfs_ds_encoder_data": (vp, [vp]),
            "tfs_ds_block_write_files": (ctypes.c_int, [vp, ctypes.c_char_p, i32, i32, u32, u32, i32, vp, u32,
                                                         ctypes.POINTER(u32)]),
            "tfs_ds_block_append": (ctypes.c_int, [vp, u64, ctypes.c_char_p, i32, u32]),
            "tfs_ds_loaded_new": (vp, [vp]),
            "tfs_ds_loaded_free": (None, [vp]),
            "tfs_ds_loaded_load": (ctypes.c_int, [vp, ctypes.c_char_p, i32, i32, u32]),
            "tfs_ds_loaded_size": (i64, [vp]),
            "tfs_ds_loaded_data": (vp, [vp]),
            "tfs_ds_loaded_logic_id": (u32, [vp]),
            "tfs_ds_loaded_metas": (u32, [vp, vp, vp, u32, vp, u32, ctypes.POINTER(u32), vp]),
            "tfs_ds_verify_block_files": (ctypes.c_int, [vp, ctypes.c_char_p, i32, i32, u32, vp, u32,
                                                         ctypes.POINTER(u32), vp]),
            "tfs_ds_compact_block_files": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_char_p, i32, i32, u32, u32,
                                                          u32, i32, ctypes.c_int, vp, vp, u32, vp, u32,
                                                          ctypes.POINTER(u32), vp]),
            "tfs_ds_compactor_new": (vp, [vp, ctypes.c_int]),
            "tfs_ds_compactor_free": (None, [vp]),
            "tfs_ds_compactor_compact": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_char_p, i32, i32, u32, u32, u32,
                                                        i32, vp, vp, u32, vp, u32, ctypes.POINTER(u32), vp]),
            "tfs_ds_decode": (ctypes.c_int, [vp, vp, i64, vp, vp, vp, u32, ctypes.POINTER(u32),
                                             ctypes.POINTER(i64)]),
            "tfs_ds_close_latency": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, i32, vp]),
            "tfs_ds_close_latency_phases": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, i32, vp, vp]),
            "tfs_ds_scalar_latency": (ctypes.c_int, [ctypes.c_int, i32, vp]),
            "tfs_ds_close_stream": (ctypes.c_int, [vp, ctypes.c_int, i32, vp, vp, u64, ctypes.POINTER(u64)]),
            "tfs_ds_service_new": (vp, [vp, u32, ctypes.c_int]),
            "tfs_ds_service_free": (None, [vp]),
            "tfs_ds_service_ctx_for_block": (vp, [vp, u32]),
            "tfs_ds_service_close": (ctypes.c_int, [vp, vp, u64, u32, vp]),
            "tfs_ds_service_verify_blocks": (ctypes.c_int, [vp, vp, u32, vp]),
            "tfs_ds_service_loopback": (ctypes.c_int, [vp, vp, u32, u32, i32, vp, ctypes.c_int, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


class DataFile:
    """DataFile (src/dataserver/data_file.h:33-96)."""

    def __init__(self, ctx, fn, tmp_dir="/tmp", pool=None):
        if pool is None:
            self.h = lib().tfs_ds_datafile_new(_ctx(ctx), fn, tmp_dir.encode())
        else:  # the buffer from a LeaseBufferPool (the heap when it is exhausted)
            self.pool = pool
            self.h = lib().tfs_ds_datafile_new2(_ctx(ctx), fn, tmp_dir.encode(), pool.h)

    def pooled(self):
        return bool(lib().tfs_ds_datafile_pooled(self.h))

    def set_data(self, data, offset):
        b = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8))
        return lib().tfs_ds_datafile_set_data(self.h, b.ctypes.data, b.size, offset)

    def get_length(self):
        return lib().tfs_ds_datafile_length(self.h)

    def get_crc(self):
        st = ctypes.c_int(0)
        c = lib().tfs_ds_datafile_get_crc(self.h, ctypes.byref(st))
        if st.value != 0:
            raise _crc.TfsCrcError(st.value, "DataFile::get_crc")
        return c

    def free(self):
        if self.h:
            lib().tfs_ds_datafile_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class BlockImagePool:
    """Page-locked block buffers allocated once and lent to LogicBlocks (a dataserver's
    preallocated blocks); a page-locked image is verified in place (zero-copy)."""

    def __init__(self, ctx, count, nbytes):
        self.h = lib().tfs_ds_pool_new(_ctx(ctx), count, nbytes)

    def size(self):
        return lib().tfs_ds_pool_size(self.h)

    def in_use(self):
        """Arenas lent to live LogicBlocks."""
        return lib().tfs_ds_pool_in_use(self.h)

    def free(self):
        """Free the page-locked arenas; refused while a LogicBlock still uses one."""
        if self.h:
            if self.in_use():
                raise RuntimeError("BlockImagePool.free: %d arenas still lent to live blocks (free them first)"
                                   % self.in_use())
            lib().tfs_ds_pool_free(self.h)
            self.h = None


class LogicBlock:
    """One logical block: FileInfo|payload records + index (logic_block.cpp)."""

    def __init__(self, block_id, capacity=1 << 40, pool=None):
        self.block_id = block_id
        self.pool = pool  # kept alive while this block may hold one of its arenas
        self.h = lib().tfs_ds_block_new_in(pool.h, block_id, capacity) if pool else \
            lib().tfs_ds_block_new(block_id, capacity)

    def close_write_file(self, file_id, client_crc, df):
        """DataManagement::close_write_file: 0, or EXIT_DATA_FILE_ERROR (-8013) on crc mismatch."""
        return lib().tfs_ds_close_write_file(self.h, file_id, client_crc, df.h)

    def raw(self):
        n = lib().tfs_ds_block_size(self.h)
        if n == 0:
            return np.zeros(0, np.uint8)
        p = lib().tfs_ds_block_data(self.h)
        return np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p)).copy()

    def append(self, file_id, payload, crc):
        """Append FileInfo|payload with a caller-supplied crc (fixtures; no CRC computed)."""
        b = bytes(payload)
        return lib().tfs_ds_block_append(self.h, file_id, b, len(b), crc)

    def read_file(self, file_id, nbytes, offset=0, force=False):
        """LogicBlock::read_file (logic_block.cpp:374-440): returns (rc, bytes)."""
        buf = np.zeros(max(nbytes, 1), np.uint8)
        n = ctypes.c_int32(nbytes)
        rc = lib().tfs_ds_block_read_file(self.h, file_id, buf.ctypes.data, ctypes.byref(n), offset, int(force))
        return rc, buf[:max(n.value, 0)].tobytes()

    def read_file_verified(self, ctx, file_id, checker=None, cap=1 << 24):
        """read_data + GPU verify-on-read against FileInfo.crc_: returns (rc, FileInfo|payload)."""
        buf = np.zeros(cap, np.uint8)
        n = ctypes.c_int32(0)
        rc = lib().tfs_ds_read_file_verified(_ctx(ctx), self.h, file_id, buf.ctypes.data, cap, ctypes.byref(n),
                                             checker.h if checker else None)
        return rc, buf[:min(max(n.value, 0), cap)].tobytes()

    def set_flag(self, file_id, flag):
        return lib().tfs_ds_block_set_flag(self.h, file_id, flag)

    def corrupt(self, offset, mask=1):
        return lib().tfs_ds_block_corrupt(self.h, offset, mask)

    def metas(self):
        n = lib().tfs_ds_block_metas(self.h, None, None, 0)
        m = np.zeros(n, _crc.META_DTYPE)
        f = np.zeros(n, np.int32)
        lib().tfs_ds_block_metas(self.h, m.ctypes.data, f.ctypes.data, n)
        return m, f

    def free(self):
        if self.h:
            lib().tfs_ds_block_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class LeaseBufferPool:
    """Page-locked DataFile buffers (2 MiB each) in one allocation: a CloseBatcher
    on the pool checks each lease's payload where set_data put it."""

    def __init__(self, ctx, nbuffers):
        self.h = lib().tfs_ds_lease_pool_new(_ctx(ctx), nbuffers)
        if not self.h:
            raise RuntimeError("tfs_ds_lease_pool_new(%d) failed" % nbuffers)

    def in_use(self):
        return lib().tfs_ds_lease_pool_in_use(self.h)

    def free(self):
        """Refused while a DataFile still holds one of the buffers."""
        if self.h:
            if self.in_use():
                raise RuntimeError("LeaseBufferPool.free: %d buffers still held by DataFiles" % self.in_use())
            lib().tfs_ds_lease_pool_free(self.h)
            self.h = None


class CloseBatcher:
    """Batches close_write_file CRC checks from many threads into one GPU verify."""

    def __init__(self, ctx, max_batch=64, max_wait_us=200, in_flight=None, pool=None):
        if pool is not None:  # keep the pool alive as long as the batcher
            self.pool = pool
            self.h = lib().tfs_ds_batcher_new3(_ctx(ctx), max_batch, max_wait_us, in_flight or 8, pool.h)
        elif in_flight is None:
            self.h = lib().tfs_ds_batcher_new(_ctx(ctx), max_batch, max_wait_us)
        else:  # batches in use at once, 1..16 (default 8)
            self.h = lib().tfs_ds_batcher_new2(_ctx(ctx), max_batch, max_wait_us, in_flight)

    def close(self, block, file_id, client_crc, df):
        return lib().tfs_ds_batcher_close(self.h, block.h, file_id, client_crc, df.h)

    def batches(self):
        return lib().tfs_ds_batcher_batches(self.h)

    def free(self):
        if self.h:
            lib().tfs_ds_batcher_free(self.h)
            self.h = None


class CrcService:
    """DataService's CRC side on a multi-GPU node: a device group and one CloseBatcher
    per member; DataFiles, closes and block verifies are routed by block id."""

    def __init__(self, group, max_batch=8, max_wait_us=100):
        self.group = group
        self.h = lib().tfs_ds_service_new(group.handle, max_batch, max_wait_us)

    def ctx_for_block(self, block_id):
        return _crc.Context.wrap(lib().tfs_ds_service_ctx_for_block(self.h, block_id), -1)

    def close(self, block, file_id, client_crc, df):
        return lib().tfs_ds_service_close(self.h, block.h, file_id, client_crc, df.h)

    def verify_blocks(self, blocks):
        arr = (ctypes.c_void_p * len(blocks))(*[b.h for b in blocks])
        nb = np.zeros(len(blocks), np.uint32)
        rc = lib().tfs_ds_service_verify_blocks(self.h, arr, len(blocks), nb.ctypes.data)
        return rc, nb

    def loopback(self, payloads, files_per_block, length, client_crc, nthreads, blocks):
        p = np.ascontiguousarray(payloads, dtype=np.uint8)
        c = np.ascontiguousarray(client_crc, dtype=np.uint32)
        n = len(blocks) * files_per_block
        if p.size < n * length or c.size < n:
            raise ValueError("payloads/client_crc too small")
        arr = (ctypes.c_void_p * len(blocks))(*[b.h for b in blocks])
        return lib().tfs_ds_service_loopback(self.h, p.ctypes.data, len(blocks), files_per_block, length,
                                             c.ctypes.data, nthreads, arr)

    def free(self):
        if self.h:
            lib().tfs_ds_service_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class BlockCrcChecker:
    def __init__(self, max_crc_error_nums=4):
        self.h = lib().tfs_ds_checker_new(max_crc_error_nums)

    def errors(self, block_id):
        return lib().tfs_ds_checker_errors(self.h, block_id)

    def needs_repair(self, block_id):
        return bool(lib().tfs_ds_checker_needs_repair(self.h, block_id))

    def free(self):
        if self.h:
            lib().tfs_ds_checker_free(self.h)
            self.h = None


class PacketEncoder:
    """Send-side packet batch (packet_codec.h): V1 frames sealed on the GPU."""

    def __init__(self, ctx):
        self.h = lib().tfs_ds_encoder_new(_ctx(ctx))

    def add(self, pcode, version, pid, body):
        b = bytes(body)
        lib().tfs_ds_encoder_add(self.h, pcode, version, pid, b, len(b))

    def flush(self):
        return lib().tfs_ds_encoder_flush(self.h)

    def output(self):
        n = lib().tfs_ds_encoder_size(self.h)
        if n == 0:
            return b""
        return ctypes.string_at(lib().tfs_ds_encoder_data(self.h), n)

    def free(self):
        if self.h:
            lib().tfs_ds_encoder_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def decode_stream(ctx, data, cap=1 << 16):
    """Receive side: returns (rc, offsets, status, crc, consumed)."""
    b = np.frombuffer(bytes(data), np.uint8)
    off = np.zeros(cap, np.int64)
    st = np.zeros(cap, np.int32)
    crc = np.zeros(cap, np.uint32)
    nfr = ctypes.c_uint32()
    consumed = ctypes.c_int64()
    rc = lib().tfs_ds_decode(_ctx(ctx), b.ctypes.data, b.size, off.ctypes.data, st.ctypes.data, crc.ctypes.data,
                             cap, ctypes.byref(nfr), ctypes.byref(consumed))
    k = min(nfr.value, cap)
    return rc, off[:k], st[:k], crc[:k], consumed.value


MAIN_BLOCK_SIZE = 64 * 1024 * 1024  # mainblock_size (config_item.h:132)
EXT_BLOCK_SIZE = 32 * 1024 * 1024   # extblock_size (config_item.h:133)
INDEX_HEADER_DTYPE = np.dtype([("block_id", "<u4"), ("version", "<i4"), ("file_count", "<i4"), ("size", "<i4"),
                               ("del_file_count", "<i4"), ("del_size", "<i4"), ("seq_no", "<u4"), ("flag", "<i4"),
                               ("bucket_size", "<i4"), ("data_file_offset", "<i4"), ("index_file_size", "<i4"),
                               ("free_head_offset", "<i4")])


def write_block_files(block, mount, main_id, first_ext_id, bucket_size=1024, main_size=MAIN_BLOCK_SIZE,
                      ext_size=EXT_BLOCK_SIZE):
    """Persist a LogicBlock in TFS's on-disk format (block_store.h); returns the ext ids."""
    ids = np.zeros(64, np.uint32)
    n = ctypes.c_uint32()
    rc = lib().tfs_ds_block_write_files(block.h, mount.encode(), main_size, ext_size, main_id, first_ext_id,
                                        bucket_size, ids.ctypes.data, 64, ctypes.byref(n))
    if rc != 0:
        raise _crc.TfsCrcError(rc, "write_block_files")
    return ids[:n.value].tolist()


class LoadedBlock:
    """A block read back from disk (chain, index, flags, data in pinned memory)."""

    def __init__(self, ctx, mount, main_id, main_size=MAIN_BLOCK_SIZE, ext_size=EXT_BLOCK_SIZE):
        self.h = lib().tfs_ds_loaded_new(_ctx(ctx) if ctx is not None else None)
        self.rc = lib().tfs_ds_loaded_load(self.h, mount.encode(), main_size, ext_size, main_id)
        if self.rc != 0:
            return
        n = lib().tfs_ds_loaded_metas(self.h, None, None, 0, None, 0, None, None)
        self.metas = np.zeros(n, _crc.META_DTYPE)
        self.flags = np.zeros(n, np.int32)
        chain = np.zeros(64, np.uint32)
        clen = ctypes.c_uint32()
        self.header = np.zeros(1, INDEX_HEADER_DTYPE)
        lib().tfs_ds_loaded_metas(self.h, self.metas.ctypes.data, self.flags.ctypes.data, n, chain.ctypes.data, 64,
                                  ctypes.byref(clen), self.header.ctypes.data)
        self.chain = chain[:clen.value].tolist()
        self.logic_block_id = lib().tfs_ds_loaded_logic_id(self.h)

    def data(self):
        n = lib().tfs_ds_loaded_size(self.h)
        if n == 0:
            return np.zeros(0, np.uint8)
        return np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(lib().tfs_ds_loaded_data(self.h))).copy()

    def free(self):
        if self.h:
            lib().tfs_ds_loaded_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def verify_block_files(ctx, mount, main_id, checker=None, main_size=MAIN_BLOCK_SIZE, ext_size=EXT_BLOCK_SIZE):
    """Verify-on-read from block files on disk: returns (nbad or <0, live statuses)."""
    st = np.zeros(1 << 16, np.int32)
    nl = ctypes.c_uint32()
    rc = lib().tfs_ds_verify_block_files(_ctx(ctx), mount.encode(), main_size, ext_size, main_id, st.ctypes.data,
                                         st.size, ctypes.byref(nl), checker.h if checker else None)
    return rc, st[:nl.value]


def compact_block_files(ctx, src_mount, src_main_id, dst_mount, dst_main_id, first_ext_id, bucket_size=0,
                        windows_per_launch=4, main_size=MAIN_BLOCK_SIZE, ext_size=EXT_BLOCK_SIZE, cap=1 << 20):
    """real_compact from block files on disk through 8 MiB windows (block_store.h
    compact_block_files).  Returns (rc, dest metas, statuses, ext ids, counters)
    with counters {n_live, dest_size, windows, launches, big_files, n_bad, n_dropped}."""
    metas = np.zeros(cap, _crc.META_DTYPE)
    st = np.zeros(cap, np.int32)
    ext = np.zeros(64, np.uint32)
    next_ = ctypes.c_uint32()
    cnt = np.zeros(7, np.int64)
    rc = lib().tfs_ds_compact_block_files(_ctx(ctx), src_mount.encode(), dst_mount.encode(), main_size, ext_size,
                                          src_main_id, dst_main_id, first_ext_id, bucket_size, windows_per_launch,
                                          metas.ctypes.data, st.ctypes.data, cap, ext.ctypes.data, 64,
                                          ctypes.byref(next_), cnt.ctypes.data)
    n = int(cnt[0])
    keys = ("n_live", "dest_size", "windows", "launches", "big_files", "n_bad", "n_dropped")
    return rc, metas[:n], st[:n], ext[:next_.value].tolist(), dict(zip(keys, (int(x) for x in cnt)))


class BlockFileCompactor:
    """compact_block_files with its window buffers and streams kept across blocks
    (block_store.h BlockFileCompactor: a compaction thread's state)."""

    def __init__(self, ctx, windows_per_launch=4):
        self.h = lib().tfs_ds_compactor_new(_ctx(ctx), windows_per_launch)
        if not self.h:
            raise _crc.TfsCrcError(-1016, "tfs_ds_compactor_new")
        self.metas = np.zeros(1 << 16, _crc.META_DTYPE)
        self.status = np.zeros(1 << 16, np.int32)
        self.ext = np.zeros(64, np.uint32)
        self.cnt = np.zeros(7, np.int64)

    def compact(self, src_mount, src_main_id, dst_mount, dst_main_id, first_ext_id, bucket_size=0,
                main_size=MAIN_BLOCK_SIZE, ext_size=EXT_BLOCK_SIZE):
        """Returns (rc, dest metas, statuses, ext ids, counters) as compact_block_files (views valid
        until the next call)."""
        next_ = ctypes.c_uint32()
        rc = lib().tfs_ds_compactor_compact(self.h, src_mount.encode(), dst_mount.encode(), main_size, ext_size,
                                            src_main_id, dst_main_id, first_ext_id, bucket_size,
                                            self.metas.ctypes.data, self.status.ctypes.data, self.metas.size,
                                            self.ext.ctypes.data, self.ext.size, ctypes.byref(next_),
                                            self.cnt.ctypes.data)
        n = int(self.cnt[0])
        keys = ("n_live", "dest_size", "windows", "launches", "big_files", "n_bad", "n_dropped")
        return (rc, self.metas[:n], self.status[:n], self.ext[:next_.value].tolist(),
                dict(zip(keys, (int(x) for x in self.cnt))))

    def free(self):
        if self.h:
            lib().tfs_ds_compactor_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def verify_block(ctx, block, checker=None):
    m, f = block.metas()
    st = np.zeros(max(len(m), 1), np.int32)
    nbad = lib().tfs_ds_verify_block(_ctx(ctx), block.h, st.ctypes.data, st.size, checker.h if checker else None)
    live = (f & (_crc.FI_DELETED | _crc.FI_INVALID)) == 0
    return nbad, st[:int(live.sum())]


def compact_block(ctx, src, dest):
    m, _ = src.metas()
    ok = np.zeros(max(len(m), 1), np.uint8)
    rc = lib().tfs_ds_compact_block(_ctx(ctx), src.h, dest.h, ok.ctypes.data, ok.size)
    return rc, ok[:len(m)]


def loopback_block(ctx, payloads, n, length, client_crc, nthreads, block, batcher=None):
    """BASELINE configs[0] through the harness: n payloads written by `nthreads`
    worker threads (DataFile -> CloseBatcher close), then the whole block verified.
    `batcher`: a long-lived CloseBatcher (else one per call).  Returns the number
    of files that failed either check (or a negative status)."""
    p = np.ascontiguousarray(payloads, dtype=np.uint8)
    c = np.ascontiguousarray(client_crc, dtype=np.uint32)
    if p.size < n * length or c.size < n:
        raise ValueError("payloads/client_crc too small")
    return lib().tfs_ds_loopback_block_with(_ctx(ctx), batcher.h if batcher else None, p.ctypes.data, n, length,
                                            c.ctypes.data, nthreads, block.h)


CLOSE_PHASES = ("claim_us", "copy_us", "wait_us", "append_us", "lead_wait_us", "verify_us", "leader", "batch_n",
                "relaunches", "ring_full")


def close_latency(ctx, nleases, iters, length=65536, phases=False):
    """Microseconds per CloseBatcher close with `nleases` leases closing concurrently.
    phases: also each close's CloseTiming (ds_harness.h), a (closes, 10) array in
    CLOSE_PHASES order; returns (us, phases)."""
    out = np.zeros(nleases * iters, np.float64)
    if phases:
        ph = np.zeros((nleases * iters, len(CLOSE_PHASES)), np.float64)
        rc = lib().tfs_ds_close_latency_phases(_ctx(ctx), nleases, iters, length, out.ctypes.data, ph.ctypes.data)
    else:
        rc = lib().tfs_ds_close_latency(_ctx(ctx), nleases, iters, length, out.ctypes.data)
    if rc != 0:
        raise _crc.TfsCrcError(rc, "close_latency")
    return (out, ph) if phases else out


class CloseStream:
    """Closes from `nleases` worker threads through one CloseBatcher, in a
    background thread, until stop(): the close traffic a throughput launch
    shares its GPU with (tfs_ds_close_stream)."""

    def __init__(self, ctx, nleases=8, length=65536, cap=1 << 20):
        import threading
        self._stop = ctypes.c_int(0)
        self.lat = np.zeros(cap, np.float64)
        self.count = ctypes.c_uint64(0)
        self.rc = None
        h = _ctx(ctx)

        def run():
            self.rc = lib().tfs_ds_close_stream(h, nleases, length, ctypes.byref(self._stop), self.lat.ctypes.data,
                                                cap, ctypes.byref(self.count))
        self._t = threading.Thread(target=run)
        self._t.start()

    def stop(self):
        """Stop, join; returns (rc, closes done, latencies in us)."""
        self._stop.value = 1
        self._t.join()
        n = min(int(self.count.value), self.lat.size)
        lat = self.lat[:n]
        return self.rc, int(self.count.value), lat[lat > 0]


def scalar_latency(iters, length=65536):
    """Microseconds per tfs_crc32(0, data, length) call (pageable data, default context)."""
    out = np.zeros(iters, np.float64)
    rc = lib().tfs_ds_scalar_latency(iters, length, out.ctypes.data)
    if rc != 0:
        raise _crc.TfsCrcError(rc, "scalar_latency")
    return out


def recombine_block(ctx, src, dest):
    """TranBlock::recombine_data over the GPU: returns (rc, files skipped for their CRC)."""
    k = ctypes.c_int(0)
    rc = lib().tfs_ds_recombine_block(_ctx(ctx), src.h, dest.h, ctypes.byref(k))
    return rc, k.value
