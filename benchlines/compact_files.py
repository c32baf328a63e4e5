"""bench.py --workload compact_files."""
import ctypes
import os
import time

import numpy as np

from benchlines.common import *  # noqa: F401,F403


def bench_compact_files(args):
    """Compaction from block files (CompactTask::real_compact over FileIterator's 8 MiB
    windows, task.cpp:713-880, logic_block.cpp:1132-1329): configs[3]'s fragmented
    blocks written in TFS's on-disk format (main block + extension block, index),
    then compacted file to file by one BlockFileCompactor (the compaction thread):
    windows read into page-locked memory, live records verified and repacked on the
    GPU straight into page-locked write buffers, new block files and index written.
    The source files are in the page cache (just written) and the new ones go to it
    (no fsync, as the reference's pwrite without O_SYNC)."""
    import shutil
    import tempfile
    import tfs_amd.crc as crc
    import tfs_amd.dataserver as ds
    from tfs_amd.synth import synth_bytes
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    nfiles, L = FILES_PER_BLOCK, FILE_SIZE
    nb, ndistinct = args.file_blocks, 4
    flags = _fragmented_flags(nfiles)
    live = int((flags == 0).sum())
    root = tempfile.mkdtemp(prefix="tfs_compact_files_r%d_" % rank)
    src, dst = os.path.join(root, "src"), os.path.join(root, "dst")
    comp = None
    try:
        # ---- the source blocks on disk (not timed)
        offs = np.arange(nfiles, dtype=np.uint64) * L
        sets = []
        for j in range(ndistinct):
            pay = synth_bytes(0xF11E + 7919 * j + rank, nfiles * L)
            sets.append((pay, ctx.batch(pay, offs, np.full(nfiles, L, np.uint32))))
        for j in range(nb):
            pay, crcs = sets[j % ndistinct]
            blk = ds.LogicBlock(1000 + j)
            for i in range(nfiles):
                if blk.append(i + 1, memoryview(pay)[i * L:(i + 1) * L], int(crcs[i])) != 0:
                    raise SystemExit("compact_files: append failed")
            for i in np.nonzero(flags)[0]:
                blk.set_flag(int(i) + 1, 1)
            ds.write_block_files(blk, src, 1 + j, 100000 + 8 * j)
            blk.free()
        src_bytes = sum(os.path.getsize(os.path.join(src, f)) for f in os.listdir(src)) + sum(
            os.path.getsize(os.path.join(src, "extend", f)) for f in os.listdir(os.path.join(src, "extend")))
        comp = ds.BlockFileCompactor(ctx, windows_per_launch=4)
        # ---- parity: block 1 against the oracle's real_compact of the stitched source
        ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
        ora.oracle_compact.restype = ctypes.c_int64
        ora.oracle_compact.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4
        lb = ds.LoadedBlock(None, src, 1)
        img = lb.data()
        mo = lb.metas["offset"].astype(np.int64)
        ms = lb.metas["size"].astype(np.int32)
        fl = lb.flags.copy()
        n = len(mo)
        odest = np.zeros(img.size, np.uint8)
        doff = np.zeros(n, np.int64)
        dsz = np.zeros(n, np.int32)
        ook = np.zeros(n, np.uint8)
        w = ora.oracle_compact(img.ctypes.data, mo.ctypes.data, ms.ctypes.data, fl.ctypes.data, n,
                               odest.ctypes.data, doff.ctypes.data, dsz.ctypes.data, ook.ctypes.data)
        lb.free()
        rc, dmetas, st, ext, cnt = comp.compact(src, 1, dst, 1, 200000)
        out = ds.LoadedBlock(None, dst, 1)
        if rc != 0 or cnt["n_live"] != live or cnt["dest_size"] != w or not np.array_equal(out.data(), odest[:w]):
            raise SystemExit("compact_files: new block files differ from the oracle's real_compact (rc %d, %s)" %
                             (rc, cnt))
        out.free()
        shutil.rmtree(dst)
        # ---- timed: every block, file to file, one compaction thread
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        windows = launches = 0
        dest_total = 0
        for j in range(nb):
            rc, _, _, _, cnt = comp.compact(src, 1 + j, dst, 1 + j, 200000 + 8 * j)
            if rc != 0 or cnt["n_live"] != live:
                raise SystemExit("compact_files: block %d rc %d %s" % (j, rc, cnt))
            windows += cnt["windows"]
            launches += cnt["launches"]
            dest_total += cnt["dest_size"]
        el = _max_over_ranks(dist, time.perf_counter() - t0)
        # ---- the same bytes moved by the host alone: the source files read by one
        # thread while a second writes the new block's bytes, page cache (the I/O
        # floor of the compactor's reader + writer threads)
        import threading
        buf = np.empty(8 << 20, np.uint8)
        wbuf = np.empty(8 << 20, np.uint8)
        names = sorted(os.listdir(src))
        scratch = os.path.join(root, "io_floor.dat")

        def read_all():
            for f in [os.path.join(src, x) for x in names if x.isdigit()] + [
                    os.path.join(src, "extend", x) for x in os.listdir(os.path.join(src, "extend"))]:
                with open(f, "rb", buffering=0) as fh:
                    while fh.readinto(buf):
                        pass

        def write_all():
            fd = os.open(scratch, os.O_CREAT | os.O_WRONLY, 0o644)
            left = dest_total
            while left > 0:
                left -= os.write(fd, wbuf[:min(left, wbuf.size)])
            os.close(fd)

        t1 = time.perf_counter()
        read_all()
        write_all()
        io_serial = time.perf_counter() - t1
        os.unlink(scratch)
        t1 = time.perf_counter()
        wt = threading.Thread(target=write_all)
        wt.start()
        read_all()
        wt.join()
        io_conc = time.perf_counter() - t1
        os.unlink(scratch)
        writer_thread = os.environ.get("TFS_DS_COMPACT_WRITER", "0") not in ("", "0")
        io_s = io_conc if writer_thread else io_serial
        live_total = float(world) * nb * live * L
        res = {
            "metric": "GiB/s of live payload compacted from block files (FileIterator 8 MiB windows, re-CRC, repack, "
                      "new block files + index written)",
            "value": live_total / el / 2**30, "unit": "GiB/s of live payload", "n_gpus": world,
            "source_block_GiBs": float(world) * src_bytes / el / 2**30,
            "steps": nb, "warmup": 1, "ms_per_step": el / nb * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic 64 KiB files, 1024 per block (main 64 MiB block + extension block), evens + every "
                    "3rd of the rest deleted (%d live), written in TFS's block-file format" % live,
            "config": {"workload": "compaction from block files: %d blocks on disk per GPU, one BlockFileCompactor "
                                   "(4 windows per launch, zero-copy%s)" % (
                                       nb, "; new bytes written by a writer thread" if os.environ.get(
                                           "TFS_DS_COMPACT_WRITER", "0") not in ("", "0") else ""),
                       "storage": "page cache (source just written; new files not fsynced)",
                       "windows": windows, "launches": launches},
            "roofline": {"bound": "host-io", "achieved": (src_bytes + dest_total) / el / 1e9,
                         "peak": (src_bytes + dest_total) / io_s / 1e9, "unit": "GB/s (source read + new block written)",
                         "frac": io_s / el,
                         "peak_source": "measured this run: the same source files read and as many bytes "
                                        "written through the page cache, no CRC or repack, %s (%.1f ms; %s: %.1f ms)" % (
                                            "by two threads at once" if writer_thread else "by one thread in turn",
                                            io_s * 1e3, "in turn" if writer_thread else "two threads at once",
                                            (io_serial if writer_thread else io_conc) * 1e3),
                         "traffic": "whole source block files read from the page cache, live records over PCIe "
                                    "(zero-copy), new block files written"},
            "parity": "block 1: new block files byte-identical to oracle real_compact of the stitched source",
        }
        if rank == 0 and not args.no_cpu:
            # The same walk on the CPU: read the block files (LoadedBlock into
            # malloc'd memory), oracle real_compact with the re-CRC, write the new
            # bytes to a file; single thread, bounded sample.
            lib = ds.lib()
            reps, t2, dt = 0, time.perf_counter(), 0.0
            cdest = np.zeros(img.size, np.uint8)
            while dt < min(args.cpu_seconds, 10.0):
                j = reps % nb
                lb2 = ds.LoadedBlock(None, src, 1 + j)
                nbytes = lib.tfs_ds_loaded_size(lb2.h)
                ptr = lib.tfs_ds_loaded_data(lb2.h)
                m2 = lb2.metas
                mo2, ms2, fl2 = m2["offset"].astype(np.int64), m2["size"].astype(np.int32), lb2.flags.copy()
                wc = ora.oracle_compact(ptr, mo2.ctypes.data, ms2.ctypes.data, fl2.ctypes.data, len(mo2),
                                        cdest.ctypes.data, doff.ctypes.data, dsz.ctypes.data, ook.ctypes.data)
                lb2.free()
                if wc != w or nbytes != img.size:
                    raise SystemExit("compact_files: CPU leg disagrees")
                fd = os.open(scratch, os.O_CREAT | os.O_WRONLY | os.O_TRUNC, 0o644)
                os.write(fd, cdest[:wc])
                os.close(fd)
                reps += 1
                dt = time.perf_counter() - t2
            os.unlink(scratch)
            res["cpu_baseline"] = {
                "value": reps * live * L / dt / 2**30, "unit": "GiB/s of live payload", "cores": 1, "kind": "port",
                "sample": "%d blocks: block files read (LoadedBlock, malloc), oracle real_compact with re-CRC, new "
                          "block bytes written, single thread, %.1f s" % (reps, dt)}
        if dist and not args.no_cpu:
            dist.barrier()
        emit(rank, res)
    finally:
        if comp is not None:
            comp.free()
        shutil.rmtree(root, ignore_errors=True)
        ctx.close()
        if dist:
            dist.destroy_process_group()

