"""bench.py --workload block_verify / block_verify_device: verify-on-read of
block images (sync_backup.cpp:345-435, block_console.cpp:543-577 checks), from
page-locked host memory and device-resident."""
import ctypes
import os
import time

import numpy as np

from benchlines.common import *  # noqa: F401,F403


def bench_block_verify(args):
    """Verify-on-read of fragmented blocks held in page-locked host memory (the
    block files of tfs_amd/ds/block_store.h load into such buffers): per block one
    tfs_block_verify over its live records (sync_backup.cpp:345-435 checks).
    The kernel reads only the named records over PCIe (zero-copy)."""
    import tfs_amd.crc as crc
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    nfiles, rec = FILES_PER_BLOCK, FILEINFO + FILE_SIZE
    blk_bytes = nfiles * rec
    ndistinct, nblocks = 8, args.compact_blocks
    d_img = crc.DeviceBuffer(ctx, blk_bytes + 64)
    d_desc = crc.DeviceBuffer(ctx, 16 * nfiles)
    d_crc = crc.DeviceBuffer(ctx, 4 * nfiles)
    d_off = crc.DeviceBuffer(ctx, 8 * nfiles).upload(np.arange(nfiles, dtype=np.uint64) * rec)
    d_len = crc.DeviceBuffer(ctx, 4 * nfiles).upload(np.full(nfiles, FILE_SIZE, np.uint32))
    desc = np.zeros(nfiles, crc.DESC_DTYPE)
    desc["offset"], desc["len"] = np.arange(nfiles) * rec + FILEINFO, FILE_SIZE
    d_desc.upload(desc)
    srcs = []
    for b in range(ndistinct):
        ctx.synth_fill_device(d_img, blk_bytes + 64 - (blk_bytes + 64) % 8, 0xB1F + 13 * b + rank, 0)
        ctx.batch_device(d_desc, nfiles, d_img, d_crc)
        ctx.write_headers_device(d_img, d_off, d_len, d_crc, 1, nfiles)
        ctx.sync()
        p = crc.PinnedBuffer(ctx, blk_bytes)
        p.array[:] = d_img.download(np.uint8, blk_bytes)
        srcs.append(p)
    live = np.nonzero(_fragmented_flags(nfiles) == 0)[0]
    metas = np.zeros(live.size, crc.META_DTYPE)
    metas["file_id"], metas["offset"], metas["size"] = 1 + live, live * rec, rec
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_verify_file.restype = ctypes.c_int32
    ora.oracle_verify_file.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.POINTER(ctypes.c_uint32)]
    c0, st0, nb0, _ = ctx.block_verify(srcs[0].array, metas)
    for i in np.linspace(0, live.size - 1, 16).astype(np.int64):  # parity spot check (test infrastructure)
        oc = ctypes.c_uint32()
        code = ora.oracle_verify_file(srcs[0].ptr, blk_bytes, int(metas["offset"][i]), rec, ctypes.byref(oc))
        if code != st0[i] or oc.value != int(c0[i]):
            raise SystemExit("block_verify: GPU disagrees with oracle at record %d" % i)
    nb = nblocks
    ctx.block_verify(srcs[0].array, metas)
    # the timed loop calls the C ABI directly on arrays made once, as a dataserver
    # thread would (the Python wrapper's per-call array set-up is not the library's),
    # from `threads` threads (the mirror, repair and checker call sites each verify on
    # their own thread; round 6: their calls run side by side)
    import threading
    L = crc.lib()
    threads = max(1, args.verify_threads)
    outs = [(np.zeros(live.size, np.uint32), np.zeros(live.size, np.int32), np.zeros(1, np.uint32))
            for _ in range(threads)]
    errs = []

    def worker(t, go):
        o_crc, o_st, o_bad = outs[t]
        margs = (metas.ctypes.data, live.size, o_crc.ctypes.data, o_st.ctypes.data, o_bad.ctypes.data)
        go.wait()
        for j in range(t, nb, threads):
            rc = L.tfs_block_verify(ctx.handle, srcs[j % ndistinct].ptr, blk_bytes, *margs)
            if rc != 0 or o_bad[0]:
                errs.append((j, rc, int(o_bad[0])))
                return

    def warm_and_time():
        go = threading.Barrier(threads + 1)
        ts = [threading.Thread(target=worker, args=(t, go)) for t in range(threads)]
        for x in ts:
            x.start()
        go.wait()
        t0 = time.perf_counter()
        for x in ts:
            x.join()
        return time.perf_counter() - t0

    if dist:
        dist.barrier()
    el = _max_over_ranks(dist, warm_and_time())
    if errs:
        raise SystemExit("block_verify: rc / mismatches on clean blocks: %s" % errs[:4])
    ceil = pcie_ceiling(ctx, dist=dist)
    pcie_gbs = float(nb) * live.size * rec / el / 1e9
    res = {
        "metric": "GiB/s of live payload verified on read from fragmented blocks in page-locked host memory",
        "value": float(world) * nb * live.size * FILE_SIZE / el / 2**30, "unit": "GiB/s of live payload",
        "source_block_GiBs": float(world) * nb * blk_bytes / el / 2**30, "n_gpus": world, "steps": nb,
        "warmup": 1, "ms_per_step": el / nb * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic 64 KiB files, 1024 per block, evens + every 3rd of the rest deleted (%d live)" % live.size,
        "config": {"workload": "one tfs_block_verify per block over its live records, %d blocks from %d caller "
                               "threads (C ABI called directly, arrays made once)" % (nb, threads),
                   "threads": threads,
                   "live_payload_GiBs": float(world) * nb * live.size * FILE_SIZE / el / 2**30},
        "roofline": {"bound": "pcie", "achieved": pcie_gbs, "peak": ceil["h2d_GBs"], "unit": "GB/s (per GPU)",
                     "frac": pcie_gbs / ceil["h2d_GBs"], "peak_source": ceil["source"],
                     "traffic": "the live records (FileInfo + payload) read in place over PCIe"},
    }
    if rank == 0 and not args.no_cpu:
        # the reference CRC over the live payloads of the same page-locked image, checked against the
        # FileInfo crc_ values the GPU verified (sync_backup.cpp:412-435's loop without the pread)
        cb = cpu_baseline(srcs[0].array, live * rec + FILEINFO, np.full(live.size, FILE_SIZE), c0,
                          args.cpu_seconds, "live 64 KiB payloads of a page-locked block image")
        cb["source_block_GiBs"] = cb["value"] * blk_bytes / (live.size * FILE_SIZE)
        cb["unit"] = "GiB/s of live payload"
        res["cpu_baseline"] = cb
    if dist and not args.no_cpu:
        dist.barrier()
    emit(rank, res)
    for b in srcs:
        b.free()
    for b in (d_img, d_desc, d_crc, d_off, d_len):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()


def bench_block_verify_device(args):
    """Device-resident verify-on-read of block images (sync_backup.cpp:345-435 /
    block_console.cpp:543-577 shape): per record the FileInfo is read, its id and
    size checked against the index entry, the payload re-CRC'd and compared with
    the stored crc_.  The resident set is the headline's (1,024 blocks x 1,024
    records of 64 KiB), all records in one launch (tfs_blocks_verify_device)."""
    import tfs_amd.crc as crc
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    nblocks = args.blocks
    nfiles = nblocks * FILES_PER_BLOCK
    rec = FILEINFO + FILE_SIZE
    total = nfiles * rec
    img = crc.DeviceBuffer(ctx, (total + 4095) // 4096 * 4096)
    gblocks = rank_blocks(nblocks * world, world, rank)
    block_bytes = FILES_PER_BLOCK * rec
    for i, g in enumerate(gblocks):
        ctx.synth_fill_device(img.ptr + i * block_bytes, block_bytes, 0x9E3779B97F4A7C15, int(g) * (block_bytes // 8))
    rec_off = np.arange(nfiles, dtype=np.uint64) * rec
    desc = np.zeros(nfiles, crc.DESC_DTYPE)
    desc["offset"], desc["len"] = rec_off + FILEINFO, FILE_SIZE
    d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_crc = crc.DeviceBuffer(ctx, 4 * nfiles)
    ctx.batch_device(d_desc, nfiles, img, d_crc)
    d_off = crc.DeviceBuffer(ctx, 8 * nfiles).upload(rec_off)
    d_len = crc.DeviceBuffer(ctx, 4 * nfiles).upload(np.full(nfiles, FILE_SIZE, np.uint32))
    ctx.write_headers_device(img, d_off, d_len, d_crc, 1, nfiles)   # FileInfo{id = 1 + k, crc_}
    ctx.sync()
    expected = d_crc.download(np.uint32)
    for b in (d_desc, d_off, d_len):
        b.free()
    jobs = np.zeros(nfiles, crc.COMPACT_JOB_DTYPE)
    jobs["src_offset"], jobs["file_id"], jobs["size"] = rec_off, 1 + np.arange(nfiles, dtype=np.uint64), rec
    d_jobs = crc.DeviceBuffer(ctx, jobs.nbytes).upload(jobs)
    d_out = crc.DeviceBuffer(ctx, 4 * nfiles)
    d_st = crc.DeviceBuffer(ctx, 4 * nfiles)
    d_bad = crc.DeviceBuffer(ctx, 4)
    d_bad.zero()

    def step(c=ctx):
        c.blocks_verify_device(img, total, d_jobs, nfiles, d_out, d_st, d_bad)

    for _ in range(max(1, args.warmup)):
        step()
    ctx.sync()
    # parity (test infrastructure): every status 0, every CRC equal to the write pass's,
    # and one block in every --parity-every against the oracle's verify of the same bytes
    if int(d_bad.download(np.uint32, 1)[0]) or (d_st.download(np.int32) != 0).any():
        raise SystemExit("block_verify_device: bad statuses on clean blocks")
    if (d_out.download(np.uint32) != expected).any():
        raise SystemExit("block_verify_device: CRCs differ from the write pass")
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_verify_file.restype = ctypes.c_int32
    ora.oracle_verify_file.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.POINTER(ctypes.c_uint32)]
    checked = 0
    for b in range(0, nblocks, max(1, args.parity_every)):
        host = img.download(np.uint8, block_bytes, b * block_bytes)
        for k in range(0, FILES_PER_BLOCK, 64):
            oc = ctypes.c_uint32()
            code = ora.oracle_verify_file(host.ctypes.data, block_bytes, k * rec, rec, ctypes.byref(oc))
            if code != 0 or oc.value != int(expected[b * FILES_PER_BLOCK + k]):
                raise SystemExit("block_verify_device: oracle disagrees at block %d record %d" % (b, k))
            checked += 1
    def timed(c, fn):
        e0, e1 = crc.Event(c), crc.Event(c)
        # warm up again right before the clock: the parity pass above leaves the GPU
        # idle for seconds, and the first launches after an idle gap run slower
        for _ in range(max(1, args.warmup)):
            fn(c)
        if dist:
            dist.barrier()
        c.sync()
        t0 = time.perf_counter()
        e0.record()
        for _ in range(args.steps):
            fn(c)
        e1.record()
        c.sync()
        if dist:
            dist.barrier()
        return _max_over_ranks(dist, time.perf_counter() - t0), e0.elapsed_ms(e1) / args.steps

    el, kms = timed(ctx, step)
    algo_per_rec = FILEINFO + FILE_SIZE + 40 + 4 + 4   # header + payload + job read, crc + status written
    achieved = nfiles * algo_per_rec / (kms / 1e3) / 1e9
    bv_traffic, bv_src = _pmc_traffic("profiles/r06/pmc/block_verify_device/pmc_summary.json",
                                      "compact_pipe_kernel<true, true, 12, 5, 4, 3", nblocks == 1024)
    res = {
        "metric": "GiB/s payload verified on read from device-resident block images (FileInfo checks + re-CRC)",
        "value": world * args.steps * nfiles * FILE_SIZE / el / 2**30, "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64) 64 KiB payloads behind FileInfo headers, generated on device",
        "config": {"workload": "%d resident blocks x %d records of 64 KiB (%.1f GiB), one launch per pass" % (
            nblocks, FILES_PER_BLOCK, nfiles * FILE_SIZE / 2**30), "files_per_gpu": nfiles,
            "algorithmic_bytes_per_record": algo_per_rec},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": bv_traffic, "traffic_source": bv_src, "traffic_measured_in_this_run": False, "traffic_note": TRAFFIC_NOTE,
                     "kernel": "compact_pipe_kernel<true,true,true> (verify form)", "kernel_ms_avg": kms,
                     "algorithmic_bytes_per_launch": nfiles * algo_per_rec},
        "parity": {"statuses_all_ok": True, "crcs_equal_write_pass": nfiles, "oracle_checked": checked},
    }
    if rank == 0 and not args.no_cpu:
        # the reference's Func::crc over the payloads of resident block 0 copied to host,
        # against the stored crc_ (the loop of sync_backup.cpp:383-435 without the pread)
        host = img.download(np.uint8, block_bytes)
        cb = cpu_baseline(host, np.arange(FILES_PER_BLOCK) * rec + FILEINFO, np.full(FILES_PER_BLOCK, FILE_SIZE),
                          expected[:FILES_PER_BLOCK], args.cpu_seconds, "64 KiB payloads of resident block 0")
        res["cpu_baseline"] = cb
    if dist and not args.no_cpu:
        dist.barrier()
    emit(rank, res)
    for b in (img, d_crc, d_jobs, d_out, d_st, d_bad):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()

