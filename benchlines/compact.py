"""bench.py --workload compact: BASELINE configs[3], compaction of fragmented
block images held in page-locked host memory (CompactTask::real_compact,
src/dataserver/task.cpp:713-836, with the re-CRC), PCIe included."""
import ctypes
import os
import time

import numpy as np

from benchlines.common import *  # noqa: F401,F403


def bench_compact(args):
    """BASELINE configs[3]: host block images -> pinned H2D -> verify live files +
    repack on the GPU -> D2H of the new block, 4096 fragmented 64 MiB blocks."""
    import tfs_amd.crc as crc
    from tfs_amd.synth import synth_bytes  # noqa: F401
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    psize = FILE_SIZE
    nfiles, rec = FILES_PER_BLOCK, FILEINFO + psize
    blk_bytes = nfiles * rec
    ndistinct = 8
    nblocks = args.compact_blocks
    srcs, dests = [], []
    metas = np.zeros(nfiles, crc.META_DTYPE)
    metas["file_id"] = np.arange(1, nfiles + 1)
    metas["offset"] = np.arange(nfiles) * rec
    metas["size"] = rec
    flags = _fragmented_flags(nfiles)
    d_img = crc.DeviceBuffer(ctx, blk_bytes + 64)
    d_desc = crc.DeviceBuffer(ctx, 16 * nfiles)
    d_crc = crc.DeviceBuffer(ctx, 4 * nfiles)
    d_off = crc.DeviceBuffer(ctx, 8 * nfiles).upload(np.arange(nfiles, dtype=np.uint64) * rec)
    d_len = crc.DeviceBuffer(ctx, 4 * nfiles).upload(np.full(nfiles, psize, np.uint32))
    desc = np.zeros(nfiles, crc.DESC_DTYPE)
    desc["offset"] = np.arange(nfiles) * rec + FILEINFO
    desc["len"] = psize
    d_desc.upload(desc)
    for b in range(ndistinct):
        # build one real block image (checksum-on-write + FileInfo headers) on the GPU, then to pinned host
        ctx.synth_fill_device(d_img, blk_bytes + 64 - (blk_bytes + 64) % 8, 0xB10C + 97 * b + rank, 0)
        ctx.batch_device(d_desc, nfiles, d_img, d_crc)
        ctx.write_headers_device(d_img, d_off, d_len, d_crc, 1, nfiles)  # file ids are per block
        ctx.sync()
        p = crc.PinnedBuffer(ctx, blk_bytes)
        p.array[:] = d_img.download(np.uint8, blk_bytes)
        srcs.append(p)
        dests.append(crc.PinnedBuffer(ctx, blk_bytes))
    live = int((flags == 0).sum())
    jobs = (crc.BlockJob * nblocks)()
    dm = np.zeros((4, nfiles), crc.META_DTYPE)
    oks = np.zeros((4, nfiles), np.uint8)
    for j in range(nblocks):
        x = jobs[j]
        x.src_image, x.src_len = srcs[j % ndistinct].ptr, blk_bytes
        x.metas, x.flags, x.n = metas.ctypes.data, flags.ctypes.data, nfiles
        x.dest_image, x.dest_cap = dests[j % ndistinct].ptr, blk_bytes
        x.dest_metas, x.crc_ok = dm[j % 4].ctypes.data, oks[j % 4].ctypes.data
    warm = (crc.BlockJob * min(8, nblocks))(*jobs[:min(8, nblocks)])
    ctx.blocks_compact(warm)
    # parity: the first block against the oracle's real_compact restatement
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_compact.restype = ctypes.c_int64
    ora.oracle_compact.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4
    mo = metas["offset"].astype(np.int64)
    ms = metas["size"].astype(np.int32)
    odest = np.zeros(blk_bytes, np.uint8)
    doff = np.zeros(nfiles, np.int64)
    dsz = np.zeros(nfiles, np.int32)
    ook = np.zeros(nfiles, np.uint8)
    w = ora.oracle_compact(srcs[0].ptr, mo.ctypes.data, ms.ctypes.data, flags.ctypes.data, nfiles,
                           odest.ctypes.data, doff.ctypes.data, dsz.ctypes.data, ook.ctypes.data)
    if w != warm[0].dest_len or not (odest[:w] == dests[0].array[:w]).all():
        raise SystemExit("compact: GPU repack disagrees with oracle")
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    rc = ctx.blocks_compact(jobs)
    el = _max_over_ranks(dist, time.perf_counter() - t0)
    if rc != 0 or any(jobs[j].status != 0 for j in range(nblocks)):
        raise SystemExit("compact: unexpected CRC mismatches on clean blocks")
    src_total = float(world) * nblocks * blk_bytes
    live_total = float(world) * nblocks * live * psize
    # Zero-copy form: the kernel reads only the live records from the pinned
    # source image and writes the new block into the pinned destination.
    pcie_block = 2 * live * rec
    ceil = pcie_ceiling(ctx, dist=dist)
    pcie_gbs = float(nblocks) * pcie_block / el / 1e9
    res = {
        "metric": "GiB/s of live payload compacted (re-read + re-CRC + repack), host block images, PCIe included",
        "value": live_total / el / 2**30, "unit": "GiB/s of live payload", "n_gpus": world,
        "source_block_GiBs": src_total / el / 2**30,
        "steps": nblocks, "warmup": len(warm), "ms_per_step": el / nblocks * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic 64 KiB files, 1024 per block, evens + every 3rd of the rest deleted (%d live)" % live,
        "config": {"workload": "BASELINE configs[3]: %d fragmented blocks (%d distinct pinned images cycled)" % (
            nblocks, ndistinct), "live_bytes_per_block": live * rec,
            "pcie_bytes_per_block": pcie_block,
            "distinct_note": "%d distinct page-locked source images (and destinations) are cycled over the %d blocks: "
                             "4,096 distinct 64 MiB source images would need 256 GiB of page-locked host memory per GPU "
                             "(512 GiB with their destinations) "
                             "(the box allows ~270 GiB per command, all ranks together); the GPU keeps no copy of "
                             "an image, so every live byte of every block still crosses PCIe each time, and %d MiB "
                             "is far above every GPU cache" % (ndistinct, nblocks, ndistinct * blk_bytes >> 20),
            "transfer": "zero-copy: fused kernel reads live records from pinned host memory and writes the "
                        "new block to pinned host memory"},
        "pcie_GBs": float(world) * nblocks * pcie_block / el / 1e9,
        "roofline": {"bound": "pcie", "achieved": pcie_gbs, "peak": ceil["h2d_GBs"] + ceil["d2h_GBs"],
                     "unit": "GB/s (per GPU, both directions)", "frac": pcie_gbs / (ceil["h2d_GBs"] + ceil["d2h_GBs"]),
                     "peak_source": ceil["source"] + " (H2D + D2H: the link is full duplex)",
                     "duplex_measured_GBs": ceil["duplex_GBs"],
                     "frac_of_duplex_measured": pcie_gbs / ceil["duplex_GBs"],
                     "duplex_source": ceil["duplex_source"],
                     "traffic": "live records read over PCIe + the new block written back (%d B per block)" %
                                pcie_block},
    }
    if rank == 0 and not args.no_cpu:
        # CPU restatement of CompactTask::real_compact with the added re-CRC
        # (oracle_compact, task.cpp:713-836) over the same pinned source images,
        # single thread; the dataserver itself is not buildable here (tbsys/tbnet).
        reps, t0 = 0, time.perf_counter()
        while True:
            wc = ora.oracle_compact(srcs[reps % ndistinct].ptr, mo.ctypes.data, ms.ctypes.data, flags.ctypes.data,
                                    nfiles, odest.ctypes.data, doff.ctypes.data, dsz.ctypes.data, ook.ctypes.data)
            if wc != w or not ook[flags == 0].all():
                raise SystemExit("compact: oracle baseline disagrees")
            reps += 1
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {
            "value": reps * live * psize / dt / 2**30, "unit": "GiB/s of live payload", "cores": 1,
            "kind": "port", "source_block_GiBs": reps * blk_bytes / dt / 2**30,
            "sample": "%d compactions of the %d pinned source block images (re-CRC of %d live files + repack), "
                      "oracle_compact single thread, %.1f s" % (reps, ndistinct, live, dt),
            "allcore": _compact_allcore(ora, [b.ptr for b in srcs], mo, ms, flags, nfiles, odest.size, w,
                                        live * psize, blk_bytes, min(3.0, args.cpu_seconds))}
    if dist and not args.no_cpu:
        dist.barrier()
    emit(rank, res)
    for b in srcs + dests:
        b.free()
    for b in (d_img, d_desc, d_crc, d_off, d_len):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()

