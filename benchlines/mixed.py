"""bench.py --workload mixed."""
import ctypes
import os
import time

import numpy as np

from benchlines.common import *  # noqa: F401,F403


def bench_mixed(args):
    """The dataserver's own mix on one GPU: packet workers closing 64 KiB writes
    (DataManagement::close_write_file, data_management.cpp:173-236, through
    CloseBatcher and the resident kernel) while the task thread runs a block
    compaction (dataservice.cpp:2915-2918 -> task.cpp:713-836) or a whole-set
    verify.  The headline verify launch (configs[1]: 1 M x 64 KiB) and a
    compaction of the same resident blocks (every 3rd record live, one
    tfs_compact_jobs_device launch) are timed with HIP events, interleaved
    over rounds, in three modes: no closes; closes flowing with the resident
    kernel's CUs left out of the throughput grid (the product);
    closes flowing with every CU asked for (tfs_crc32_set_cu_reserve(ctx, 0)).
    Reports each launch's stretch against the idle mode and the close latency
    in each mode.  Results are checked: every verdict 1 and no mismatch after
    every timed launch; block 0's compaction against the oracle."""
    import tfs_amd.crc as crc
    import tfs_amd.dataserver as ds
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    nblocks = args.blocks
    nfiles = nblocks * FILES_PER_BLOCK
    rec = FILEINFO + FILE_SIZE
    blk = FILES_PER_BLOCK * rec
    total = nblocks * blk
    img = crc.DeviceBuffer(ctx, (total + 4095) // 4096 * 4096)
    ctx.synth_fill_device(img, (total + 7) // 8 * 8, 0x5EED + rank, 0)
    rec_off = np.arange(nfiles, dtype=np.uint64) * rec
    desc = np.zeros(nfiles, crc.DESC_DTYPE)
    desc["offset"], desc["len"] = rec_off + FILEINFO, FILE_SIZE
    d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_crc = crc.DeviceBuffer(ctx, 4 * nfiles)
    ctx.batch_device(d_desc, nfiles, img, d_crc)
    d_roff = crc.DeviceBuffer(ctx, rec_off.nbytes).upload(rec_off)
    d_len = crc.DeviceBuffer(ctx, 4 * nfiles).upload(np.full(nfiles, FILE_SIZE, np.uint32))
    ctx.write_headers_device(img, d_roff, d_len, d_crc, 1, nfiles)
    ctx.sync()
    desc["aux"] = d_crc.download(np.uint32)
    d_vdesc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    for b in (d_desc, d_roff, d_len):
        b.free()
    d_ok = crc.DeviceBuffer(ctx, nfiles)
    d_bad = crc.DeviceBuffer(ctx, 4)
    live = np.arange(0, FILES_PER_BLOCK, 3)
    nl = live.size
    jobs = np.zeros(nblocks * nl, crc.COMPACT_JOB_DTYPE)
    bidx = np.repeat(np.arange(nblocks, dtype=np.uint64), nl)
    loc = np.tile(np.arange(nl, dtype=np.uint64) * rec, nblocks)
    jobs["src_offset"] = bidx * blk + np.tile(live.astype(np.uint64) * rec, nblocks)
    jobs["dest_offset"] = bidx * (nl * rec) + loc
    jobs["file_id"] = 1 + bidx * FILES_PER_BLOCK + np.tile(live.astype(np.uint64), nblocks)
    jobs["size"] = rec
    jobs["new_offset"] = loc.astype(np.int32)
    d_jobs = crc.DeviceBuffer(ctx, jobs.nbytes).upload(jobs)
    d_dst = crc.DeviceBuffer(ctx, jobs.size * rec + 64)
    d_st = crc.DeviceBuffer(ctx, 4 * jobs.size)
    d_bad2 = crc.DeviceBuffer(ctx, 4)

    def verify():
        ctx.verify_device(d_vdesc, nfiles, img, None, d_ok, d_bad)

    def compact():
        ctx.compact_jobs_device(img, total, d_jobs, int(jobs.size), d_dst, None, d_st, d_bad2)

    def check(what):
        if int(d_bad.download(np.uint32)[0]) or int(d_bad2.download(np.uint32)[0]):
            raise SystemExit("mixed: mismatches on clean data (%s)" % what)

    for b in (d_bad, d_bad2):
        b.zero()
    verify()
    compact()
    ctx.sync()
    check("warmup")
    # parity (outside the timed region): block 0's compaction against the oracle's real_compact
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_compact.restype = ctypes.c_int64
    ora.oracle_compact.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4
    host = img.download(np.uint8, blk)
    fl = np.where(np.arange(FILES_PER_BLOCK) % 3 == 0, 0, 1).astype(np.int32)
    mo = np.arange(FILES_PER_BLOCK, dtype=np.int64) * rec
    ms = np.full(FILES_PER_BLOCK, rec, np.int32)
    odest = np.zeros(blk, np.uint8)
    doff = np.zeros(FILES_PER_BLOCK, np.int64)
    dsz = np.zeros(FILES_PER_BLOCK, np.int32)
    ook = np.zeros(FILES_PER_BLOCK, np.uint8)
    wlen = ora.oracle_compact(host.ctypes.data, mo.ctypes.data, ms.ctypes.data, fl.ctypes.data, FILES_PER_BLOCK,
                              odest.ctypes.data, doff.ctypes.data, dsz.ctypes.data, ook.ctypes.data)
    if not (d_dst.download(np.uint8, int(wlen)) == odest[:wlen]).all():
        raise SystemExit("mixed: GPU compaction disagrees with the oracle")
    modes = ("idle", "closes", "closes_all_cus")
    ctx_full_grid = ctx.throughput_grid()
    res = {m: {"verify_ms": [], "compact_ms": [], "grid": [], "closes": 0, "close_s": 0.0, "lat": []} for m in modes}
    K = max(1, args.steps // 2)
    for rnd in range(max(1, args.rounds)):
        for m in modes:
            ctx.set_cu_reserve(m != "closes_all_cus")
            cs = None
            if m == "idle":  # no resident kernel alive or recently used: the full grid
                t_w = time.perf_counter()
                while ctx.throughput_grid() != ctx_full_grid and time.perf_counter() - t_w < 1.0:
                    time.sleep(0.01)
            else:
                cs = ds.CloseStream(ctx, nleases=8)
                time.sleep(0.05)  # the close stream in steady state (resident kernel up)
            d_ok.zero()
            ctx.sync()
            t0 = time.perf_counter()
            res[m]["grid"].append(ctx.throughput_grid())
            for fn, key in ((verify, "verify_ms"), (compact, "compact_ms")):
                e0, e1 = crc.Event(ctx), crc.Event(ctx)
                e0.record()
                for _ in range(K):
                    fn()
                e1.record()
                res[m][key].append(e0.elapsed_ms(e1) / K)
            ctx.sync()
            el = time.perf_counter() - t0
            if cs is not None:
                rc, cnt, lat = cs.stop()
                if rc != 0:
                    raise SystemExit("mixed: close stream failed with %d" % rc)
                res[m]["closes"] += cnt
                res[m]["close_s"] += el + 0.05
                res[m]["lat"].append(lat)
            check(m)
            if not bool((d_ok.download(np.uint8, nfiles) == 1).all()):
                raise SystemExit("mixed: verify left files without a verdict (%s)" % m)
    ctx.set_cu_reserve(True)
    out = {}
    idle_v = float(np.median(res["idle"]["verify_ms"]))
    idle_c = float(np.median(res["idle"]["compact_ms"]))
    for m in modes:
        r = res[m]
        v, c = float(np.median(r["verify_ms"])), float(np.median(r["compact_ms"]))
        o = {"verify_ms_median": v, "verify_ms": r["verify_ms"], "compact_ms_median": c, "compact_ms": r["compact_ms"],
             "verify_stretch": v / idle_v - 1.0, "compact_stretch": c / idle_c - 1.0, "grid": r["grid"]}
        if r["lat"]:
            lat = np.concatenate(r["lat"])
            o.update(close_p50_us=float(np.percentile(lat, 50)), close_p99_us=float(np.percentile(lat, 99)),
                     close_p999_us=float(np.percentile(lat, 99.9)), close_max_us=float(lat.max()),
                     closes_over_1ms=int((lat > 1000).sum()), closes=r["closes"],
                     closes_per_s=r["closes"] / r["close_s"])
        out[m] = o
    line = {
        "metric": "GiB/s CRC32 verify, device-resident 64 KiB files, with 64 KiB closes flowing on the same GPU",
        "value": world * nfiles * FILE_SIZE / (out["closes"]["verify_ms_median"] / 1e3) / 2**30, "unit": "GiB/s",
        "n_gpus": world, "steps": K, "warmup": 1, "ms_per_step": out["closes"]["verify_ms_median"],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 payloads, FileInfo-headed block images); closes of one 64 KiB payload",
        "config": {"workload": "mixed: %d blocks x 1024 x 64 KiB verify + compaction of every 3rd record (%d "
                               "records, one launch), interleaved over %d rounds with and without 8 closing "
                               "threads through CloseBatcher" % (nblocks, jobs.size, max(1, args.rounds)),
                   "value_mode": "closes (CU reserve on: the product)"},
        "modes": out,
        "roofline": {"bound": "hbm", "achieved": nfiles * ALGO_BYTES_PER_FILE / (out["closes"]["verify_ms_median"] / 1e3)
                     / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": nfiles * ALGO_BYTES_PER_FILE / (out["closes"]["verify_ms_median"] / 1e3) / 1e9 / HBM_PEAK_GBS,
                     "traffic": None, "kernel": "crc_files_kernel<1> (verify) beside crc_resident_kernel"},
        "parity": {"compaction_block0_vs_oracle": True, "verdicts_all_ok": True},
    }
    if dist and not args.no_cpu:
        dist.barrier()
    emit(rank, line)
    for b in (img, d_crc, d_vdesc, d_ok, d_bad, d_jobs, d_dst, d_st, d_bad2):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()

