"""bench.py --workload loopback."""
import ctypes
import os
import time

import numpy as np

from benchlines.common import *  # noqa: F401,F403


def close_tail(us, ph):
    """Where the slowest closes' time went: the mean of each
    CloseTiming phase over the closes at or above p99 against those at or below p50,
    and how many of each saw a resident-kernel relaunch or a ring-full launch during
    their batch's verify."""
    import tfs_amd.dataserver as ds
    p50, p99 = np.percentile(us, 50), np.percentile(us, 99)
    out = {}
    for name, sel in (("at_or_above_p99", us >= p99), ("at_or_below_p50", us <= p50)):
        sub = ph[sel]
        d = {k: float(sub[:, i].mean()) for i, k in enumerate(ds.CLOSE_PHASES[:6])}
        d["total_us"] = float(us[sel].mean())
        d["closes"] = int(sel.sum())
        d["with_relaunch"] = int((sub[:, 8] > 0).sum())
        d["with_ring_full"] = int((sub[:, 9] > 0).sum())
        out[name] = d
    out["note"] = ("phases of a close (ds_harness.h CloseTiming): claim = batch slot, copy = payload into the gather "
                   "buffer, wait = until the verdicts are in (a leader's wait is its own verify call: lead_wait + "
                   "verify), append = FileInfo|payload persist; with_relaunch = closes whose batch verify spanned a "
                   "resident kernel launch")
    return out


def bench_loopback(args):
    """BASELINE configs[0]: src/dataserver write + verify over one 64 MiB block of
    1024 x 64 KiB synthetic payloads, single-process loopback (no nameserver).
    Per file: stage (DataFile::set_data), CRC (DataFile::get_crc), compare with the
    client CRC, append FileInfo|payload; then verify every record against its
    stored crc_.  GPU leg (the value): the dataserver-shaped C++ harness through
    the C ABI, 8 worker threads (thread_count default, base_service.cpp:163-166)
    closing through the CloseBatcher.  CPU legs (cpu_baseline, test
    infrastructure): the oracle's restatement of the same loop, one thread and
    all cores (one block per thread)."""
    import concurrent.futures as cf
    import tfs_amd.crc as crc
    import tfs_amd.dataserver as ds
    from tfs_amd.synth import synth_bytes
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    n, L = FILES_PER_BLOCK, FILE_SIZE
    pay = synth_bytes(0x9E3779B97F4A7C15 + rank, n * L)
    offs = np.arange(n, dtype=np.uint64) * L
    client = ctx.batch(pay, offs, np.full(n, L, np.uint32))  # the client's Func::crc (tfs_file.cpp:961-963)
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_loopback_block.restype = ctypes.c_int32
    ora.oracle_loopback_block.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]

    def cpu_once(stage, image, stored):
        return ora.oracle_loopback_block(pay.ctypes.data, n, L, client.ctypes.data, stage.ctypes.data,
                                         image.ctypes.data, stored.ctypes.data)

    ora.oracle_loopback_block_fn.restype = ctypes.c_int32
    ora.oracle_loopback_block_fn.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint32, ctypes.c_int32] + \
        [ctypes.c_void_p] * 4

    def cpu_once_fn(fn, stage, image, stored):
        return ora.oracle_loopback_block_fn(fn, pay.ctypes.data, n, L, client.ctypes.data, stage.ctypes.data,
                                            image.ctypes.data, stored.ctypes.data)

    bufs = (np.zeros(L, np.uint8), np.zeros(n * (L + FILEINFO), np.uint8), np.zeros(n, np.uint32))
    if cpu_once(*bufs) != 0:
        raise SystemExit("loopback: CPU restatement rejects the GPU client CRCs")
    cpu_image = bufs[1].copy()

    # The block's storage: page-locked buffers allocated once (a dataserver
    # preallocates its blocks), so the final verify reads the block in place.
    pool = ds.BlockImagePool(ctx, 2, n * (L + FILEINFO) + 4096)

    # One CloseBatcher per thread count, created once (DataService::initialize),
    # with the harness's rule (CloseBatcher::batch_for): one lease per batch up to
    # 8 threads, threads/16 beyond (4 of 64).  Several batches are in flight at
    # once, their round trips overlapping; with the resident kernel a batch costs
    # no launch, so small batches pay (tools/loopback_probe.py,
    # profiles/r03/s2/loopback_batches/).
    # (Lease buffers from a page-locked LeaseBufferPool, checked in place with no
    # gather copy, measured 7-10 % slower in tools/loopback_probe.py: the gather
    # copy costs ~0.75 us per close)
    close_batch = {8: 1, 64: 4}
    batchers = {t: ds.CloseBatcher(ctx, max_batch=b, max_wait_us=100) for t, b in close_batch.items()}

    def gpu_once(threads=8):
        blk = ds.LogicBlock(1, pool=pool)
        bad = ds.loopback_block(ctx, pay, n, L, client, threads, blk, batchers[threads])
        return bad, blk

    bad, blk = gpu_once()
    if bad != 0:
        raise SystemExit("loopback: harness reported %d bad files" % bad)
    # parity: every record the harness persisted equals the CPU loop's record for that file id
    m, _ = blk.metas()
    raw = blk.raw()
    for i in np.linspace(0, n - 1, 64).astype(np.int64):
        k = int(np.nonzero(m["file_id"] == i + 1)[0][0])
        o = int(m["offset"][k])
        got = raw[o:o + FILEINFO + L]
        exp = cpu_image[i * (L + FILEINFO):(i + 1) * (L + FILEINFO)]
        if not ((got[FILEINFO:] == exp[FILEINFO:]).all() and (got[32:36] == exp[32:36]).all()):
            raise SystemExit("loopback: harness record %d differs from the CPU loop" % i)
    blk.free()
    reps = max(args.steps, 4)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        bad, blk = gpu_once()
        blk.free()
        if bad:
            raise SystemExit("loopback: bad files")
    el = _max_over_ranks(dist, time.perf_counter() - t0)
    # 64 leases closing at once (a busy dataserver): larger CloseBatcher batches
    t1 = time.perf_counter()
    for _ in range(reps):
        bad, blk = gpu_once(64)
        blk.free()
        if bad:
            raise SystemExit("loopback: bad files (64 threads)")
    el64 = time.perf_counter() - t1
    # phase breakdown: the whole-block verify alone, and the appends alone (no CRC)
    bad, blk = gpu_once()
    t2 = time.perf_counter()
    for _ in range(reps):
        ds.verify_block(ctx, blk)
    verify_ms = (time.perf_counter() - t2) / reps * 1e3
    blk.free()
    t3 = time.perf_counter()
    for _ in range(reps):
        b2 = ds.LogicBlock(2)
        for i in range(n):
            b2.append(i + 1, memoryview(pay)[i * L:(i + 1) * L], int(client[i]))
        b2.free()
    append_ms = (time.perf_counter() - t3) / reps * 1e3
    res = {
        "metric": "GiB/s payload written + verified, single-process loopback of one 64 MiB block (BASELINE configs[0])",
        "value": world * reps * n * L / el / 2**30, "unit": "GiB/s", "n_gpus": world, "steps": reps, "warmup": 1,
        "ms_per_step": el / reps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (splitmix64) 1024 x 64 KiB payloads",
        "config": {"workload": "configs[0]: DataFile set_data -> close (CloseBatcher, 8 worker threads) -> "
                               "FileInfo|payload append; then verify_block of the whole block",
                   "block_storage": "page-locked, allocated once (%d buffers)" % pool.size(),
                   "files": n, "file_size": L, "close_batch": close_batch},
        "threads64_GiBs": reps * n * L / el64 / 2**30,
        "phases_ms": {"verify_block": verify_ms, "append_only_python": append_ms},
    }
    # Write-path latency (SURVEY §7 "Batching vs. latency"): the scalar drop-in on
    # one 64 KiB payload, and a CloseBatcher close with 1, 8 and 64 leases closing
    # at once (the reference's close is one RPC per file on thread_count workers).
    lat = {}
    sl = ds.scalar_latency(300)
    lat["scalar_tfs_crc32_64KiB"] = {"p50_us": float(np.percentile(sl, 50)), "p99_us": float(np.percentile(sl, 99)),
                                     "calls": int(sl.size)}
    st0 = ctx.stats()
    for nl, it in ((1, 300), (8, 64), (64, 8)):
        cl, ph = ds.close_latency(ctx, nl, it, phases=True)
        lat["close_%d_leases" % nl] = {"p50_us": float(np.percentile(cl, 50)), "p99_us": float(np.percentile(cl, 99)),
                                       "closes": int(cl.size), "tail": close_tail(cl, ph)}
    st1 = ctx.stats()
    res["latency"] = lat
    res["latency_counters"] = {k: st1[k] - st0[k] for k in ("resident_launches", "resident_files",
                                                            "resident_ring_full", "lone_calls", "host_calls")}
    # resident kernel over this whole line: launches (first + relaunches after
    # idle or lifetime exits) against the files it took
    launches, rfiles = ctx.resident_stats()
    res["resident_kernel"] = {"launches": int(launches), "files": int(rfiles),
                              "ring": {1: "device memory", 0: "host memory"}.get(ctx.resident_ring_in_device_memory(),
                                                                                 "not set up")}
    # PCIe bytes of one loopback: every payload crosses once for the close check
    # (zero-copy reads of the lease buffers) and once for the whole-block verify.
    pcie_bytes = 2.0 * n * L
    ceil = pcie_ceiling(ctx, dist=dist)
    res["roofline"] = {"bound": "pcie", "achieved": reps * pcie_bytes / el / 1e9, "peak": ceil["h2d_GBs"],
                       "unit": "GB/s (per GPU)", "frac": reps * pcie_bytes / el / 1e9 / ceil["h2d_GBs"],
                       "traffic": None, "peak_source": ceil["source"],
                       "kernel": "crc_resident_kernel (close batches, no launch per batch) + compact_pipe_kernel verify form (whole block, zero-copy)",
                       "note": "latency-bound: one GPU round trip per batch of concurrent closes"}
    if rank == 0 and not args.no_cpu:
        # CPU legs (test infrastructure): the restated loop of config 1 with the
        # reference's own Func::crc text inside (oracle/_ref, built from
        # src/common/func.{h,cpp}); one thread, then one block per thread on every
        # core this process may use.
        fn, kind = _ref_crc_fn()
        secs = min(args.cpu_seconds, 10.0)
        t0, k = time.perf_counter(), 0
        while True:
            if cpu_once_fn(fn, *bufs) != 0:
                raise SystemExit("loopback: CPU loop rejects the client CRCs")
            k += 1
            if time.perf_counter() - t0 >= secs:
                break
        one = k * n * L / (time.perf_counter() - t0) / 2**30
        threads = _cpu_budget()
        tb = [(np.zeros(L, np.uint8), np.zeros(n * (L + FILEINFO), np.uint8), np.zeros(n, np.uint32))
              for _ in range(threads)]
        with cf.ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda b: cpu_once_fn(fn, *b), tb))
            t0 = time.perf_counter()
            rounds = 0
            while time.perf_counter() - t0 < min(secs, 5.0):
                list(ex.map(lambda b: cpu_once_fn(fn, *b), tb))
                rounds += 1
            allc = rounds * threads * n * L / (time.perf_counter() - t0) / 2**30
        res["cpu_baseline"] = {
            "value": one, "unit": "GiB/s", "cores": 1, "kind": kind,
            "sample": "%d loopbacks of the 1024 x 64 KiB block (stage, crc, compare, append, then re-CRC verify), "
                      "restated loop around the reference's Func::crc text, single thread, %.1f s" % (k, secs),
            "allcore": {"value": allc, "cores": threads, "nproc": os.cpu_count(), "cpu_model": _cpu_model(),
                        "cores_source": "sched affinity capped by the cgroup cpu.max quota"},
        }
        res["vs_cpu_allcore"] = res["value"] / allc
    if dist and not args.no_cpu:
        dist.barrier()
    emit(rank, res)
    for b in batchers.values():
        b.free()
    pool.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()

