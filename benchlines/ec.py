"""bench.py --workload ec."""
import ctypes
import os
import time

import numpy as np

from benchlines.common import *  # noqa: F401,F403


def bench_ec(args):
    """ErasureCode encode (MarshallingTask, task.cpp:1179-1290) and
    decode of 3 erased members (ReinstateTask) with k=5, m=3 (the reference
    test's configuration), device-resident members of --ec-mib MiB each."""
    import tfs_amd.crc as crc
    from tfs_amd.ec import ErasureCode
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    k, m = 5, 3
    size = args.ec_mib << 20
    if size >= 1 << 31:
        raise SystemExit("ec: member size must stay below 2 GiB (int, erasure_code.h)")
    d = [crc.DeviceBuffer(ctx, size + 64) for _ in range(k + m)]
    for i in range(k):
        ctx.synth_fill_device(d[i], size, 0xEC0 + 31 * rank + i, 0)
    enc = ErasureCode(ctx, k, m)
    if enc.encode_device(d, size) != 0:
        raise SystemExit("ec: encode failed")
    ctx.sync()
    # parity spot check against the oracle on the first 64 KiB (test infrastructure)
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_ec.so"))
    ora.oracle_ec_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    chunk = 64 << 10
    host = [d[i].download(np.uint8, chunk) for i in range(k)] + [np.zeros(chunk, np.uint8) for _ in range(m)]
    pp = (ctypes.c_void_p * (k + m))(*[h.ctypes.data for h in host])
    ora.oracle_ec_encode(k, m, pp, None, chunk)
    for i in range(k, k + m):
        if not (d[i].download(np.uint8, chunk) == host[i]).all():
            raise SystemExit("ec: GPU parity disagrees with oracle")
    erased = [1, 0, 1, 0, 0, 0, 1, 0]   # two data members and one parity member lost
    dec = ErasureCode(ctx, k, m, erased)
    out = {}
    for name, fn, rd, wr in (("encode", lambda: enc.encode_device(d, size), k, m),
                             ("decode", lambda: dec.decode_device(d, size), k, 3)):
        for _ in range(max(1, args.warmup)):
            fn()
        e0, e1 = crc.Event(ctx), crc.Event(ctx)
        if dist:
            dist.barrier()
        ctx.sync()
        t0 = time.perf_counter()
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        ctx.sync()
        if dist:
            dist.barrier()
        el = _max_over_ranks(dist, time.perf_counter() - t0)
        kms = e0.elapsed_ms(e1) / args.steps
        out[name] = {"ms": kms, "GiBs_data": world * args.steps * k * size / el / 2**30,
                     "hbm_GBs": (rd + wr) * size / (kms / 1e3) / 1e9}
    e_traffic, e_src = _pmc_traffic("profiles/r06/pmc/ec/pmc_summary.json", "ec_apply_kernel<3", args.ec_mib == 1536)
    res = {
        "metric": "GiB/s of data encoded (ErasureCode k=5 m=3, Cauchy bitmatrix w=8 ps=128), device-resident",
        "value": out["encode"]["GiBs_data"], "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": out["encode"]["ms"], "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (splitmix64) members",
        "config": {"workload": "SURVEY §8 f4: k=5 + m=3 members of %d MiB" % args.ec_mib},
        "roofline": {"bound": "hbm", "achieved": out["encode"]["hbm_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": out["encode"]["hbm_GBs"] / HBM_PEAK_GBS, "traffic": e_traffic, "traffic_source": e_src, "traffic_measured_in_this_run": False, "traffic_note": TRAFFIC_NOTE,
                     "algorithmic_bytes_per_launch": float(k + m) * size,
                     "kernel": "ec_apply_kernel<3, true>", "kernel_ms_avg": out["encode"]["ms"]},
        "decode": out["decode"],
    }
    if rank == 0 and not args.no_cpu:
        res["cpu_baseline"] = ec_cpu_baseline(d, k, m, args.cpu_seconds, min(4 << 20, size // 1024 * 1024))
    if dist and not args.no_cpu:
        dist.barrier()
    emit(rank, res)
    enc.free()
    dec.free()
    for b in d:
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()


def ec_cpu_baseline(d, k, m, seconds, chunk=4 << 20):
    """The reference's jerasure bitmatrix encode (oracle/_ref/libref_ec.so, built
    from the reference sources) or the oracle's restatement, single thread, over
    the first `chunk` bytes of the same members; its parity must equal the GPU's."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libref_ec.so")
    if os.path.exists(ref_so):
        L, kind = ctypes.CDLL(ref_so), "reference"
        L.ref_ec_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        run = lambda pp: L.ref_ec_encode(k, m, pp, chunk)  # noqa: E731
    else:
        L, kind = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_ec.so")), "port"
        L.oracle_ec_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        run = lambda pp: L.oracle_ec_encode(k, m, pp, None, chunk)  # noqa: E731
    host = [d[i].download(np.uint8, chunk) for i in range(k)] + [np.zeros(chunk, np.uint8) for _ in range(m)]
    pp = (ctypes.c_void_p * (k + m))(*[h.ctypes.data for h in host])
    reps, t0 = 0, time.perf_counter()
    while True:
        run(pp)
        reps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    for i in range(k, k + m):
        if not (d[i].download(np.uint8, chunk) == host[i]).all():
            raise SystemExit("ec: CPU baseline parity disagrees with the GPU")
    try:
        # jerasure keeps process-wide byte counters (jerasure.cpp:42-44, bumped per
        # packet at :336-340) that every encoding thread writes: threads of one
        # library copy serialise on that cache line.  Each thread here runs its own
        # loaded copy of the library (as separate dataserver processes would).
        import shutil
        import tempfile
        tmpd = tempfile.mkdtemp(prefix="tfs_ec_ref_")

        def make(i):
            par = [np.zeros(chunk, np.uint8) for _ in range(m)]
            ptrs = (ctypes.c_void_p * (k + m))(*([h.ctypes.data for h in host[:k]] + [p.ctypes.data for p in par]))
            make.keep.append((par, ptrs))
            if kind != "reference":
                return lambda: run(ptrs)
            cp = os.path.join(tmpd, "libref_ec_%d.so" % i)
            shutil.copyfile(ref_so, cp)
            Li = ctypes.CDLL(cp, mode=os.RTLD_LOCAL)
            Li.ref_ec_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
            make.libs.append(Li)
            return lambda: Li.ref_ec_encode(k, m, ptrs, chunk)
        make.keep, make.libs = [], []
        try:
            calls, adt, threads = _allcore_threads(make, min(3.0, seconds))
        finally:
            shutil.rmtree(tmpd, ignore_errors=True)
        for par, _ in make.keep:
            if not all((par[j] == host[k + j]).all() for j in range(m)):
                raise SystemExit("ec: all-core CPU parity disagrees with the GPU")
        allcore = {"value": calls * k * chunk / adt / 2**30, "cores": threads, "nproc": os.cpu_count(),
                   "cpu_model": _cpu_model(), "kind": kind,
                   "cores_source": "sched affinity capped by the cgroup cpu.max quota",
                   "sample": "%d encodes over %d threads, one loaded copy of the library per thread, %.1f s" % (
                       calls, threads, adt)}
    except Exception as e:  # reported, never fatal
        allcore = {"error": str(e)}
    return {"value": reps * k * chunk / dt / 2**30, "unit": "GiB/s", "cores": 1, "kind": kind,
            "sample": "%d encodes of k=%d x %d MiB (first bytes of the same members), jerasure_bitmatrix_encode "
                      "w=8 ps=128, single thread, %.1f s" % (reps, k, chunk >> 20, dt),
            "allcore": allcore}

