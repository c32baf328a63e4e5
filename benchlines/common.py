"""Shared pieces of bench.py's lines (constants, rank plumbing, CPU baselines, PCIe ceiling)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

__all__ = ['ROOT', 'emit', 'DATA_SEED', 'FILE_SIZE', 'FILES_PER_BLOCK', 'FILEINFO', 'HBM_PEAK_GBS', 'ALGO_BYTES_PER_FILE', 'rank_blocks', '_init_gloo', 'TRAFFIC_NOTE', 'HEADLINE_KERNEL', 'PACKET_KERNEL', '_pmc_traffic', 'cpu_baseline', '_dist_init', '_NUMA', '_bind_numa', '_gather_floats', 'per_rank', '_max_over_ranks', 'BLOCK_DATA', 'zipf_sizes', '_fragmented_flags', 'live_bytes_total', '_ref_crc_fn', '_PCIE', 'pcie_ceiling', '_pcie_measure', '_cpu_budget', '_allcore_threads', '_cpu_model', 'e2e_blocks', '_compact_allcore']


FILE_SIZE = 65536


FILES_PER_BLOCK = 1024


FILEINFO = 36


HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md (8.0 TB/s)


ALGO_BYTES_PER_FILE = FILE_SIZE + 16 + 4 + 1  # payload + descriptor + crc out + verdict


DATA_SEED = 0x9E3779B97F4A7C15  # the headline's synthetic stream (splitmix64 seed)


def rank_blocks(total_blocks, world, rank):
    """Global block ids owned by `rank`: partition by block id (block_id % world == rank)."""
    return np.arange(rank, total_blocks, world, dtype=np.int64)


def _init_gloo(dist):
    """init_process_group(gloo) with the process's stdout pointed at stderr meanwhile:
    gloo prints "[Gloo] Rank r is connected to ..." on stdout in every rank, and the
    line the driver reads from rank 0's stdout must be the only one there."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group(backend="gloo")
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


TRAFFIC_NOTE = ("quoted: HBM bytes per launch from the committed rocprofv3 PMC passes of this same command at "
                "full size (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, tools/pmc_summary.py), not counted in this "
                "run; null when this run is not the profiled configuration")


HEADLINE_KERNEL = "crc_files_kernel<1, 4, 3>"


PACKET_KERNEL = "packet_files_kernel<1>"


def _pmc_traffic(rel, kernel, applies):
    """HBM bytes per launch from a committed rocprofv3 PMC summary of this same
    command at full size (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), or
    (None, None) when the run is not the one profiled."""
    if not applies or os.environ.get("TFS_CRC_VARIANT", "0") != "0":
        return None, None
    try:
        with open(os.path.join(ROOT, rel)) as fh:
            pmc = json.load(fh)
    except (OSError, ValueError):
        return None, None
    if pmc.get("kernel") != kernel:
        return None, None
    return pmc.get("traffic_bytes_per_launch"), rel


def cpu_baseline(sample_u8, offs, lens, expected, seconds, what="64 KiB payloads", seed=0):
    """Single-thread reference CRC over a bounded sample (test infrastructure)."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libref_crc.so")
    ora_so = os.path.join(ROOT, "oracle", "liboracle_crc.so")
    if os.path.exists(ref_so):
        L = ctypes.CDLL(ref_so)
        f = L.ref_func_crc
        kind = "reference"
    else:
        L = ctypes.CDLL(ora_so)
        f = L.oracle_crc
        kind = "port"
    f.restype = ctypes.c_uint32
    f.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int32]
    base = sample_u8.ctypes.data
    nbytes = 0
    passes = 0
    t0 = time.perf_counter()
    while True:
        for i in range(len(offs)):
            c = f(seed, base + int(offs[i]), int(lens[i]))
            if c != int(expected[i]):
                raise SystemExit("cpu baseline disagrees with GPU expected crc at file %d" % i)
            nbytes += int(lens[i])
        passes += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    # All-core variant: the same Func::crc (the reference text when built) on every
    # CPU this process may use, one file per task (oracle_crc_batch_mt_fn's pthreads).
    allcore = None
    try:
        O = ctypes.CDLL(ora_so)
        O.oracle_crc_batch_mt_fn.restype = ctypes.c_int
        O.oracle_crc_batch_mt_fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_int]
        import tfs_amd.crc as crc
        d = np.zeros(len(offs), crc.DESC_DTYPE)
        d["offset"] = offs
        d["len"] = lens
        d["aux"] = seed
        out = np.zeros(len(offs), np.uint32)
        fn, _ = _ref_crc_fn()
        threads = _cpu_budget()
        O.oracle_crc_batch_mt_fn(fn, d.ctypes.data, len(offs), base, out.ctypes.data, threads)
        t1 = time.perf_counter()
        reps = 0
        while True:
            O.oracle_crc_batch_mt_fn(fn, d.ctypes.data, len(offs), base, out.ctypes.data, threads)
            reps += 1
            if time.perf_counter() - t1 >= min(3.0, seconds):
                break
        ad = time.perf_counter() - t1
        assert (out == expected).all()
        allcore = {"value": reps * float(np.sum(lens)) / ad / 2**30, "cores": threads, "nproc": os.cpu_count(),
                   "cpu_model": _cpu_model(), "kind": kind,
                   "cores_source": "sched affinity capped by the cgroup cpu.max quota"}
    except Exception as e:  # reported, never fatal
        allcore = {"error": str(e)}
    return {
        "value": nbytes / dt / 2**30,
        "unit": "GiB/s",
        "cores": 1,
        "kind": kind,
        "sample": "%d passes over %d x %s (%.0f MiB) copied from the GPU-resident batch; "
                  "Func::crc(%s, payload) vs stored crc, single thread, %.1f s" % (
                      passes, len(offs), what, float(np.sum(lens)) / 2**20, "0" if seed == 0 else hex(seed), dt),
        "allcore": allcore,
    }


def _dist_init():
    """One process per GPU (torch.distributed.run env).  Rendezvous, barrier and
    max-of-times only: the data path has no collective, so a CPU (gloo) group is
    enough and keeps torch's own HIP runtime out of the process (the product
    library brings /opt/rocm's).  TFS_BENCH_SHARE_DEVICE=1 maps every rank to
    device 0 (multi-rank rehearsal on a one-GPU box)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("TFS_BENCH_SHARE_DEVICE") == "1":
        local = 0
    dist = None
    if world > 1:
        import torch.distributed as dist
        _init_gloo(dist)
    _bind_numa(local)
    return world, rank, local, dist


_NUMA = {}


def _bind_numa(device):
    """Keep this rank's threads (and so its page-locked buffers, placed where they
    are first touched) on the NUMA node of its GPU (tfs_crc32_device_numa_node),
    as the device group's workers are: with 8 GPUs over two sockets, half the
    ranks would otherwise stage host data across the socket link."""
    import tfs_amd.crc as crc
    node = crc.lib().tfs_crc32_device_numa_node(device)
    _NUMA.update(node=node, bound=False)
    if node < 0:
        return
    try:
        with open("/sys/devices/system/node/node%d/cpulist" % node) as fh:
            cpus = set()
            for part in fh.read().strip().split(","):
                a, _, b = part.partition("-")
                cpus.update(range(int(a), int(b or a) + 1))
        mine = cpus & os.sched_getaffinity(0)
        if mine:
            os.sched_setaffinity(0, mine)
            _NUMA.update(bound=True, cpus=len(mine))
    except (OSError, ValueError):
        pass


def _gather_floats(dist, world, v):
    """[v of rank 0, v of rank 1, ...] (gloo all_gather; [v] without dist)."""
    if not dist:
        return [float(v)]
    import torch
    out = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(out, torch.tensor([float(v)], dtype=torch.float64))
    return [float(t.item()) for t in out]


def per_rank(dist, world, elapsed_s, nbytes, div=2**30):
    """Every rank's own rate over its own elapsed time (taken before the
    max-over-ranks), so an N > 1 line can say which rank -- which GPU and link --
    fell short: {values: [rank 0, rank 1, ...], elapsed_s, min, max, mean,
    slowest_rank, fastest_rank, min_over_max}.  div: 2**30 for GiB/s, 1e9 for GB/s."""
    els = _gather_floats(dist, world, elapsed_s)
    vals = [float(nbytes) / e / div if e > 0 else 0.0 for e in els]
    lo, hi = min(vals), max(vals)
    return {"values": vals, "elapsed_s": els, "min": lo, "max": hi, "mean": sum(vals) / len(vals),
            "slowest_rank": vals.index(lo), "fastest_rank": vals.index(hi),
            "min_over_max": lo / hi if hi > 0 else 0.0}


def _max_over_ranks(dist, v):
    if not dist:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


BLOCK_DATA = 64 * 1024 * 1024 - 512  # main block (config_item.h:132) minus BlockPrefix reserve (physical_block.h:31)


def zipf_sizes(seed, nblocks):
    """BASELINE configs[2] / SURVEY §8d: k ~ Zipf(s=1.1) truncated to 1..255,
    len = 4096*k + U[0,4095]; packed FileInfo|payload into 64 MiB blocks until full."""
    rng = np.random.default_rng(seed)
    k = np.arange(1, 256, dtype=np.float64)
    p = k ** -1.1
    p /= p.sum()
    blocks = []
    for _ in range(nblocks):
        lens = []
        used = 0
        while True:
            draw = (rng.choice(255, 64, p=p) + 1) * 4096 + rng.integers(0, 4096, 64)
            stop = False
            for L in draw:
                if used + 36 + int(L) > BLOCK_DATA:
                    stop = True
                    break
                lens.append(int(L))
                used += 36 + int(L)
            if stop:
                break
        blocks.append(np.array(lens, np.int64))
    return blocks


def _fragmented_flags(n):
    """Delete every even file, then every 3rd of the rest (test_logic_block_and_compact.cpp:946-975)."""
    flags = np.zeros(n, np.int32)
    flags[0::2] = 1
    rest = np.arange(1, n, 2)
    flags[rest[0::3]] = 1
    return flags


def live_bytes_total(windows, rec):
    return float(sum(w["n"] for w in windows)) * rec


def _ref_crc_fn():
    """Address of the reference's own Func::crc (oracle/_ref/libref_crc.so, built from
    src/common/func.{h,cpp}) or, without it, the oracle restatement's."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libref_crc.so")
    if os.path.exists(ref_so):
        L = ctypes.CDLL(ref_so)
        _ref_crc_fn.keep = L
        return ctypes.cast(L.ref_func_crc, ctypes.c_void_p).value, "reference"
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    _ref_crc_fn.keep = L
    return ctypes.cast(L.oracle_crc, ctypes.c_void_p).value, "port"


_PCIE = {}


def pcie_ceiling(ctx, nbytes=256 << 20, dist=None):
    """The link's measured DMA ceiling, this run: best of 5 pinned hipMemcpyAsync
    of 256 MiB host->device and device->host after 0.1 s of the same copies (the
    `peak` of the PCIe-bound lines),
    and the duplex rate: both directions at once on two streams (best of 3, the
    sum of the bytes moved over the longer of the two).  With N ranks (dist) each
    rank measures its own link in turn while the others wait at a barrier, so the
    peak is the per-GPU link's, not N links sharing the host at once."""
    if _PCIE:
        return _PCIE
    if dist is not None:
        world, rank = dist.get_world_size(), dist.get_rank()
        for r in range(world):
            dist.barrier()
            if r == rank:
                _pcie_measure(ctx, nbytes)
        dist.barrier()
        _PCIE["measured"] = "by each of the %d ranks in turn (the others waiting at a barrier)" % world
        _PCIE["source"] += "; per GPU link, " + _PCIE["measured"]
        return _PCIE
    _pcie_measure(ctx, nbytes)
    _PCIE["measured"] = "one rank"
    return _PCIE


def _pcie_measure(ctx, nbytes):
    import tfs_amd.crc as crc
    h = crc.PinnedBuffer(ctx, nbytes)
    h.array[:] = 1
    d = crc.DeviceBuffer(ctx, nbytes)
    out = {}
    for name, dst, src in (("h2d_GBs", d.ptr, h.ptr), ("d2h_GBs", h.ptr, d.ptr)):
        # ~0.1 s of the same copies first: the link's power management can hold it at a
        # lower speed after a pause (some boxes measured ~30 GB/s here, right after a leg
        # that had moved 50 GB/s), which would make `frac` exceed 1
        t_end = time.perf_counter() + 0.1
        while time.perf_counter() < t_end:
            ctx._check(ctx.L.tfs_crc32_memcpy(ctx.handle, dst, src, nbytes, None), "memcpy")
        best = 0.0
        for _ in range(5):
            t0 = time.perf_counter()
            ctx._check(ctx.L.tfs_crc32_memcpy(ctx.handle, dst, src, nbytes, None), "memcpy")
            best = max(best, nbytes / (time.perf_counter() - t0) / 1e9)
        out[name] = best
    h2 = crc.PinnedBuffer(ctx, nbytes)
    d2 = crc.DeviceBuffer(ctx, nbytes)
    s_up, s_down = ctx.stream_create(), ctx.stream_create()
    best = 0.0
    for _ in range(3):
        t0 = time.perf_counter()
        ctx._check(ctx.L.tfs_crc32_memcpy(ctx.handle, d.ptr, h.ptr, nbytes, s_up), "memcpy")
        ctx._check(ctx.L.tfs_crc32_memcpy(ctx.handle, h2.ptr, d2.ptr, nbytes, s_down), "memcpy")
        ctx.stream_sync(s_up)
        ctx.stream_sync(s_down)
        best = max(best, 2 * nbytes / (time.perf_counter() - t0) / 1e9)
    out["duplex_GBs"] = best
    ctx.stream_destroy(s_up)
    ctx.stream_destroy(s_down)
    for b in (h, d, h2, d2):
        b.free()
    out["source"] = "measured: best of 5 pinned 256 MiB hipMemcpy per direction after 0.1 s of the same copies, this run"
    out["duplex_source"] = ("measured: 256 MiB H2D and 256 MiB D2H issued together on two streams, "
                            "best of 3, 512 MiB over the wall time")
    _PCIE.update(out)


def _cpu_budget(shared=False):
    """Host CPUs this process may use: the scheduler affinity capped by the cgroup
    quota (cpu.max) -- on the GPU box 16 of the machine's 256 hardware threads.
    shared: a leg every local rank runs at the same time (the parity oracle) gets
    its share of the container-wide quota, quota / LOCAL_WORLD_SIZE, so N ranks
    never ask for N times the quota (cpu.max throttles the whole container)."""
    n = len(os.sched_getaffinity(0))
    quota_cpus = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            quota, period = fh.read().split()[:2]
        if quota != "max":
            quota_cpus = max(1, int(int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    if shared:
        local_world = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))))
        if quota_cpus is not None:
            quota_cpus = max(1, quota_cpus // local_world)
        else:
            n = max(1, min(n, (os.cpu_count() or n) // local_world))
    if quota_cpus is not None:
        n = min(n, quota_cpus)
    return n


def _allcore_threads(make_worker, seconds):
    """All-core CPU leg for the oracle routines that have no pthread driver: one
    Python thread per CPU this process may use, each calling `make_worker(i)()`
    (a ctypes call into the oracle, which releases the GIL) on its own output
    buffers until `seconds` have passed.  Returns (calls, elapsed s, threads)."""
    import threading
    threads = _cpu_budget()
    workers = [make_worker(i) for i in range(threads)]
    counts = [0] * threads
    stop = [False]

    def body(i):
        w = workers[i]
        while not stop[0]:
            w()
            counts[i] += 1

    ts = [threading.Thread(target=body, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    time.sleep(seconds)
    stop[0] = True
    for t in ts:
        t.join()
    return sum(counts), time.perf_counter() - t0, threads


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def e2e_blocks(ctx, dist, world, rank, nsub, inflight=3, cpu=None):
    """configs[4] end-to-end leg: pinned host block images -> (read over PCIe in place) verify ->
    verdicts back, `inflight` blocks in flight (submit/wait), timed between
    barriers, max over ranks.  Returns (payload GiB/s over all ranks, PCIe GB/s,
    elapsed s, per-rank {payload GiB/s, PCIe GB/s} (per_rank))."""
    import tfs_amd.crc as crc
    nfiles, rec = FILES_PER_BLOCK, FILEINFO + FILE_SIZE
    blk_bytes = nfiles * rec
    ndistinct = 8
    d_img = crc.DeviceBuffer(ctx, blk_bytes + 64)
    d_desc = crc.DeviceBuffer(ctx, 16 * nfiles)
    d_crc = crc.DeviceBuffer(ctx, 4 * nfiles)
    desc = np.zeros(nfiles, crc.DESC_DTYPE)
    desc["offset"] = np.arange(nfiles) * rec + FILEINFO
    desc["len"] = FILE_SIZE
    d_desc.upload(desc)
    srcs, exps = [], []
    for b in range(ndistinct):
        ctx.synth_fill_device(d_img, blk_bytes + 64 - (blk_bytes + 64) % 8, 0xE2E + b + 31 * rank, 0)
        ctx.batch_device(d_desc, nfiles, d_img, d_crc)
        ctx.sync()
        p = crc.PinnedBuffer(ctx, blk_bytes)
        p.array[:] = d_img.download(np.uint8, blk_bytes)
        srcs.append(p)
        exps.append(d_crc.download(np.uint32))
    offs = desc["offset"]
    lens = desc["len"]
    hs = []
    for _ in range(2):  # warmup: `inflight` submissions at once, so every slot the timed loop
        # uses has its stream and staging buffers before the clock starts
        ws = [ctx.submit_verify(srcs[i].array, offs, lens, exps[i]) for i in range(inflight)]
        for h in ws:
            ctx.wait(h)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    bad = 0
    for i in range(nsub):
        if len(hs) >= inflight:
            bad += ctx.wait(hs.pop(0))[2]
        hs.append(ctx.submit_verify(srcs[i % ndistinct].array, offs, lens, exps[i % ndistinct]))
    while hs:
        bad += ctx.wait(hs.pop(0))[2]
    el_local = time.perf_counter() - t0
    el = _max_over_ranks(dist, el_local)
    ranks = {"payload_GiBs": per_rank(dist, world, el_local, float(nsub) * nfiles * FILE_SIZE),
             "pcie_GBs": per_rank(dist, world, el_local, float(nsub) * blk_bytes, 1e9)}
    if bad:
        raise SystemExit("e2e: mismatches on clean data")
    if cpu is not None:
        cpu(srcs[0].array, offs, lens, exps[0])
    for b in srcs:
        b.free()
    for b in (d_img, d_desc, d_crc):
        b.free()
    payload = float(world) * nsub * nfiles * FILE_SIZE
    return payload / el / 2**30, float(world) * nsub * blk_bytes / el / 1e9, el, ranks


def _compact_allcore(ora, src_ptrs, mo, ms, flags, nfiles, dest_cap, expect_len, live_bytes, blk_bytes, seconds):
    """oracle_compact on every CPU this process may use: thread i compacts source
    image i % len(src_ptrs) into its own destination (reported, never fatal)."""
    try:
        def make(i):
            odest = np.zeros(dest_cap, np.uint8)
            doff = np.zeros(nfiles, np.int64)
            dsz = np.zeros(nfiles, np.int32)
            ook = np.zeros(nfiles, np.uint8)
            src = src_ptrs[i % len(src_ptrs)]

            def run():
                wc = ora.oracle_compact(src, mo.ctypes.data, ms.ctypes.data, flags.ctypes.data, nfiles,
                                        odest.ctypes.data, doff.ctypes.data, dsz.ctypes.data, ook.ctypes.data)
                if (expect_len is not None and wc != expect_len) or not ook[flags == 0].all():
                    raise SystemExit("compact: all-core oracle baseline disagrees")
            return run
        calls, dt, threads = _allcore_threads(make, seconds)
        return {"value": calls * live_bytes / dt / 2**30, "source_block_GiBs": calls * blk_bytes / dt / 2**30,
                "cores": threads, "nproc": os.cpu_count(), "cpu_model": _cpu_model(), "kind": "port",
                "cores_source": "sched affinity capped by the cgroup cpu.max quota",
                "sample": "%d compactions over %d threads, %.1f s" % (calls, threads, dt)}
    except Exception as e:  # reported, never fatal
        return {"error": str(e)}



def emit(rank, res):
    """Rank 0 prints the line: the one JSON line on stdout."""
    if rank == 0:
        print(json.dumps(res), flush=True)
