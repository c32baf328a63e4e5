#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: GiB/s CRC32 verify of device-resident 64 KiB files.

Workload (BASELINE.json configs[1]): per GPU, a resident set of 1,024 TFS blocks x
1,024 files x 64 KiB payload (1 M files, 64 GiB of payload), laid out as block
images: each file is a 36-byte FileInfo followed by its payload
(LogicBlock::close_write_file, logic_block.cpp:171-178,295-300), so payloads sit
at 65,572*k + 36 -- 4-byte aligned only, as on disk.  One step = one verify pass
over the whole resident set (recompute Func::crc(0, payload) and compare with
the stored crc_ carried in the descriptor).  16 steps = the 1 TiB of config 2.

Multi-GPU: one process per GPU, blocks partitioned by block id (each rank owns
its own 1,024 blocks); no collective on the data path (torch.distributed is
used only for the barrier and the max-over-ranks of the timing).  Weak scaling.

Timing: W warmup steps, then K steps bracketed by barrier + synchronize; HIP
events on the launch stream give the per-launch kernel time for the roofline.
cpu_baseline: the reference Func::crc text (oracle/_ref, kind "reference") or the
oracle restatement (kind "port"), single thread, on a bounded sample of the same
resident bytes, rank 0 at N=1 only.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FILE_SIZE = 65536
FILES_PER_BLOCK = 1024
FILEINFO = 36
HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md (8.0 TB/s)
ALGO_BYTES_PER_FILE = FILE_SIZE + 16 + 4 + 1  # payload + descriptor + crc out + verdict


def rank_blocks(total_blocks, world, rank):
    """Global block ids owned by `rank`: partition by block id (block_id % world == rank)."""
    return np.arange(rank, total_blocks, world, dtype=np.int64)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=16)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--blocks", type=int, default=1024, help="resident blocks per GPU (1024 = 1 M files)")
    p.add_argument("--compact-blocks", type=int, default=4096, help="blocks per GPU for --workload compact/e2e")
    p.add_argument("--file-blocks", type=int, default=32, help="blocks on disk per GPU for --workload compact_files")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--parity-every", type=int, default=64,
                   help="headline: every K-th resident block is checked in full against the oracle "
                        "(outside the timed region)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--e2e-blocks", type=int, default=128,
                   help="blocks per GPU for the end-to-end (H2D-inclusive) leg of the default line; 0 = off")
    p.add_argument("--e2e", action="store_true", help="also measure the pinned H2D-inclusive rate (stderr)")
    p.add_argument("--ec-mib", type=int, default=1536,
                   help="member size in MiB for --workload ec (< 2048: ErasureCode sizes are int)")
    p.add_argument("--membench", action="store_true", help="also time raw streaming reads (stderr)")
    p.add_argument("--workload", default="verify", choices=["verify", "zipf", "compact", "e2e", "packet", "compact_device", "ec", "loopback", "block_verify",
                            "block_verify_device", "compact_files", "mixed"],
                   help="verify = BASELINE configs[1] (the headline line); zipf = configs[2]; "
                        "compact = configs[3]; e2e = pinned-host verify incl. H2D (configs[4] end-to-end)")
    p.add_argument("--ab", default="", help="comma list of TFS_CRC_VARIANT ids: interleaved A/B timing (stderr)")
    p.add_argument("--ab-rounds", type=int, default=6)
    p.add_argument("--slots", default="", help="--workload compact: also time these blocks-in-flight counts (stderr A/B)")
    p.add_argument("--launch-check", action="store_true",
                   help="rank plumbing only: every rank reports (rank, world, device) and exits (CPU test of --gpus N)")
    return p.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`python3 bench.py --gpus N` with no launcher around it: start the N ranks
    (one process per GPU) through torch.distributed.run and relay rank 0's line.
    This parent never touches the GPU (no HIP call before the ranks exist: each
    rank binds its own device), so it can start them safely; it exits with the
    launcher's status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    print("bench.py: starting %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


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


def launch_check(args):
    """--launch-check: the rank plumbing of --gpus N without any GPU work."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        _init_gloo(dist)
        got = [None] * world
        dist.all_gather_object(got, [rank, local, os.getpid()])
        dist.destroy_process_group()
    else:
        got = [[rank, local, os.getpid()]]
    if rank == 0:
        print(json.dumps({"launch_check": {"world": world, "gpus": args.gpus, "ranks": got}}), flush=True)


TRAFFIC_NOTE = ("quoted: HBM bytes per launch from the committed rocprofv3 PMC passes of this same command at "
                "full size (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, tools/pmc_summary.py), not counted in this "
                "run; null when this run is not the profiled configuration")
# The product verify kernel as rocprofv3 names it (profiles/pmc_latest.json is of this kernel).
HEADLINE_KERNEL = "crc_files_kernel<1, 16, 5, true, true, true, 1, false, true, 1, false, false, 4, 3"
PACKET_PIPELINE = ("packet pipeline: packet_parse_kernel + crc_files_kernel<1, ..., 4, 3> + "
                   "packet_finish_kernel")


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


def main():
    args = parse()
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None and int(ws) != args.gpus:
        # One rank per GPU: a launcher that started another number of ranks than
        # --gpus asks for would report a line for the wrong N.
        raise SystemExit("bench.py: WORLD_SIZE=%s but --gpus %d; launch --gpus ranks (or run plain "
                         "`python3 bench.py --gpus N`, which starts them itself)" % (ws, args.gpus))
    if ws is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if args.launch_check:
        return launch_check(args)
    if args.workload != "verify":
        return {"zipf": bench_zipf, "compact": bench_compact, "e2e": bench_e2e,
                "packet": bench_packet, "compact_device": bench_compact_device, "ec": bench_ec,
                "loopback": bench_loopback, "block_verify": bench_block_verify,
                "block_verify_device": bench_block_verify_device,
                "compact_files": bench_compact_files, "mixed": bench_mixed}[args.workload](args)
    world, rank, local, dist = _dist_init()
    import tfs_amd.crc as crc
    from tfs_amd.synth import synth_bytes
    ctx = crc.Context(local)

    nblocks = args.blocks
    nfiles = nblocks * FILES_PER_BLOCK
    rec = FILEINFO + FILE_SIZE
    block_bytes = FILES_PER_BLOCK * rec
    total = nblocks * block_bytes
    total_al = (total + 4095) // 4096 * 4096
    data_seed = 0x9E3779B97F4A7C15
    # This rank's blocks: global block ids g = rank, rank+world, ... (partition by
    # block id).  Block g holds bytes [g*block_bytes, (g+1)*block_bytes) of one
    # global synthetic stream, so its content does not depend on the world size.
    gblocks = rank_blocks(nblocks * world, world, rank)
    img = crc.DeviceBuffer(ctx, total_al)
    for i, g in enumerate(gblocks):
        ctx.synth_fill_device(img.ptr + i * block_bytes, block_bytes, data_seed, int(g) * (block_bytes // 8))
    rec_off = np.arange(nfiles, dtype=np.uint64) * rec
    desc = np.zeros(nfiles, crc.DESC_DTYPE)
    desc["offset"] = rec_off + FILEINFO
    desc["len"] = FILE_SIZE
    d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_crc = crc.DeviceBuffer(ctx, 4 * nfiles)
    # write path: checksum-on-write of every payload, then persist FileInfo{crc_} headers
    ctx.batch_device(d_desc, nfiles, img, d_crc)
    d_off = crc.DeviceBuffer(ctx, 8 * nfiles).upload(rec_off)
    d_len = crc.DeviceBuffer(ctx, 4 * nfiles).upload(np.full(nfiles, FILE_SIZE, np.uint32))
    ctx.write_headers_device(img, d_off, d_len, d_crc, 1 + rank * nfiles, nfiles)  # file ids unique per rank
    ctx.sync()
    expected = d_crc.download(np.uint32)
    desc["aux"] = expected
    d_vdesc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_ok = crc.DeviceBuffer(ctx, nfiles)
    d_bad = crc.DeviceBuffer(ctx, 4)

    # Parity outside the timed region (test infrastructure): 48 files' bytes against
    # the host generator, and every K-th resident block in full -- all 1,024 CRCs
    # of the block recomputed by the oracle (multi-threaded) over the device's bytes.
    sample_idx = np.linspace(0, nfiles - 1, 48).astype(np.int64)
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_crc.restype = ctypes.c_uint32
    ora.oracle_crc.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int32]
    ora.oracle_crc_batch_mt.restype = ctypes.c_int
    ora.oracle_crc_batch_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int]
    for i in sample_idx:
        o = int(desc["offset"][i])
        host = img.download(np.uint8, FILE_SIZE, o).tobytes()
        g = int(gblocks[i // FILES_PER_BLOCK])
        assert host == synth_bytes(data_seed, FILE_SIZE, g * block_bytes + o % block_bytes).tobytes()
        if ora.oracle_crc(0, host, FILE_SIZE) != int(expected[i]):
            raise SystemExit("GPU CRC disagrees with oracle at file %d" % i)
    checked = mism = 0
    bd = np.zeros(FILES_PER_BLOCK, crc.DESC_DTYPE)
    bd["offset"] = np.arange(FILES_PER_BLOCK, dtype=np.uint64) * rec + FILEINFO
    bd["len"] = FILE_SIZE
    bout = np.zeros(FILES_PER_BLOCK, np.uint32)
    for b in range(0, nblocks, max(1, args.parity_every)):
        host = img.download(np.uint8, block_bytes, b * block_bytes)
        ora.oracle_crc_batch_mt(bd.ctypes.data, FILES_PER_BLOCK, host.ctypes.data, bout.ctypes.data,
                                _cpu_budget(shared=True))
        mism += int((bout != expected[b * FILES_PER_BLOCK:(b + 1) * FILES_PER_BLOCK]).sum())
        checked += FILES_PER_BLOCK
    if mism:
        raise SystemExit("GPU CRCs disagree with the oracle on %d of %d fully checked files" % (mism, checked))

    def step():
        ctx.verify_device(d_vdesc, nfiles, img, None, d_ok, d_bad)

    for _ in range(args.warmup):
        step()
    ctx.sync()
    d_bad.zero()
    ev = [(crc.Event(ctx), crc.Event(ctx)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record()
        step()
        ev[k][1].record()
    ctx.sync()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = [a.elapsed_ms(b) for a, b in ev]
    nbad = int(d_bad.download(np.uint32)[0])
    if nbad:
        raise SystemExit("verify reported %d mismatches on clean data" % nbad)
    # every file of the last pass has verdict 1 (a skipped file would keep its 0)
    d_ok.zero()
    ctx.sync()
    step()
    ctx.sync()
    all_ok = bool((d_ok.download(np.uint8, nfiles) == 1).all())
    if not all_ok:
        raise SystemExit("verify left files without a verdict")
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        t = torch.tensor([checked, mism, 0 if all_ok else 1], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        checked, mism, all_ok = int(t[0]), int(t[1]), int(t[2]) == 0
    # the partition by block id: rank r owns global blocks r, r+N, ...
    parts = [rank_blocks(nblocks * world, world, r) for r in range(world)]
    allb = np.concatenate(parts)
    partition = {"rule": "global block g -> rank g % N", "blocks_per_rank": [int(p.size) for p in parts],
                 "disjoint": bool(np.unique(allb).size == allb.size),
                 "covers": bool(np.array_equal(np.sort(allb), np.arange(nblocks * world)))}
    payload_bytes = float(world) * args.steps * nfiles * FILE_SIZE
    value = payload_bytes / elapsed / 2**30
    # Every rank's mean kernel time (HIP events on its own launch stream); the
    # roofline is priced at the slowest GPU's, with the spread beside it.
    rank_kms = _gather_floats(dist, world, float(np.mean(kern_ms)))
    avg_kern_s = max(rank_kms) / 1e3
    achieved = nfiles * ALGO_BYTES_PER_FILE / avg_kern_s / 1e9

    if args.ab:
        ab_compare(args, crc, img, d_vdesc, nfiles, d_ok, d_bad)
    if os.environ.get("TFS_BENCH_SPLIT_AB"):
        split_ab(ctx, crc, local, args, lambda c: c.verify_device(d_vdesc, nfiles, img, None, d_ok, d_bad),
                 nfiles * ALGO_BYTES_PER_FILE)

    extra = {}
    if args.membench:  # calibration kernels: measurement build (libtfs_crc_measure.so)
        out = crc.DeviceBuffer(ctx, 16)
        mctx = crc.Context(local, measure=True)
        mb = [(1000, 0), (1000, 1024), (16, 0), (1016, 0), (10016, 0), (11016, 0), (54004, 0), (54016, 0),
              (54064, 0), (55404, 0), (55804, 0), (55416, 0), (55404, 512), (55804, 512), (55816, 512), (55264, 0)]
        if os.environ.get("TFS_BENCH_MEMBENCH"):  # "pattern:grid,..." (measurement)
            mb = [tuple(int(x) for x in p.split(":")) for p in os.environ["TFS_BENCH_MEMBENCH"].split(",")]
        for pat, grid in mb:
            e0, e1 = crc.Event(mctx), crc.Event(mctx)
            mctx.membench_device(pat, img, d_vdesc, nfiles, total, out, grid=grid)
            e0.record()
            for _ in range(5):
                mctx.membench_device(pat, img, d_vdesc, nfiles, total, out, grid=grid)
            e1.record()
            ms = e0.elapsed_ms(e1) / 5
            run = pat % 1000
            if pat >= 54000:  # wave- / workgroup-contiguous chunks of (pat % 100) x 16 KiB over the whole image
                ch = (pat % 100) * 16384
                nb = total // ch * ch
            else:
                nb = total if run == 0 else nfiles * ((FILE_SIZE - 127) // (64 * run)) * 64 * run
            extra["membench_p%d_g%d_GBs" % (pat, grid)] = nb / (ms / 1e3) / 1e9
        mctx.close()
        print(json.dumps({"membench": extra}), file=sys.stderr)

    # HBM traffic per launch from the committed rocprofv3 PMC passes of this same
    # command (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; profiles/pmc_latest.json).
    hv_traffic, hv_src = _pmc_traffic("profiles/pmc_latest.json", HEADLINE_KERNEL, nfiles == 1048576)
    pmc = {"traffic_bytes_per_launch": hv_traffic, "source": hv_src} if hv_traffic else {}
    result = {
        "metric": "GiB/s CRC32 verify, device-resident 64 KiB files; 1/2/4/8 MI355X",
        "value": value,
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 payloads, FileInfo-headed block images, generated on device)",
        "config": {
            "workload": "device-resident CRC32 verify: %d blocks x %d files x 64 KiB per GPU (%d files, %.1f GiB "
                        "payload); %d steps = %.3g TiB per GPU (BASELINE configs[1]: 16 steps of 1024 blocks = 1 TiB)" % (
                            nblocks, FILES_PER_BLOCK, nfiles, nfiles * FILE_SIZE / 2**30,
                            args.steps, args.steps * nfiles * FILE_SIZE / 2**40),
            "files_per_gpu": nfiles,
            "file_size": FILE_SIZE,
            "layout": "block image, FileInfo(36 B)|payload, payload 4-byte aligned",
            "partition": "by block id across ranks, no collective",
            "partition_check": partition,
            "host_numa": dict(_NUMA),
        },
        "parity": {"files_checked": checked, "mismatches": mism, "verdicts_all_ok": all_ok,
                   "method": "every %d-th resident block of every rank: all 1,024 CRCs recomputed by the oracle "
                             "(pthreads) over the device's bytes; 48 files' bytes vs the host generator; every "
                             "verdict of a full pass is 1" % max(1, args.parity_every)},
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": pmc.get("traffic_bytes_per_launch"),
            "traffic_source": pmc.get("source"), "traffic_measured_in_this_run": False, "traffic_note": TRAFFIC_NOTE,
            "kernel": "crc_files_kernel<1> (verify)",
            "kernel_ms_avg": avg_kern_s * 1e3,
            "kernel_ms_per_rank": {"ms": rank_kms, "min": min(rank_kms), "max": max(rank_kms),
                                   "frac_at_min": nfiles * ALGO_BYTES_PER_FILE / (min(rank_kms) / 1e3) / 1e9
                                   / HBM_PEAK_GBS,
                                   "note": "mean kernel ms of each rank (HIP events on its stream); achieved and "
                                           "frac are priced at the slowest rank (max)"},
            "algorithmic_bytes_per_launch": nfiles * ALGO_BYTES_PER_FILE,
        },
    }
    # The reference CRC on the host cores, in the same run at every N: rank 0 times
    # it after the timed loops while the other ranks wait at a barrier (idle), so
    # its all-core leg has the box's CPU quota to itself.
    if rank == 0 and not args.no_cpu:
        ns = min(2048, nfiles)
        idx = np.linspace(0, nfiles - 1, ns).astype(np.int64)
        # copy the sampled payloads (identical bytes) to host
        sample = np.zeros(ns * FILE_SIZE, np.uint8)
        for j, i in enumerate(idx):
            o = int(desc["offset"][i])
            sample[j * FILE_SIZE:(j + 1) * FILE_SIZE] = img.download(np.uint8, FILE_SIZE, o)
        result["cpu_baseline"] = cpu_baseline(sample, np.arange(ns) * FILE_SIZE, np.full(ns, FILE_SIZE),
                                              expected[idx], args.cpu_seconds)
        result["cpu_baseline"]["run"] = ("rank 0 of %d, after the timed loops, the other ranks waiting at a barrier"
                                         % world)
    if dist and not args.no_cpu:
        dist.barrier()
    if args.e2e:
        print(json.dumps({"e2e": e2e_rate(ctx)}), file=sys.stderr)
    if args.e2e_blocks > 0:
        # configs[4] asks for device-resident AND end-to-end at every N: the same
        # job's PCIe-inclusive rate, reported beside `value` (never as `value`).
        gibs, pcie, el = e2e_blocks(ctx, dist, world, rank, args.e2e_blocks)
        ceil = pcie_ceiling(ctx, dist=dist)
        result["end_to_end"] = {
            "value": gibs, "unit": "GiB/s", "pcie_GBs": pcie, "ms_per_block": el / args.e2e_blocks * 1e3,
            "workload": "%d pinned host 64 MiB block images per GPU -> H2D -> verify -> verdicts back, "
                        "3 in flight, max over ranks" % args.e2e_blocks,
            "roofline": {"bound": "pcie", "achieved": pcie / world, "peak": ceil["h2d_GBs"], "unit": "GB/s (per GPU)",
                         "frac": pcie / world / ceil["h2d_GBs"], "peak_source": ceil["source"],
                         "traffic": "whole block images host->device (64 MiB + 36 B headers per 1,024 files)"}}
    if rank == 0:
        print(json.dumps(result), flush=True)
    del ev
    for b in (img, d_desc, d_crc, d_off, d_len, d_vdesc, d_ok, d_bad):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()


def ab_compare(args, crc, img, d_vdesc, nfiles, d_ok, d_bad, mode=1, algo_bytes=None, d_out=None):
    """Rule: perf deltas come from interleaved rounds in one process on one device."""
    algo_bytes = algo_bytes if algo_bytes is not None else nfiles * ALGO_BYTES_PER_FILE
    variants = list(dict.fromkeys(int(v) for v in args.ab.split(",") if v != ""))  # each id once, in order
    ctxs = {}
    for v in variants:
        os.environ["TFS_CRC_VARIANT"] = str(v)
        ctxs[v] = crc.Context(img.ctx.device)
    os.environ["TFS_CRC_VARIANT"] = "0"
    times = {v: [] for v in variants}
    for _ in range(args.ab_rounds):
        for v in variants:
            c = ctxs[v]
            e0, e1 = crc.Event(c), crc.Event(c)

            def run():
                if mode == 1:
                    c.verify_device(d_vdesc, nfiles, img, None, d_ok, d_bad)
                else:
                    c.batch_device(d_vdesc, nfiles, img, d_out)
            run()
            e0.record()
            for _ in range(3):
                run()
            e1.record()
            times[v].append(e0.elapsed_ms(e1) / 3)
    out = {}
    for v in variants:
        ms = sorted(times[v])
        out[v] = {"median_ms": ms[len(ms) // 2], "min_ms": ms[0],
                  "frac_at_median": algo_bytes / (ms[len(ms) // 2] / 1e3) / 1e9 / HBM_PEAK_GBS}
        ctxs[v].close()
    print(json.dumps({"ab": out}), file=sys.stderr)


def split_ab(ctx, crc, device, args, run, algo_bytes):
    """Measurement: the product with split files (tfs_crc32_set_split on, the
    default) against the same library with every file on one wave, interleaved
    rounds in one process (stderr)."""
    c2 = crc.Context(device)
    c2.set_split(False)
    times = {"split": [], "whole": []}
    for _ in range(max(1, args.ab_rounds)):
        for key, c in (("split", ctx), ("whole", c2)):
            run(c)
            e0, e1 = crc.Event(c), crc.Event(c)
            e0.record()
            for _ in range(3):
                run(c)
            e1.record()
            times[key].append(e0.elapsed_ms(e1) / 3)
    c2.close()
    out = {k: {"median_ms": sorted(v)[len(v) // 2], "min_ms": min(v),
               "frac_at_median": algo_bytes / (sorted(v)[len(v) // 2] / 1e3) / 1e9 / HBM_PEAK_GBS} for k, v in times.items()}
    print(json.dumps({"split_ab": out}), file=sys.stderr)


def e2e_rate(ctx):
    """Host block image (pinned) -> GPU verify -> verdicts back: the PCIe-inclusive rate."""
    import tfs_amd.crc as crc
    from tfs_amd.synth import synth_bytes
    nfiles = 4096
    rec = FILEINFO + FILE_SIZE
    host = crc.PinnedBuffer(ctx, nfiles * rec)
    host.array[:] = synth_bytes(5, nfiles * rec)
    offs = np.arange(nfiles) * rec + FILEINFO
    exp = ctx.batch(host.array, offs, [FILE_SIZE] * nfiles)
    reps = 4
    t0 = time.perf_counter()
    for _ in range(reps):
        c, ok, nbad, rc = ctx.verify(host.array, offs, [FILE_SIZE] * nfiles, exp)
        assert nbad == 0
    dt = time.perf_counter() - t0
    host.free()
    return {"GiBps_incl_pinned_h2d": reps * nfiles * FILE_SIZE / dt / 2**30, "files": nfiles}


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


def bench_zipf(args):
    """Compute-on-write over device-resident Zipf-sized files (checksum of every payload, seed 0)."""
    import tfs_amd.crc as crc
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    nblocks = args.blocks
    blocks = zipf_sizes(42 + rank, nblocks)
    # A/B knob (measurement only): TFS_BENCH_ZIPF_ALIGN=a places every payload
    # at an a-byte boundary and trims its length to a multiple of a.
    align = int(os.environ.get("TFS_BENCH_ZIPF_ALIGN", "0"))
    offs, lens = [], []
    for b, L in enumerate(blocks):
        if align:
            L = np.maximum(L // align * align, align)
            o, po = b * (64 << 20), []
            for x in L:
                o = (o + 36 + align - 1) // align * align
                po.append(o)
                o += int(x)
            offs.append(np.array(po, np.int64))
        else:
            rec = np.concatenate([[0], np.cumsum(36 + L)[:-1]])
            offs.append(b * (64 << 20) + rec + 36)
        lens.append(L)
    offs = np.concatenate(offs).astype(np.uint64)
    lens = np.concatenate(lens).astype(np.uint32)
    n = len(lens)
    total = max(nblocks * (64 << 20), (int(offs[-1]) + int(lens[-1]) + 8191) // 4096 * 4096)
    img = crc.DeviceBuffer(ctx, total)
    ctx.synth_fill_device(img, total, 0xC0FFEE + rank, 0)
    desc = np.zeros(n, crc.DESC_DTYPE)
    desc["offset"], desc["len"] = offs, lens
    d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_out = crc.DeviceBuffer(ctx, 4 * n)
    for _ in range(args.warmup):
        ctx.batch_device(d_desc, n, img, d_out)
    ctx.sync()
    # parity spot check (oracle, test infrastructure)
    got = d_out.download(np.uint32)
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_crc.restype = ctypes.c_uint32
    ora.oracle_crc.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int32]
    for i in np.linspace(0, n - 1, 32).astype(np.int64):
        h = img.download(np.uint8, int(lens[i]), int(offs[i])).tobytes()
        if ora.oracle_crc(0, h, len(h)) != int(got[i]):
            raise SystemExit("zipf: GPU CRC disagrees with oracle at file %d" % i)
    if args.ab:
        ab_compare(args, crc, img, d_desc, n, None, None, mode=0,
                   algo_bytes=float(lens.astype(np.float64).sum()) + 21.0 * n, d_out=d_out)
    ev = [(crc.Event(ctx), crc.Event(ctx)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record()
        ctx.batch_device(d_desc, n, img, d_out)
        ev[k][1].record()
    ctx.sync()
    if dist:
        dist.barrier()
    el = _max_over_ranks(dist, time.perf_counter() - t0)
    kms = float(np.mean([a.elapsed_ms(b) for a, b in ev]))
    payload = float(lens.astype(np.float64).sum())
    algo = payload + 21.0 * n
    z_traffic, z_src = _pmc_traffic("profiles/r03/zipf/pmc_summary.json", HEADLINE_KERNEL.replace("<1,", "<0,", 1),
                                    nblocks == 1024 and not align)
    res = {
        "metric": "GiB/s CRC32 compute-on-write, device-resident Zipf 4 KiB-1 MiB files",
        "value": world * args.steps * payload / el / 2**30, "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64), Zipf(1.1) k in 1..255, len = 4096k + U[0,4095], seed 42",
        "config": {"workload": "BASELINE configs[2]: %d blocks x 64 MiB, %d files, mean %.1f KiB" % (
            nblocks, n, payload / n / 1024), "files_per_gpu": n},
        "roofline": {"bound": "hbm", "achieved": algo / (kms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": algo / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, "traffic": z_traffic,
                     "traffic_source": z_src, "traffic_measured_in_this_run": False, "traffic_note": TRAFFIC_NOTE, "algorithmic_bytes_per_launch": algo,
                     "kernel": "crc_files_kernel<0> (compute)", "kernel_ms_avg": kms},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        # the reference CRC on the host over a bounded sample of the same Zipf files
        idx = np.linspace(0, n - 1, min(n, 1024)).astype(np.int64)
        sl = lens[idx].astype(np.int64)
        so = np.concatenate([[0], np.cumsum(sl)[:-1]])
        sample = np.zeros(int(sl.sum()), np.uint8)
        for j, i in enumerate(idx):
            sample[so[j]:so[j] + sl[j]] = img.download(np.uint8, int(lens[i]), int(offs[i]))
        res["cpu_baseline"] = cpu_baseline(sample, so, sl, got[idx], args.cpu_seconds,
                                           "Zipf-sized payloads (evenly spaced files of the batch)")
    if os.environ.get("TFS_BENCH_SPLIT_AB"):
        split_ab(ctx, crc, local, args, lambda c: c.batch_device(d_desc, n, img, d_out),
                 float(lens.astype(np.float64).sum()) + 21.0 * n)
    if os.environ.get("TFS_BENCH_SPLIT_PROBE"):
        # Measurement: would splitting large files into fixed segments (several
        # waves per file, their CRCs folded afterwards) read faster?  The same
        # payload bytes as descriptor lists where every file longer than T is cut
        # into a ragged first piece and S-byte segments; timed interleaved with
        # the unsplit list in this process (the fold is not timed: it is per file).
        def split_list(T, S):
            so, sl = [], []
            big = lens > T
            so.append(offs[~big]); sl.append(lens[~big])
            for o, L in zip(offs[big], lens[big]):
                L = int(L)
                first = L - (L - 1) // S * S
                so.append(np.array([int(o)] + [int(o) + first + S * j for j in range((L - first) // S)], np.uint64))
                sl.append(np.array([first] + [S] * ((L - first) // S), np.uint32))
            so, sl = np.concatenate(so), np.concatenate(sl)
            order = np.argsort(so, kind="stable")
            d = np.zeros(len(so), crc.DESC_DTYPE)
            d["offset"], d["len"] = so[order], sl[order]
            return d
        lists = {"unsplit": (d_desc, n)}
        spec = [tuple(int(x) for x in v.split(":")) for v in os.environ["TFS_BENCH_SPLIT_PROBE"].split(",")]
        bufs = []
        for T, S in spec:
            d = split_list(T, S)
            assert int(d["len"].astype(np.int64).sum()) == int(lens.astype(np.int64).sum())
            dd = crc.DeviceBuffer(ctx, d.nbytes).upload(d)
            bufs.append(dd)
            lists["T%d_S%d" % (T, S)] = (dd, len(d))
        dout = crc.DeviceBuffer(ctx, 4 * max(v[1] for v in lists.values()))
        times = {k: [] for k in lists}
        for _ in range(max(1, args.ab_rounds)):
            for k, (dd, nn) in lists.items():
                ctx.batch_device(dd, nn, img, dout)
                e0, e1 = crc.Event(ctx), crc.Event(ctx)
                e0.record()
                for _ in range(3):
                    ctx.batch_device(dd, nn, img, dout)
                e1.record()
                times[k].append(e0.elapsed_ms(e1) / 3)
        print(json.dumps({"split_probe": {k: {"units": lists[k][1], "median_ms": sorted(v)[len(v) // 2],
                                              "min_ms": min(v), "frac_at_median": algo / (sorted(v)[len(v) // 2] / 1e3)
                                              / 1e9 / HBM_PEAK_GBS} for k, v in times.items()}}), file=sys.stderr)
        for b in bufs + [dout]:
            b.free()
    if args.membench:
        # The kernel's access pattern over this geometry without the CRC arithmetic
        # (whole 1 KiB stripes of every file, 128-byte anchored, nt), and a plain
        # grid-stride stream of the same image: the ceilings the Zipf kernel is held to.
        mb = crc.DeviceBuffer(ctx, 16)
        mctx = crc.Context(local, measure=True)  # calibration kernels: measurement build
        stripes = np.maximum(lens.astype(np.int64) - 127, 0) // 1024
        for pat, nb in ((11016, float(stripes.sum()) * 1024.0), (1000, float(total))):
            mctx.membench_device(pat, img, d_desc, n, total, mb)
            e0, e1 = crc.Event(mctx), crc.Event(mctx)
            e0.record()
            for _ in range(5):
                mctx.membench_device(pat, img, d_desc, n, total, mb)
            e1.record()
            mctx.sync()
            res.setdefault("membench_GBs", {})["p%d" % pat] = nb / (e0.elapsed_ms(e1) / 5 / 1e3) / 1e9
        mctx.close()
        mb.free()
    if rank == 0:
        print(json.dumps(res), flush=True)
    del ev
    for b in (img, d_desc, d_out):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()


def bench_packet(args):
    """Receive-side packet CRC (BasePacket::decode, base_packet.cpp:117-148) over
    device-resident V1 frames carrying 64 KiB WriteDataMessages.
    Frames are sealed on the device first (the send side), then decoded K times."""
    import tfs_amd.crc as crc
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    # WriteDataMessage body: WriteDataInfo 32 B | vint64 ds_ (3 servers + lease triple: 4 + 6*8) | 64 KiB data
    body = 32 + 4 + 6 * 8 + FILE_SIZE
    frame = 24 + body
    n = args.blocks * FILES_PER_BLOCK
    total = n * frame
    img = crc.DeviceBuffer(ctx, (total + 4095) // 4096 * 4096)
    ctx.synth_fill_device(img, (total + 7) // 8 * 8, 0x5EED + rank, 0)
    off = np.arange(n, dtype=np.uint64) * frame
    blen = np.full(n, body, np.uint32)
    d_off = crc.DeviceBuffer(ctx, off.nbytes).upload(off)
    d_blen = crc.DeviceBuffer(ctx, blen.nbytes).upload(blen)
    ctx.write_packet_headers_device(img, d_off, d_blen, n, pcode=9, version=2, first_id=1 + rank * n)
    pd = np.zeros(n, crc.PACKET_DESC_DTYPE)
    pd["offset"], pd["len"] = off, frame
    d_pd = crc.DeviceBuffer(ctx, pd.nbytes).upload(pd)
    d_crc = crc.DeviceBuffer(ctx, 4 * n)
    d_st = crc.DeviceBuffer(ctx, 4 * n)
    d_bad = crc.DeviceBuffer(ctx, 4)
    ctx.packet_seal_device(d_pd, n, img, d_crc, d_st)  # send side: header crc_ = Func::crc(FLAG_V1, body)
    d_bad.zero()
    for _ in range(max(1, args.warmup)):
        ctx.packet_verify_device(d_pd, n, img, d_crc, d_st, d_bad)
    ctx.sync()
    if int(d_bad.download(np.uint32, 1)[0]) != 0:
        raise SystemExit("packet: sealed frames failed to verify")
    # parity spot check against the oracle (test infrastructure)
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_crc.restype = ctypes.c_uint32
    ora.oracle_crc.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int32]
    got = d_crc.download(np.uint32, n)
    for i in np.linspace(0, n - 1, 24).astype(np.int64):
        b = img.download(np.uint8, body, int(off[i]) + 24).tobytes()
        if ora.oracle_crc(0x4E534654, b, body) != int(got[i]):
            raise SystemExit("packet: GPU CRC disagrees with oracle at frame %d" % i)
    ev = [(crc.Event(ctx), crc.Event(ctx)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record()
        ctx.packet_verify_device(d_pd, n, img, d_crc, d_st, d_bad)
        ev[k][1].record()
    ctx.sync()
    if dist:
        dist.barrier()
    el = _max_over_ranks(dist, time.perf_counter() - t0)
    kms = float(np.mean([a.elapsed_ms(b) for a, b in ev]))
    # algorithmic bytes per frame over the decode pipeline: parse reads the 24-B header
    # and the 16-B frame descriptor and writes a 16-B body descriptor + 4-B pre-status;
    # the CRC kernel reads the body and its descriptor and writes crc + ok; finish
    # reads pre-status/ok and writes status (and crc).
    algo = n * (float(frame) + 16 + 16 + 4 + 16 + 4 + 1 + 4 + 4 + 1 + 4)
    p_traffic, p_src = _pmc_traffic("profiles/r02_s4/packet/pmc_summary.json", PACKET_PIPELINE, n == 1048576)
    res = {
        "metric": "GiB/s packet bytes CRC-verified (BasePacket::decode), device-resident V1 frames",
        "value": world * args.steps * n * frame / el / 2**30, "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64) WriteDataMessage bodies, headers sealed on the GPU",
        "config": {"workload": "SURVEY §8 f1: %d V1 frames x %d B (64 KiB write + message fields)" % (n, frame),
                   "frames_per_gpu": n},
        "roofline": {"bound": "hbm", "achieved": algo / (kms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": algo / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, "traffic": p_traffic,
                     "traffic_source": p_src, "traffic_measured_in_this_run": False, "traffic_note": TRAFFIC_NOTE, "algorithmic_bytes_per_launch": algo,
                     "kernel": "packet_parse + crc_files_kernel<1> + packet_finish", "kernel_ms_avg": kms},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        # BasePacket::decode's CRC on the host: Func::crc(TFS_PACKET_FLAG_V1, body) over sampled bodies
        idx = np.linspace(0, n - 1, min(n, 1024)).astype(np.int64)
        sample = np.zeros(len(idx) * body, np.uint8)
        for j, i in enumerate(idx):
            sample[j * body:(j + 1) * body] = img.download(np.uint8, body, int(off[i]) + 24)
        cb = cpu_baseline(sample, np.arange(len(idx)) * body, np.full(len(idx), body), got[idx],
                          args.cpu_seconds, "%d-B WriteDataMessage bodies" % body, seed=0x4E534654)
        cb["unit"] = "GiB/s of body bytes"
        res["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(res), flush=True)
    del ev
    for b in (img, d_off, d_blen, d_pd, d_crc, d_st, d_bad):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()


def _fragmented_flags(n):
    """Delete every even file, then every 3rd of the rest (test_logic_block_and_compact.cpp:946-975)."""
    flags = np.zeros(n, np.int32)
    flags[0::2] = 1
    rest = np.arange(1, n, 2)
    flags[rest[0::3]] = 1
    return flags


def bench_compact(args):
    """BASELINE configs[3]: host block images -> pinned H2D -> verify live files +
    repack on the GPU -> D2H of the new block, 4096 fragmented 64 MiB blocks."""
    import tfs_amd.crc as crc
    from tfs_amd.synth import synth_bytes  # noqa: F401
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    psize = int(os.environ.get("TFS_BENCH_PAYLOAD", FILE_SIZE))  # A/B knob: 65548 -> 16-byte multiple records
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
    # A/B: the whole-block DMA form (TFS_CRC_VARIANT=8: H2D of every source
    # block, kernel device to device, D2H of the new block) on the same jobs.
    os.environ["TFS_CRC_VARIANT"] = "8"
    ctx_dma = crc.Context(local)
    os.environ["TFS_CRC_VARIANT"] = "38"  # live records read in place, the new block back by DMA
    ctx_hyb = crc.Context(local)
    os.environ["TFS_CRC_VARIANT"] = "0"
    nab = min(nblocks, 512)
    ab_jobs = (crc.BlockJob * nab)(*jobs[:nab])
    for c in (ctx_dma, ctx_hyb):
        dests[0].array[:] = 0
        c.blocks_compact(warm)
        if not (dests[0].array[:w] == odest[:w]).all():
            raise SystemExit("compact: DMA / hybrid form disagrees with oracle")
    ab = {}
    for name, c in (("dma", ctx_dma), ("zero_copy", ctx), ("zc_read_dma_write", ctx_hyb)):
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        c.blocks_compact(ab_jobs)
        ab[name + "_ms_per_block"] = _max_over_ranks(dist, time.perf_counter() - t0) / nab * 1e3
    ctx_dma.close()
    ctx_hyb.close()
    for s in [int(x) for x in args.slots.split(",") if x]:  # blocks in flight (measurement knob)
        os.environ["TFS_CRC_COMPACT_SLOTS"] = str(s)
        cs = crc.Context(local)
        del os.environ["TFS_CRC_COMPACT_SLOTS"]
        cs.blocks_compact(warm)
        t0 = time.perf_counter()
        cs.blocks_compact(ab_jobs)
        ab["zero_copy_slots%d_ms_per_block" % s] = (time.perf_counter() - t0) / nab * 1e3
        cs.close()
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
        "ab": dict(ab, speedup=ab["dma_ms_per_block"] / ab["zero_copy_ms_per_block"], blocks=nab),
    }
    if rank == 0 and world == 1 and not args.no_cpu:
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
    if rank == 0:
        print(json.dumps(res), flush=True)
    for b in srcs + dests:
        b.free()
    for b in (d_img, d_desc, d_crc, d_off, d_len):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()


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
        if rank == 0 and world == 1 and not args.no_cpu:
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
        if rank == 0:
            print(json.dumps(res), flush=True)
    finally:
        if comp is not None:
            comp.free()
        shutil.rmtree(root, ignore_errors=True)
        ctx.close()
        if dist:
            dist.destroy_process_group()


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


def bench_block_verify(args):
    """Verify-on-read of fragmented blocks held in page-locked host memory (the
    block files of tfs_amd/ds/block_store.h load into such buffers): per block one
    tfs_block_verify over its live records (sync_backup.cpp:345-435 checks).
    The kernel reads only the named records over PCIe (zero-copy); the
    whole-block DMA form (TFS_CRC_VARIANT=8) is timed beside it."""
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
    os.environ["TFS_CRC_VARIANT"] = "8"
    ctx_dma = crc.Context(local)
    os.environ["TFS_CRC_VARIANT"] = "0"
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
    out = {}
    for name, c, nb in (("dma", ctx_dma, min(nblocks, 512)), ("zero_copy", ctx, nblocks)):
        c.block_verify(srcs[0].array, metas)
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        for j in range(nb):
            _, st, nbad, _ = c.block_verify(srcs[j % ndistinct].array, metas)
            if nbad:
                raise SystemExit("block_verify: mismatches on clean blocks")
        out[name] = (_max_over_ranks(dist, time.perf_counter() - t0), nb)
    ctx_dma.close()
    el, nb = out["zero_copy"]
    ceil = pcie_ceiling(ctx, dist=dist)
    pcie_gbs = float(nb) * live.size * rec / el / 1e9
    res = {
        "metric": "GiB/s of live payload verified on read from fragmented blocks in page-locked host memory",
        "value": float(world) * nb * live.size * FILE_SIZE / el / 2**30, "unit": "GiB/s of live payload",
        "source_block_GiBs": float(world) * nb * blk_bytes / el / 2**30, "n_gpus": world, "steps": nb,
        "warmup": 1, "ms_per_step": el / nb * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic 64 KiB files, 1024 per block, evens + every 3rd of the rest deleted (%d live)" % live.size,
        "config": {"workload": "one tfs_block_verify per block over its live records, %d blocks" % nb,
                   "live_payload_GiBs": float(world) * nb * live.size * FILE_SIZE / el / 2**30},
        "ab": {"zero_copy_ms_per_block": el / nb * 1e3, "dma_ms_per_block": out["dma"][0] / out["dma"][1] * 1e3},
        "roofline": {"bound": "pcie", "achieved": pcie_gbs, "peak": ceil["h2d_GBs"], "unit": "GB/s (per GPU)",
                     "frac": pcie_gbs / ceil["h2d_GBs"], "peak_source": ceil["source"],
                     "traffic": "the live records (FileInfo + payload) read in place over PCIe"},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        # the reference CRC over the live payloads of the same page-locked image, checked against the
        # FileInfo crc_ values the GPU verified (sync_backup.cpp:412-435's loop without the pread)
        cb = cpu_baseline(srcs[0].array, live * rec + FILEINFO, np.full(live.size, FILE_SIZE), c0,
                          args.cpu_seconds, "live 64 KiB payloads of a page-locked block image")
        cb["source_block_GiBs"] = cb["value"] * blk_bytes / (live.size * FILE_SIZE)
        cb["unit"] = "GiB/s of live payload"
        res["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(res), flush=True)
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
    # A/B in one process (measurement): round 1's static grid-stride block_verify_kernel
    # over 34 windows of 31 blocks (int32 RawMeta offsets), TFS_CRC_VARIANT=24.
    os.environ["TFS_CRC_VARIANT"] = "24"
    c24 = crc.Context(local)
    os.environ["TFS_CRC_VARIANT"] = "0"
    W = 31
    wins = []
    for w0 in range(0, nblocks, W):
        nb = min(W, nblocks - w0)
        m = np.zeros(nb * FILES_PER_BLOCK, crc.META_DTYPE)
        m["file_id"] = 1 + w0 * FILES_PER_BLOCK + np.arange(m.size)
        m["offset"] = np.arange(m.size) * rec
        m["size"] = rec
        wins.append((img.ptr + w0 * block_bytes, nb * block_bytes, crc.DeviceBuffer(c24, m.nbytes).upload(m), m.size))

    def step_windows(c):
        for base, ln, dm, nm in wins:
            c.block_verify_device(base, ln, dm, nm, None, d_st, d_bad)

    def timed(c, fn):
        e0, e1 = crc.Event(c), crc.Event(c)
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

    step_windows(c24)
    c24.sync()
    _, kms_old = timed(c24, step_windows)
    step_windows(ctx)
    ctx.sync()
    _, kms_win = timed(ctx, step_windows)
    el, kms = timed(ctx, step)
    for w in wins:
        w[2].free()
    c24.close()
    algo_per_rec = FILEINFO + FILE_SIZE + 40 + 4 + 4   # header + payload + job read, crc + status written
    achieved = nfiles * algo_per_rec / (kms / 1e3) / 1e9
    bv_traffic, bv_src = _pmc_traffic("profiles/r03/block_verify_device/pmc_summary.json",
                                      "compact_pipe_kernel<true, true, true, 12, 5, 4, 3", nblocks == 1024)
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
        "ab": {"pipelined_one_launch_ms": kms, "pipelined_31_block_windows_ms": kms_win,
               "round1_block_verify_kernel_windows_ms": kms_old, "speedup_vs_round1": kms_old / kms},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        # the reference's Func::crc over the payloads of resident block 0 copied to host,
        # against the stored crc_ (the loop of sync_backup.cpp:383-435 without the pread)
        host = img.download(np.uint8, block_bytes)
        cb = cpu_baseline(host, np.arange(FILES_PER_BLOCK) * rec + FILEINFO, np.full(FILES_PER_BLOCK, FILE_SIZE),
                          expected[:FILES_PER_BLOCK], args.cpu_seconds, "64 KiB payloads of resident block 0")
        res["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(res), flush=True)
    for b in (img, d_crc, d_jobs, d_out, d_st, d_bad):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()


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
    for rnd in range(max(1, args.ab_rounds)):
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
                               "threads through CloseBatcher" % (nblocks, jobs.size, max(1, args.ab_rounds)),
                   "value_mode": "closes (CU reserve on: the product)"},
        "modes": out,
        "roofline": {"bound": "hbm", "achieved": nfiles * ALGO_BYTES_PER_FILE / (out["closes"]["verify_ms_median"] / 1e3)
                     / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": nfiles * ALGO_BYTES_PER_FILE / (out["closes"]["verify_ms_median"] / 1e3) / 1e9 / HBM_PEAK_GBS,
                     "traffic": None, "kernel": "crc_files_kernel<1> (verify) beside crc_resident_kernel"},
        "parity": {"compaction_block0_vs_oracle": True, "verdicts_all_ok": True},
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    for b in (img, d_crc, d_vdesc, d_ok, d_bad, d_jobs, d_dst, d_st, d_bad2):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()


def live_bytes_total(windows, rec):
    return float(sum(w["n"] for w in windows)) * rec


def bench_compact_device(args):
    """the compaction data pass on device-resident blocks -- one
    fused kernel re-CRCs every live record and writes it to its new offset
    (one read + one write of live bytes).  Blocks are processed in windows of
    31 (RawMeta offsets are int32); TFS_CRC_VARIANT=7 (two passes: verify, then
    copy) is timed beside it for the A/B."""
    import tfs_amd.crc as crc
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    nfiles, rec = FILES_PER_BLOCK, FILEINFO + FILE_SIZE
    blk = nfiles * rec
    nblocks = args.blocks
    W = 31
    total = nblocks * blk
    img = crc.DeviceBuffer(ctx, (total + 4095) // 4096 * 4096)
    ctx.synth_fill_device(img, (total + 7) // 8 * 8, 0xC0DE + rank, 0)
    n = nblocks * nfiles
    desc = np.zeros(n, crc.DESC_DTYPE)
    rec_off = np.arange(n, dtype=np.uint64) * rec
    desc["offset"], desc["len"] = rec_off + FILEINFO, FILE_SIZE
    d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_crc = crc.DeviceBuffer(ctx, 4 * n)
    ctx.batch_device(d_desc, n, img, d_crc)
    d_roff = crc.DeviceBuffer(ctx, rec_off.nbytes).upload(rec_off)
    d_len = crc.DeviceBuffer(ctx, 4 * n).upload(np.full(n, FILE_SIZE, np.uint32))
    ctx.write_headers_device(img, d_roff, d_len, d_crc, 1, n)  # file id = 1 + global index
    ctx.sync()
    for b in (d_desc, d_roff, d_len):
        b.free()
    flags1 = _fragmented_flags(nfiles)
    live1 = np.nonzero(flags1 == 0)[0]
    windows = []
    for w0 in range(0, nblocks, W):
        nb = min(W, nblocks - w0)
        idx = (np.arange(nb)[:, None] * nfiles + live1[None, :]).reshape(-1)  # window-local file index
        m = np.zeros(idx.size, crc.META_DTYPE)
        m["file_id"] = 1 + w0 * nfiles + idx
        m["offset"] = idx * rec
        m["size"] = rec
        fl = np.zeros(idx.size, np.int32)
        dstride = rec if not os.environ.get("TFS_BENCH_PAD16") else (rec + 15) // 16 * 16  # A/B: 16-aligned dests
        do = np.arange(idx.size, dtype=np.int64) * dstride
        dst = crc.DeviceBuffer(ctx, idx.size * dstride + 64)
        windows.append(dict(base=img.ptr + w0 * blk, length=nb * blk, n=int(idx.size),
                            m=crc.DeviceBuffer(ctx, m.nbytes).upload(m), f=crc.DeviceBuffer(ctx, fl.nbytes).upload(fl),
                            o=crc.DeviceBuffer(ctx, do.nbytes).upload(do), dst=dst,
                            st=crc.DeviceBuffer(ctx, 4 * idx.size)))
    d_bad = crc.DeviceBuffer(ctx, 4)
    os.environ["TFS_CRC_VARIANT"] = "7"
    ctx2 = crc.Context(local)
    os.environ["TFS_CRC_VARIANT"] = "0"
    # The product form: every live record of every block in ONE launch
    # (tfs_compact_jobs_device); block b's live records are packed into its own
    # destination block at b * blk.
    nlive1 = live1.size
    jobs = np.zeros(nblocks * nlive1, crc.COMPACT_JOB_DTYPE)
    bidx = np.repeat(np.arange(nblocks, dtype=np.uint64), nlive1)
    loc = np.tile(np.arange(nlive1, dtype=np.uint64) * rec, nblocks)
    jobs["src_offset"] = bidx * blk + np.tile(live1.astype(np.uint64) * rec, nblocks)
    jobs["dest_offset"] = bidx * (nlive1 * rec) + loc
    jobs["file_id"] = 1 + bidx * nfiles + np.tile(live1.astype(np.uint64), nblocks)
    jobs["size"] = rec
    jobs["new_offset"] = loc.astype(np.int32)
    d_jobs = crc.DeviceBuffer(ctx, jobs.nbytes).upload(jobs)
    d_jdst = crc.DeviceBuffer(ctx, nblocks * nlive1 * rec + 64)
    d_jst = crc.DeviceBuffer(ctx, 4 * jobs.size)

    def step_jobs(c):
        c.compact_jobs_device(img, total, d_jobs, int(jobs.size), d_jdst, None, d_jst, d_bad)

    def step(c):
        for w in windows:
            c.block_compact_device(w["base"], w["length"], w["m"], w["f"], w["o"], w["n"], w["dst"], None, w["st"],
                                   d_bad)

    d_bad.zero()
    for _ in range(max(1, args.warmup)):
        step_jobs(ctx)
        step(ctx)
    ctx.sync()
    if int(d_bad.download(np.uint32, 1)[0]) != 0:
        raise SystemExit("compact_device: CRC mismatches on clean blocks")
    # parity: block 0 against the oracle's real_compact restatement
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_compact.restype = ctypes.c_int64
    ora.oracle_compact.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4
    host = img.download(np.uint8, blk)
    mo = (np.arange(nfiles) * rec).astype(np.int64)
    ms = np.full(nfiles, rec, np.int32)
    odest = np.zeros(blk, np.uint8)
    doff = np.zeros(nfiles, np.int64)
    dsz = np.zeros(nfiles, np.int32)
    ook = np.zeros(nfiles, np.uint8)
    wlen = ora.oracle_compact(host.ctypes.data, mo.ctypes.data, ms.ctypes.data, flags1.ctypes.data, nfiles,
                              odest.ctypes.data, doff.ctypes.data, dsz.ctypes.data, ook.ctypes.data)
    # the bench writes flag_ = 0 for every live file (flags1 is 0 on live files) -> identical bytes
    for got in (windows[0]["dst"].download(np.uint8, int(wlen)), d_jdst.download(np.uint8, int(wlen))):
        if not os.environ.get("TFS_BENCH_PAD16") and not (got == odest[:wlen]).all():
            raise SystemExit("compact_device: GPU repack disagrees with oracle")

    def timed(c, fn=step):
        ev0, ev1 = crc.Event(c), crc.Event(c)
        if dist:
            dist.barrier()
        c.sync()
        t0 = time.perf_counter()
        ev0.record()
        for _ in range(args.steps):
            fn(c)
        ev1.record()
        c.sync()
        if dist:
            dist.barrier()
        return _max_over_ranks(dist, time.perf_counter() - t0), ev0.elapsed_ms(ev1) / args.steps

    step(ctx2)
    ctx2.sync()
    extra = {}
    if args.membench:  # streaming-copy ceiling for the same number of live bytes
        nb = int(live_bytes_total(windows, rec)) // 16 * 16
        cdst = crc.DeviceBuffer(ctx, nb + 64)
        mctx = crc.Context(local, measure=True)  # calibration kernels: measurement build
        for pat in (50000, 51000, 52001, 52004, 52008, 52104, 52114, 52014, 52118, 52108):
            e0, e1 = crc.Event(mctx), crc.Event(mctx)
            mctx.membench_device(pat, img, None, 0, nb, cdst)
            e0.record()
            for _ in range(3):
                mctx.membench_device(pat, img, None, 0, nb, cdst)
            e1.record()
            mctx.sync()
            extra["copy_p%d_GBs_rw" % pat] = 2 * nb / (e0.elapsed_ms(e1) / 3 / 1e3) / 1e9
        mctx.close()
        cdst.free()
    el_w, kms_w = timed(ctx)
    el2, kms2 = timed(ctx2)
    os.environ["TFS_CRC_VARIANT"] = "22"   # A/B: the unpipelined fused kernel (round 1's product)
    ctx22 = crc.Context(local)
    os.environ["TFS_CRC_VARIANT"] = "0"
    step_jobs(ctx22)
    ctx22.sync()
    _, kms22 = timed(ctx22, step_jobs)
    ctx22.close()
    os.environ["TFS_CRC_VARIANT"] = "23"   # A/B: the pipelined kernel with ds_bpermute lane shifts
    ctx23 = crc.Context(local)
    os.environ["TFS_CRC_VARIANT"] = "0"
    step_jobs(ctx23)
    ctx23.sync()
    _, kms23 = timed(ctx23, step_jobs)
    ctx23.close()
    el, kms = timed(ctx, step_jobs)
    nlive = sum(w["n"] for w in windows)
    live_bytes = float(nlive) * rec
    algo = 2 * live_bytes + nlive * (40 + 4)  # read + write live records, 40 B CompactJob + 4 B status
    live_payload = float(nlive) * FILE_SIZE
    cd_traffic, cd_src = _pmc_traffic("profiles/r03/compact_device/pmc_summary.json",
                                      "compact_pipe_kernel<true, true, false, 12, 5, 1, 0", nblocks == 1024)
    res = {
        "metric": "GiB/s of live payload compacted on the device (re-CRC + repack of live files)",
        "value": world * args.steps * live_payload / el / 2**30, "unit": "GiB/s of live payload", "n_gpus": world,
        "source_block_GiBs": world * args.steps * float(total) / el / 2**30,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic 64 KiB files, 1024 per block, evens + every 3rd of the rest deleted",
        "config": {"workload": "SURVEY §8 f3: %d resident blocks, %d live files (%.1f GiB live)" % (
            nblocks, nlive, live_bytes / 2**30)},
        "roofline": {"bound": "hbm", "achieved": algo / (kms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": algo / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, "traffic": cd_traffic, "traffic_source": cd_src, "traffic_measured_in_this_run": False, "traffic_note": TRAFFIC_NOTE,
                     "kernel": "compact_pipe_kernel<WIDE> (one launch)", "kernel_ms_avg": kms,
                     "algorithmic_bytes_per_launch": algo},
        "membench": extra,
        "ab": {"fused_one_launch_ms": kms, "fused_windows_ms": kms_w, "unfused_windows_ms": kms2,
               "unpipelined_fused_one_launch_ms": kms22, "pipelined_bpermute_one_launch_ms": kms23,
               "windows": len(windows), "speedup_vs_unfused": kms2 / kms,
               "speedup_vs_unpipelined": kms22 / kms},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        # CPU restatement of real_compact + re-CRC (oracle_compact) over block 0 of the same image, one thread
        ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
        ora.oracle_compact.restype = ctypes.c_int64
        ora.oracle_compact.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4
        src = img.download(np.uint8, blk)
        mo = np.arange(nfiles, dtype=np.int64) * rec
        ms = np.full(nfiles, rec, np.int32)
        odest = np.zeros(blk, np.uint8)
        doff = np.zeros(nfiles, np.int64)
        dsz = np.zeros(nfiles, np.int32)
        ook = np.zeros(nfiles, np.uint8)
        reps, t0 = 0, time.perf_counter()
        while True:
            ora.oracle_compact(src.ctypes.data, mo.ctypes.data, ms.ctypes.data, flags1.ctypes.data, nfiles,
                               odest.ctypes.data, doff.ctypes.data, dsz.ctypes.data, ook.ctypes.data)
            reps += 1
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        dt = time.perf_counter() - t0
        if not (ook[flags1 == 0] == 1).all():
            raise SystemExit("compact_device: oracle re-CRC disagrees with the GPU-written headers")
        res["cpu_baseline"] = {
            "value": reps * len(live1) * FILE_SIZE / dt / 2**30, "unit": "GiB/s of live payload", "cores": 1,
            "kind": "port", "source_block_GiBs": reps * blk / dt / 2**30,
            "sample": "%d compactions of resident block 0 copied to host (re-CRC of %d live files + repack), "
                      "oracle_compact single thread, %.1f s" % (reps, len(live1), dt),
            "allcore": _compact_allcore(ora, [src.ctypes.data], mo, ms, flags1, nfiles, blk, None,
                                        len(live1) * FILE_SIZE, blk, min(3.0, args.cpu_seconds))}
    if rank == 0:
        print(json.dumps(res), flush=True)
    for w in windows:
        for k in ("m", "f", "o", "dst", "st"):
            w[k].free()
    for b in (img, d_crc, d_bad, d_jobs, d_jdst, d_jst):
        b.free()
    ctx2.close()
    ctx.close()
    if dist:
        dist.destroy_process_group()


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
    if args.ab:  # interleaved rounds of kernel forms (TFS_EC_VARIANT ids) in this process (stderr)
        forms = list(dict.fromkeys(int(v) for v in args.ab.split(",") if v != ""))
        encs = {}
        for v in forms:
            os.environ["TFS_EC_VARIANT"] = str(v)
            encs[v] = ErasureCode(ctx, k, m)
        os.environ["TFS_EC_VARIANT"] = "0"
        times = {v: [] for v in forms}
        for _ in range(args.ab_rounds):
            for v in forms:
                encs[v].encode_device(d, size)
                e0, e1 = crc.Event(ctx), crc.Event(ctx)
                e0.record()
                for _ in range(3):
                    encs[v].encode_device(d, size)
                e1.record()
                ctx.sync()
                times[v].append(e0.elapsed_ms(e1) / 3)
        ab = {}
        for v in forms:
            t = sorted(times[v])
            ab[v] = {"median_ms": t[len(t) // 2], "min_ms": t[0],
                     "frac_at_median": (k + m) * size / (t[len(t) // 2] / 1e3) / 1e9 / HBM_PEAK_GBS}
        print(json.dumps({"ab": ab}), file=sys.stderr)
    e_traffic, e_src = _pmc_traffic("profiles/r02_s4/ec/pmc_summary.json", "ec_apply_kernel<3>", args.ec_mib == 1536)
    res = {
        "metric": "GiB/s of data encoded (ErasureCode k=5 m=3, Cauchy bitmatrix w=8 ps=128), device-resident",
        "value": out["encode"]["GiBs_data"], "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": out["encode"]["ms"], "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (splitmix64) members",
        "config": {"workload": "SURVEY §8 f4: k=5 + m=3 members of %d MiB" % args.ec_mib},
        "roofline": {"bound": "hbm", "achieved": out["encode"]["hbm_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": out["encode"]["hbm_GBs"] / HBM_PEAK_GBS, "traffic": e_traffic, "traffic_source": e_src, "traffic_measured_in_this_run": False, "traffic_note": TRAFFIC_NOTE,
                     "algorithmic_bytes_per_launch": float(k + m) * size,
                     "kernel": "ec_apply_kernel<3>", "kernel_ms_avg": out["encode"]["ms"]},
        "decode": out["decode"],
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = ec_cpu_baseline(d, k, m, args.cpu_seconds, min(4 << 20, size // 1024 * 1024))
    if rank == 0:
        print(json.dumps(res), flush=True)
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
    for nl, it in ((1, 300), (8, 64), (64, 8)):
        cl = ds.close_latency(ctx, nl, it)
        lat["close_%d_leases" % nl] = {"p50_us": float(np.percentile(cl, 50)), "p99_us": float(np.percentile(cl, 99)),
                                       "closes": int(cl.size)}
    res["latency"] = lat
    # resident kernel over this whole line: launches (first + relaunches after
    # idle or lifetime exits) against the files it took
    launches, rfiles = ctx.resident_stats()
    res["resident_kernel"] = {"launches": int(launches), "files": int(rfiles)}
    # PCIe bytes of one loopback: every payload crosses once for the close check
    # (zero-copy reads of the lease buffers) and once for the whole-block verify.
    pcie_bytes = 2.0 * n * L
    ceil = pcie_ceiling(ctx, dist=dist)
    res["roofline"] = {"bound": "pcie", "achieved": reps * pcie_bytes / el / 1e9, "peak": ceil["h2d_GBs"],
                       "unit": "GB/s (per GPU)", "frac": reps * pcie_bytes / el / 1e9 / ceil["h2d_GBs"],
                       "traffic": None, "peak_source": ceil["source"],
                       "kernel": "crc_resident_kernel (close batches, no launch per batch) + compact_pipe_kernel verify form (whole block, zero-copy)",
                       "note": "latency-bound: one GPU round trip per batch of concurrent closes"}
    if rank == 0 and world == 1 and not args.no_cpu:
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
    if rank == 0:
        print(json.dumps(res), flush=True)
    for b in batchers.values():
        b.free()
    pool.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()


def e2e_blocks(ctx, dist, world, rank, nsub, inflight=3, cpu=None):
    """configs[4] end-to-end leg: pinned host block images -> H2D -> verify ->
    verdicts back, `inflight` blocks in flight (submit/wait), timed between
    barriers, max over ranks.  Returns (payload GiB/s over all ranks, PCIe GB/s,
    elapsed s)."""
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
    el = _max_over_ranks(dist, time.perf_counter() - t0)
    if bad:
        raise SystemExit("e2e: mismatches on clean data")
    if cpu is not None:
        cpu(srcs[0].array, offs, lens, exps[0])
    for b in srcs:
        b.free()
    for b in (d_img, d_desc, d_crc):
        b.free()
    payload = float(world) * nsub * nfiles * FILE_SIZE
    return payload / el / 2**30, float(world) * nsub * blk_bytes / el / 1e9, el


def bench_e2e(args):
    """Verify-on-read starting in host memory: pinned block images -> H2D ->
    verify -> verdicts back, several blocks in flight (submit/wait)."""
    import tfs_amd.crc as crc
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    nsub, inflight = args.compact_blocks, 3
    cpu_res = {}

    def cpu(arr, offs, lens, exp):
        # the same verify of one page-locked block image on the host CPU
        cpu_res["v"] = cpu_baseline(arr, offs, lens, exp, args.cpu_seconds,
                                    "64 KiB payloads of a page-locked block image")
    gibs, pcie, el = e2e_blocks(ctx, dist, world, rank, nsub, inflight,
                                cpu if rank == 0 and world == 1 and not args.no_cpu else None)
    res = {
        "metric": "GiB/s CRC32 verify end-to-end from pinned host block images (H2D included)",
        "value": gibs, "unit": "GiB/s", "n_gpus": world, "steps": nsub, "warmup": 2,
        "ms_per_step": el / nsub * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic 64 KiB files, 1024 per 64 MiB block",
        "config": {"workload": "pinned host blocks -> GPU verify, %d in flight, %d blocks" % (inflight, nsub)},
        "pcie_GBs": pcie,
    }
    ceil = pcie_ceiling(ctx, dist=dist)
    res["roofline"] = {"bound": "pcie", "achieved": pcie / world, "peak": ceil["h2d_GBs"], "unit": "GB/s (per GPU)",
                       "frac": pcie / world / ceil["h2d_GBs"], "peak_source": ceil["source"], "traffic": None}
    if "v" in cpu_res:
        res["cpu_baseline"] = cpu_res["v"]
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
