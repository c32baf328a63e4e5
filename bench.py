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
used only for the barrier, the max-over-ranks of the timing and the gather of
per-rank kernel times).  Weak scaling.

Timing: W warmup steps, then K steps bracketed by barrier + synchronize; HIP
events on the launch stream give the per-launch kernel time for the roofline
(priced at the slowest rank).  cpu_baseline: the reference Func::crc text
(oracle/_ref, kind "reference") or the oracle restatement (kind "port"), one
thread and all cores, on a bounded sample of the same resident bytes, timed by
rank 0 after the timed loops at every N while the other ranks wait.

The other BASELINE configs and SURVEY §8 rows are `--workload` lines in
benchlines/ (one module each); the A/B and ceiling probes of DESIGN.md §4 live
in tools/, not here.
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

from benchlines.common import *  # noqa: E402,F401,F403

WORKLOADS = {
    "zipf": ("benchlines.zipf", "bench_zipf"),                      # BASELINE configs[2]
    "zipf_e2e": ("benchlines.zipf_e2e", "bench_zipf_e2e"),          # configs[2] from host receive buffers
    "compact": ("benchlines.compact", "bench_compact"),             # configs[3]
    "e2e": ("benchlines.e2e", "bench_e2e"),                         # configs[4] end-to-end
    "loopback": ("benchlines.loopback", "bench_loopback"),          # configs[0]
    "packet": ("benchlines.packet", "bench_packet"),
    "compact_device": ("benchlines.compact_device", "bench_compact_device"),  # f3
    "ec": ("benchlines.ec", "bench_ec"),                            # f4
    "block_verify": ("benchlines.block_verify", "bench_block_verify"),        # a9/a10
    "block_verify_device": ("benchlines.block_verify", "bench_block_verify_device"),
    "compact_files": ("benchlines.compact_files", "bench_compact_files"),     # a11 + f2
    "mixed": ("benchlines.mixed", "bench_mixed"),                   # closes beside throughput launches
    "small_bodies": ("benchlines.small_bodies", "bench_small_bodies"),  # latency of lone RPC bodies
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=16)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--blocks", type=int, default=1024, help="resident blocks per GPU (1024 = 1 M files)")
    p.add_argument("--compact-blocks", type=int, default=4096, help="blocks per GPU for --workload compact/e2e")
    p.add_argument("--file-blocks", type=int, default=32, help="blocks on disk per GPU for --workload compact_files")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--parity-every", type=int, default=64,
                   help="every K-th resident block is checked in full against the oracle (outside the timed region)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--e2e-blocks", type=int, default=128,
                   help="blocks (receive buffers for zipf/zipf_e2e) per GPU for the end-to-end (H2D-inclusive) leg "
                        "of the default and zipf lines; 0 = off")
    p.add_argument("--verify-threads", type=int, default=3,
                   help="--workload block_verify: caller threads (the mirror / repair / checker call sites)")
    p.add_argument("--ec-mib", type=int, default=1536,
                   help="member size in MiB for --workload ec (< 2048: ErasureCode sizes are int)")
    p.add_argument("--workload", default="verify", choices=["verify"] + sorted(WORKLOADS),
                   help="verify = BASELINE configs[1] (the headline line); zipf = configs[2]; "
                        "compact = configs[3]; e2e = pinned-host verify incl. H2D (configs[4] end-to-end)")
    p.add_argument("--rounds", type=int, default=6, help="--workload mixed: interleaved rounds per mode")
    p.add_argument("--launch-check", action="store_true",
                   help="rank plumbing only: every rank reports (rank, world, device) and exits (CPU test of --gpus N)")
    return p.parse_args(argv)

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


def build_headline(ctx, nblocks, gblocks, rank):
    """The configs[1] resident set: block images of 1,024 FileInfo|64 KiB records
    (global block g holds bytes [g*block_bytes, (g+1)*block_bytes) of one global
    synthetic stream, so its content does not depend on the world size), every
    payload checksummed on write and its FileInfo{crc_} persisted.  Returns
    (img, desc with the expected CRCs in aux, expected, total bytes)."""
    import tfs_amd.crc as crc
    nfiles = nblocks * FILES_PER_BLOCK
    rec = FILEINFO + FILE_SIZE
    block_bytes = FILES_PER_BLOCK * rec
    total = nblocks * block_bytes
    img = crc.DeviceBuffer(ctx, (total + 4095) // 4096 * 4096)
    for i, g in enumerate(gblocks):
        ctx.synth_fill_device(img.ptr + i * block_bytes, block_bytes, DATA_SEED, int(g) * (block_bytes // 8))
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
    for b in (d_desc, d_crc, d_off, d_len):
        b.free()
    return img, desc, expected, total


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
        import importlib
        mod, fn = WORKLOADS[args.workload]
        return getattr(importlib.import_module(mod), fn)(args)
    world, rank, local, dist = _dist_init()
    import tfs_amd.crc as crc
    from tfs_amd.synth import synth_bytes
    ctx = crc.Context(local)

    nblocks = args.blocks
    nfiles = nblocks * FILES_PER_BLOCK
    rec = FILEINFO + FILE_SIZE
    block_bytes = FILES_PER_BLOCK * rec
    # This rank's blocks: global block ids g = rank, rank+world, ... (partition by block id).
    gblocks = rank_blocks(nblocks * world, world, rank)
    img, desc, expected, total = build_headline(ctx, nblocks, gblocks, rank)
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
        assert host == synth_bytes(DATA_SEED, FILE_SIZE, g * block_bytes + o % block_bytes).tobytes()
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
    elapsed_local = elapsed
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
    # Each rank's own device-resident rate (its own wall time between the barriers,
    # before the max) and where it runs, so a curve below linear names its rank.
    rank_dev = per_rank(dist, world, elapsed_local, float(args.steps) * nfiles * FILE_SIZE)
    rank_where = {"local_rank": [int(x) for x in _gather_floats(dist, world, int(os.environ.get("LOCAL_RANK", 0)))],
                  "device": [int(x) for x in _gather_floats(dist, world, local)],
                  "numa_node": [int(x) for x in _gather_floats(dist, world, _NUMA.get("node", -1))]}
    avg_kern_s = max(rank_kms) / 1e3
    achieved = nfiles * ALGO_BYTES_PER_FILE / avg_kern_s / 1e9

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
        "per_rank": dict(rank_where, device_GiBs=rank_dev),
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
    if args.e2e_blocks > 0:
        # configs[4] asks for device-resident AND end-to-end at every N: the same
        # job's PCIe-inclusive rate, reported beside `value` (never as `value`).
        gibs, pcie, el, e2e_ranks = e2e_blocks(ctx, dist, world, rank, args.e2e_blocks)
        ceil = pcie_ceiling(ctx, dist=dist)
        result["end_to_end"] = {
            "value": gibs, "unit": "GiB/s", "pcie_GBs": pcie, "ms_per_block": el / args.e2e_blocks * 1e3,
            "workload": "%d pinned host 64 MiB block images per GPU, verified by the GPU reading each image "
                        "over PCIe in place (zero-copy; verdicts back in page-locked words), 3 in flight, max "
                        "over ranks" % args.e2e_blocks,
            "per_rank": e2e_ranks,
            "roofline": {"bound": "pcie", "achieved": pcie / world, "peak": ceil["h2d_GBs"], "unit": "GB/s (per GPU)",
                         "frac": pcie / world / ceil["h2d_GBs"], "peak_source": ceil["source"],
                         "traffic": "whole block images host->device (64 MiB + 36 B headers per 1,024 files)"}}
    emit(rank, result)
    del ev
    for b in (img, d_vdesc, d_ok, d_bad):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
