"""bench.py --workload zipf: BASELINE configs[2], CRC32 compute-on-write over
device-resident Zipf-sized files (Func::crc(0, payload) of every file,
src/common/func.cpp:426-435, at the close call site data_file.cpp:183-190)."""
import ctypes
import os
import time

import numpy as np

from benchlines.common import *  # noqa: F401,F403

ZIPF_PROFILE = "profiles/r06/pmc/zipf/pmc_summary.json"


def build(ctx, nblocks, seed):
    """The configs[2] image: zipf_sizes(seed, nblocks) packed FileInfo|payload
    from the start of each 64 MiB block (payloads at arbitrary byte offsets),
    filled with the splitmix64 stream.  Returns (img, offs, lens, total)."""
    import tfs_amd.crc as crc
    blocks = zipf_sizes(seed, nblocks)
    offs, lens = [], []
    for b, L in enumerate(blocks):
        rec = np.concatenate([[0], np.cumsum(36 + L)[:-1]])
        offs.append(b * (64 << 20) + rec + 36)
        lens.append(L)
    offs = np.concatenate(offs).astype(np.uint64)
    lens = np.concatenate(lens).astype(np.uint32)
    total = max(nblocks * (64 << 20), (int(offs[-1]) + int(lens[-1]) + 8191) // 4096 * 4096)
    img = crc.DeviceBuffer(ctx, total)
    ctx.synth_fill_device(img, total, 0xC0FFEE + seed, 0)
    return img, offs, lens, total


def parity_blocks(img, offs, lens, got, every):
    """Every `every`-th 64 MiB block of the image in full: all its files' CRCs
    recomputed by the oracle (pthreads, test infrastructure) over the device's
    bytes.  Returns (files checked, mismatches)."""
    import tfs_amd.crc as crc
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_crc_batch_mt.restype = ctypes.c_int
    ora.oracle_crc_batch_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int]
    blk = 64 << 20
    bidx = (offs // np.uint64(blk)).astype(np.int64)
    checked = mism = 0
    for b in range(0, int(bidx[-1]) + 1, max(1, every)):
        sel = np.nonzero(bidx == b)[0]
        if sel.size == 0:
            continue
        host = img.download(np.uint8, blk, b * blk)
        d = np.zeros(sel.size, crc.DESC_DTYPE)
        d["offset"], d["len"] = offs[sel] - np.uint64(b * blk), lens[sel]
        out = np.zeros(sel.size, np.uint32)
        if ora.oracle_crc_batch_mt(d.ctypes.data, sel.size, host.ctypes.data, out.ctypes.data,
                                   _cpu_budget(shared=True)) != 0:
            raise SystemExit("zipf: oracle failed")
        checked += int(sel.size)
        mism += int((out != got[sel]).sum())
    return checked, mism


def bench_zipf(args):
    """Compute-on-write over device-resident Zipf-sized files (checksum of every payload, seed 0)."""
    import tfs_amd.crc as crc
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    nblocks = args.blocks
    img, offs, lens, total = build(ctx, nblocks, 42 + rank)
    n = len(lens)
    desc = np.zeros(n, crc.DESC_DTYPE)
    desc["offset"], desc["len"] = offs, lens
    d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_out = crc.DeviceBuffer(ctx, 4 * n)
    for _ in range(args.warmup):
        ctx.batch_device(d_desc, n, img, d_out)
    ctx.sync()
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
    rank_kms = _gather_floats(dist, world, float(np.mean([a.elapsed_ms(b) for a, b in ev])))
    kms = max(rank_kms)
    # parity after timing (test infrastructure): every (parity_every / 4)-th block in full
    got = d_out.download(np.uint32)
    every = max(1, args.parity_every // 4)
    checked, mism = parity_blocks(img, offs, lens, got, every)
    if mism:
        raise SystemExit("zipf: GPU CRCs disagree with the oracle on %d of %d files" % (mism, checked))
    if dist:
        import torch
        t = torch.tensor([checked, mism], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        checked, mism = int(t[0]), int(t[1])
    payload = float(lens.astype(np.float64).sum())
    algo = payload + 21.0 * n
    z_traffic, z_src = _pmc_traffic(ZIPF_PROFILE, HEADLINE_KERNEL.replace("<1,", "<0,", 1), nblocks == 1024)
    res = {
        "metric": "GiB/s CRC32 compute-on-write, device-resident Zipf 4 KiB-1 MiB files",
        "value": world * args.steps * payload / el / 2**30, "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64), Zipf(1.1) k in 1..255, len = 4096k + U[0,4095], seed 42 + rank",
        "config": {"workload": "BASELINE configs[2]: %d blocks x 64 MiB, %d files, mean %.1f KiB" % (
            nblocks, n, payload / n / 1024), "files_per_gpu": n},
        "parity": {"files_checked": checked, "mismatches": mism,
                   "method": "every %d-th 64 MiB block of every rank in full: all its files' CRCs recomputed by "
                             "the oracle (pthreads) over the device's bytes" % every},
        "roofline": {"bound": "hbm", "achieved": algo / (kms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": algo / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, "traffic": z_traffic,
                     "traffic_source": z_src, "traffic_measured_in_this_run": False, "traffic_note": TRAFFIC_NOTE,
                     "algorithmic_bytes_per_launch": algo,
                     "kernel": "crc_files_kernel<0> (compute) + split plan/fold", "kernel_ms_avg": kms,
                     "kernel_ms_per_rank": {"ms": rank_kms, "min": min(rank_kms), "max": max(rank_kms)}},
    }
    if rank == 0 and not args.no_cpu:
        # the reference CRC on the host over a bounded sample of the same Zipf files
        idx = np.linspace(0, n - 1, min(n, 1024)).astype(np.int64)
        sl = lens[idx].astype(np.int64)
        so = np.concatenate([[0], np.cumsum(sl)[:-1]])
        sample = np.zeros(int(sl.sum()), np.uint8)
        for j, i in enumerate(idx):
            sample[so[j]:so[j] + sl[j]] = img.download(np.uint8, int(lens[i]), int(offs[i]))
        res["cpu_baseline"] = cpu_baseline(sample, so, sl, got[idx], args.cpu_seconds,
                                           "Zipf-sized payloads (evenly spaced files of the batch)")
    if dist and not args.no_cpu:
        dist.barrier()
    if args.e2e_blocks > 0:
        # north_star: the write path starts in host memory (the receive buffer), so
        # the PCIe-inclusive rate of the same Zipf files rides beside `value`
        from benchlines.zipf_e2e import zipf_e2e_leg
        res["end_to_end"] = zipf_e2e_leg(ctx, dist, world, rank, args.e2e_blocks)
    emit(rank, res)
    del ev
    for b in (img, d_desc, d_out):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()
