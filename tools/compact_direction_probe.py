#!/usr/bin/env python3
"""Which PCIe direction limits host compaction (BASELINE configs[3], VERDICT r4
item 2)?  Measurement only.

The product kernel (tfs_compact_jobs_device, one launch over NB fragmented
blocks: 341 of every 1,024 64 KiB records live, the bench's layout) runs with the
same jobs and only the placement of its source images and its destination
changed:

  zc_both    source page-locked, destination page-locked (the product's zero-copy
             form: live records read over PCIe, the new block written back over it)
  zc_read    source page-locked, destination in HBM (only the reads cross PCIe)
  zc_write   source in HBM, destination page-locked (only the writes cross PCIe)
  hbm        both in HBM (the kernel's own time for the same records)
  verify_zc  tfs_blocks_verify_device over the same records, source page-locked
             (reads only, no stores at all)

beside the measured DMA ceilings (H2D, D2H, both at once) and the product host
line itself (tfs_blocks_compact over the same NB blocks, 8 in flight).  Each
case: HIP events around REPS launches, ROUNDS interleaved rounds, medians.

  python tools/compact_direction_probe.py [NB] [ROUNDS]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import tfs_amd.crc as crc  # noqa: E402
from benchlines.common import pcie_ceiling  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    reps = 3
    ctx = crc.Context(0)
    nfiles, rec = bench.FILES_PER_BLOCK, bench.FILEINFO + bench.FILE_SIZE
    blk = nfiles * rec
    ndist = 8
    # 8 distinct checksummed block images, device and page-locked copies
    d_src = crc.DeviceBuffer(ctx, ndist * blk + 256)
    ctx.synth_fill_device(d_src, (ndist * blk + 256) // 8 * 8, 0xD1CE, 0)
    n_all = ndist * nfiles
    roff = np.arange(n_all, dtype=np.uint64) * rec
    desc = np.zeros(n_all, crc.DESC_DTYPE)
    desc["offset"], desc["len"] = roff + bench.FILEINFO, bench.FILE_SIZE
    d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_crc = crc.DeviceBuffer(ctx, 4 * n_all)
    ctx.batch_device(d_desc, n_all, d_src, d_crc)
    d_roff = crc.DeviceBuffer(ctx, roff.nbytes).upload(roff)
    d_len = crc.DeviceBuffer(ctx, 4 * n_all).upload(np.full(n_all, bench.FILE_SIZE, np.uint32))
    ctx.write_headers_device(d_src, d_roff, d_len, d_crc, 1, n_all)
    ctx.sync()
    h_src = crc.PinnedBuffer(ctx, ndist * blk + 256)
    h_src.array[:] = d_src.download(np.uint8, ndist * blk + 256)
    live1 = np.nonzero(bench._fragmented_flags(nfiles) == 0)[0].astype(np.uint64)
    nl = live1.size
    # jobs: block b of the launch reads distinct image b % 8 and writes its new block at b * nl * rec
    b = np.repeat(np.arange(nb, dtype=np.uint64), nl)
    j = np.zeros(nb * nl, crc.COMPACT_JOB_DTYPE)
    j["src_offset"] = (b % np.uint64(ndist)) * np.uint64(blk) + np.tile(live1 * np.uint64(rec), nb)
    j["dest_offset"] = np.arange(nb * nl, dtype=np.uint64) * np.uint64(rec)
    j["file_id"] = 1 + (b % np.uint64(ndist)) * np.uint64(nfiles) + np.tile(live1, nb)
    j["size"] = rec
    j["new_offset"] = (np.tile(np.arange(nl, dtype=np.int64), nb) * rec).astype(np.int32)
    n = j.size
    d_jobs = crc.DeviceBuffer(ctx, j.nbytes).upload(j)
    dest_bytes = n * rec + 256
    d_dst = crc.DeviceBuffer(ctx, dest_bytes)
    h_dst = crc.PinnedBuffer(ctx, dest_bytes)
    d_st = crc.DeviceBuffer(ctx, 4 * n)
    d_bad = crc.DeviceBuffer(ctx, 4)
    hp_src, hp_dst = ctx.host_device_ptr(h_src.ptr), ctx.host_device_ptr(h_dst.ptr)
    src_len = ndist * blk
    cases = {"zc_both": (hp_src, hp_dst), "zc_read": (hp_src, d_dst.ptr), "zc_write": (d_src.ptr, hp_dst),
             "hbm": (d_src.ptr, d_dst.ptr)}
    for name, (s, dd) in cases.items():  # every case byte-exact against the HBM form, no bad records
        d_bad.zero()
        ctx.compact_jobs_device(s, src_len, d_jobs, n, dd, None, d_st, d_bad)
        ctx.sync()
        if int(d_bad.download(np.uint32)[0]) != 0:
            raise SystemExit("probe: %s reports bad records" % name)
    if not (h_dst.array[:n * rec] == d_dst.download(np.uint8, n * rec)).all():
        raise SystemExit("probe: zero-copy destination differs from the HBM one")
    vj = j.copy()
    d_vjobs = crc.DeviceBuffer(ctx, vj.nbytes).upload(vj)
    times = {k: [] for k in list(cases) + ["verify_zc", "blocks_compact_product"]}
    # the product host path over the same blocks: tfs_blocks_compact, page-locked images
    metas = np.zeros(nfiles, crc.META_DTYPE)
    metas["file_id"] = np.arange(1, nfiles + 1)
    metas["offset"] = np.arange(nfiles) * rec
    metas["size"] = rec
    flags = bench._fragmented_flags(nfiles)
    pdst = [crc.PinnedBuffer(ctx, blk) for _ in range(ndist)]
    bjobs = (crc.BlockJob * nb)()
    for k in range(nb):
        x = bjobs[k]
        x.src_image, x.src_len = h_src.ptr + (k % ndist) * blk, blk
        x.metas, x.flags, x.n = metas.ctypes.data, flags.ctypes.data, nfiles
        x.dest_image, x.dest_cap = pdst[k % ndist].ptr, blk
    ctx.blocks_compact(bjobs)
    for r in range(rounds):
        for name, (s, dd) in cases.items():
            e0, e1 = crc.Event(ctx), crc.Event(ctx)
            e0.record()
            for _ in range(reps):
                ctx.compact_jobs_device(s, src_len, d_jobs, n, dd, None, d_st, d_bad)
            e1.record()
            ctx.sync()
            times[name].append(e0.elapsed_ms(e1) / reps)
        e0, e1 = crc.Event(ctx), crc.Event(ctx)
        e0.record()
        for _ in range(reps):
            ctx.blocks_verify_device(hp_src, src_len, d_vjobs, n, None, d_st, d_bad)
        e1.record()
        ctx.sync()
        times["verify_zc"].append(e0.elapsed_ms(e1) / reps)
        t0 = time.perf_counter()
        ctx.blocks_compact(bjobs)
        times["blocks_compact_product"].append((time.perf_counter() - t0) * 1e3)
        print("round %d done" % r, file=sys.stderr, flush=True)
    ceil = pcie_ceiling(ctx)
    live_bytes = float(n) * rec
    res = {}
    for name, v in times.items():
        v = sorted(v)
        med = v[len(v) // 2]
        per_dir = live_bytes / (med / 1e3) / 1e9  # GB/s of records moved in each direction that crosses PCIe
        res[name] = {"median_ms": med, "min_ms": v[0], "max_ms": v[-1], "records_GBs": per_dir}
    out = {"tool": "compact_direction_probe", "blocks": nb, "records": n, "record_bytes": rec,
           "live_bytes_per_launch": live_bytes, "rounds": rounds, "reps": reps,
           "pcie": {k: ceil[k] for k in ("h2d_GBs", "d2h_GBs", "duplex_GBs")}, "cases": res,
           "note": "records_GBs = live record bytes / time: for zc_both the rate of EACH direction (the "
                   "link carries it both ways), zc_read / verify_zc H2D only, zc_write D2H only"}
    print(json.dumps(out))
    for x in pdst + [h_src, h_dst]:
        x.free()


if __name__ == "__main__":
    main()
