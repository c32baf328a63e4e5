#!/usr/bin/env python3
"""Blocks per launch of zero-copy host compaction (tfs_blocks_compact,
TFS_CRC_COMPACT_GROUP; round 5).  Measurement only.

BASELINE configs[3]'s job list (fragmented 64 MiB blocks of 64 KiB records, 341
of every 1,024 live, 8 distinct page-locked images cycled) compacted by contexts
created with 1 (per-block launches, the round-4 product) to 256 blocks per launch, interleaved in one process, wall time per call.

  CG_GROUPS=1,8,16,32,64 python tools/compact_group_probe.py [NBLOCKS] [ROUNDS]

(bash reserves GROUPS, so the list is CG_GROUPS.)
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
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    groups = [int(x) for x in os.environ.get("CG_GROUPS", "1,8,16,32,64").split(",")]
    ctxs = {}
    for g in groups:
        os.environ["TFS_CRC_COMPACT_GROUP"] = str(g)
        ctxs[g] = crc.Context(0)
    os.environ.pop("TFS_CRC_COMPACT_GROUP")
    ctx = ctxs[groups[-1]]
    nfiles, rec = bench.FILES_PER_BLOCK, bench.FILEINFO + bench.FILE_SIZE
    blk = nfiles * rec
    ndist = 8
    d_img = crc.DeviceBuffer(ctx, blk + 64)
    desc = np.zeros(nfiles, crc.DESC_DTYPE)
    desc["offset"], desc["len"] = np.arange(nfiles) * rec + bench.FILEINFO, bench.FILE_SIZE
    d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_crc = crc.DeviceBuffer(ctx, 4 * nfiles)
    d_off = crc.DeviceBuffer(ctx, 8 * nfiles).upload(np.arange(nfiles, dtype=np.uint64) * rec)
    d_len = crc.DeviceBuffer(ctx, 4 * nfiles).upload(np.full(nfiles, bench.FILE_SIZE, np.uint32))
    srcs, dests = [], []
    for b in range(ndist):
        ctx.synth_fill_device(d_img, (blk + 64) // 8 * 8, 0xB10C + 97 * b, 0)
        ctx.batch_device(d_desc, nfiles, d_img, d_crc)
        ctx.write_headers_device(d_img, d_off, d_len, d_crc, 1, nfiles)
        ctx.sync()
        p = crc.PinnedBuffer(ctx, blk)
        p.array[:] = d_img.download(np.uint8, blk)
        srcs.append(p)
        dests.append(crc.PinnedBuffer(ctx, blk))
    metas = np.zeros(nfiles, crc.META_DTYPE)
    metas["file_id"] = np.arange(1, nfiles + 1)
    metas["offset"] = np.arange(nfiles) * rec
    metas["size"] = rec
    flags = bench._fragmented_flags(nfiles)
    live = int((flags == 0).sum())
    jobs = (crc.BlockJob * nb)()
    for j in range(nb):
        x = jobs[j]
        x.src_image, x.src_len = srcs[j % ndist].ptr, blk
        x.metas, x.flags, x.n = metas.ctypes.data, flags.ctypes.data, nfiles
        x.dest_image, x.dest_cap = dests[j % ndist].ptr, blk
    for g in groups:  # warm every context's slots and streams
        if ctxs[g].blocks_compact(jobs) != 0:
            raise SystemExit("probe: group %d reports bad records" % g)
    times = {g: [] for g in groups}
    for r in range(rounds):
        for g in groups:
            t0 = time.perf_counter()
            ctxs[g].blocks_compact(jobs)
            times[g].append(time.perf_counter() - t0)
        print("round %d done" % r, file=sys.stderr, flush=True)
    ceil = pcie_ceiling(ctx)
    res = {}
    for g in groups:
        v = sorted(times[g])
        med = v[len(v) // 2]
        gbs = 2.0 * nb * live * rec / med / 1e9
        res[str(g)] = {"median_ms_per_block": med / nb * 1e3, "pcie_GBs_both_ways": gbs,
                       "frac_of_duplex": gbs / ceil["duplex_GBs"]}
    print(json.dumps({"tool": "compact_group_probe", "blocks": nb, "live_per_block": live, "rounds": rounds,
                      "pcie": {k: ceil[k] for k in ("h2d_GBs", "d2h_GBs", "duplex_GBs")}, "groups": res}))


if __name__ == "__main__":
    main()
