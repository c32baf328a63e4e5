#!/usr/bin/env python3
"""Same-process A/B of the host-memory verify paths (round 5; measurement only).

  e2e      configs[4]'s end-to-end leg: 64 MiB page-locked block images submitted
           3 at a time (tfs_crc32_submit_verify / wait), ms per block
  blockv   one tfs_block_verify per fragmented page-locked block (341 of 1,024
           records), ms per block

each through the product context (wide page-locked batches read in place by the
throughput kernel; block verify with metas and verdicts in page-locked words) and a
measurement context with TFS_CRC_VARIANT=52 (the round-4 forms: the block image
staged by DMA; block verify with its metas and verdicts copied), interleaved round
by round.

  python tools/ab_host_paths.py [ROUNDS] [BLOCKS]
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
from benchlines.common import _fragmented_flags, pcie_ceiling  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    nblk = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    ctx = crc.Context(0)
    os.environ["TFS_CRC_VARIANT"] = "52"
    staged = crc.Context(0, measure=True)
    os.environ["TFS_CRC_VARIANT"] = "0"
    nfiles, rec = bench.FILES_PER_BLOCK, bench.FILEINFO + bench.FILE_SIZE
    blk = nfiles * rec
    d_img = crc.DeviceBuffer(ctx, blk + 64)
    desc = np.zeros(nfiles, crc.DESC_DTYPE)
    desc["offset"], desc["len"] = np.arange(nfiles) * rec + bench.FILEINFO, bench.FILE_SIZE
    d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_crc = crc.DeviceBuffer(ctx, 4 * nfiles)
    d_off = crc.DeviceBuffer(ctx, 8 * nfiles).upload(np.arange(nfiles, dtype=np.uint64) * rec)
    d_len = crc.DeviceBuffer(ctx, 4 * nfiles).upload(np.full(nfiles, bench.FILE_SIZE, np.uint32))
    srcs, exps = [], []
    for b in range(8):
        ctx.synth_fill_device(d_img, (blk + 64) // 8 * 8, 0xAB0 + b, 0)
        ctx.batch_device(d_desc, nfiles, d_img, d_crc)
        ctx.write_headers_device(d_img, d_off, d_len, d_crc, 1, nfiles)
        ctx.sync()
        p = crc.PinnedBuffer(ctx, blk)
        p.array[:] = d_img.download(np.uint8, blk)
        srcs.append(p)
        exps.append(d_crc.download(np.uint32))
    offs, lens = desc["offset"], desc["len"]
    metas = np.zeros(nfiles, crc.META_DTYPE)
    metas["file_id"] = np.arange(1, nfiles + 1)
    metas["offset"] = np.arange(nfiles) * rec
    metas["size"] = rec
    live = np.ascontiguousarray(metas[_fragmented_flags(nfiles) == 0])

    def e2e(c):
        hs, bad = [], 0
        t0 = time.perf_counter()
        for i in range(nblk):
            if len(hs) >= 3:
                bad += c.wait(hs.pop(0))[2]
            hs.append(c.submit_verify(srcs[i % 8].array, offs, lens, exps[i % 8]))
        while hs:
            bad += c.wait(hs.pop(0))[2]
        el = time.perf_counter() - t0
        if bad:
            raise SystemExit("ab_host_paths: e2e mismatches")
        return el / nblk * 1e3

    def blockv(c):
        t0 = time.perf_counter()
        for i in range(nblk):
            _, st, nbad, _ = c.block_verify(srcs[i % 8].array, live)
            if nbad:
                raise SystemExit("ab_host_paths: block verify mismatches")
        return (time.perf_counter() - t0) / nblk * 1e3

    cases = {"e2e_product": (e2e, ctx), "e2e_staged": (e2e, staged),
             "blockv_product": (blockv, ctx), "blockv_staged": (blockv, staged)}
    for fn, c in cases.values():  # warm every slot and path
        for _ in range(2):
            fn(c)
    times = {k: [] for k in cases}
    for r in range(rounds):
        for k, (fn, c) in cases.items():
            times[k].append(fn(c))
        print("round %d done" % r, file=sys.stderr, flush=True)
    ceil = pcie_ceiling(ctx)
    res = {}
    for k, v in times.items():
        v = sorted(v)
        med = v[len(v) // 2]
        nbytes = blk if k.startswith("e2e") else live.size * rec
        res[k] = {"median_ms_per_block": med, "min": v[0], "max": v[-1], "pcie_GBs": nbytes / (med / 1e3) / 1e9,
                  "frac_h2d": nbytes / (med / 1e3) / 1e9 / ceil["h2d_GBs"]}
    print(json.dumps({"tool": "ab_host_paths", "blocks": nblk, "rounds": rounds, "h2d_GBs": ceil["h2d_GBs"],
                      "ab": res}))


if __name__ == "__main__":
    main()
