#!/usr/bin/env python3
"""Read ceilings of the headline and Zipf images (measurement only).

Builds bench.py's configs[1] resident set (or benchlines.zipf's configs[2]
image), times the product kernel on it, then the calibration kernels of the
measurement build (libtfs_crc_measure.so, membench_kernel) over the same bytes:
the kernel's own access pattern without the CRC arithmetic and the grid-stride
stream -- the ceilings the kernel is held to.  One JSON line on stdout.

  python tools/ceilings.py verify|zipf [ROUNDS]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import tfs_amd.crc as crc  # noqa: E402
from benchlines import zipf as zl  # noqa: E402

# pattern ids of launch_membench (tfs_crc_kernels.hip): 1000 grid-stride; 11016 the
# kernel's 1 KiB stripes with 128-byte anchors.  (The wave- and workgroup-contiguous
# chunk reads, 54xxx / 55xxx, were deleted in round 5; DESIGN §4 keeps what they read.)
VERIFY_PATTERNS = [(1000, 0), (1000, 1024), (11016, 0)]
ZIPF_PATTERNS = [(11016, 0), (1000, 0), (1000, 1024)]


def timed(c, fn, reps=5):
    fn()
    e0, e1 = crc.Event(c), crc.Event(c)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    c.sync()
    return e0.elapsed_ms(e1) / reps


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "verify"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ctx = crc.Context(0)
    mctx = crc.Context(0, measure=True)
    out = crc.DeviceBuffer(ctx, 16)
    if mode == "zipf":
        img, offs, lens, total = zl.build(ctx, 1024, 42)
        n = len(lens)
        desc = np.zeros(n, crc.DESC_DTYPE)
        desc["offset"], desc["len"] = offs, lens
        d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
        d_out = crc.DeviceBuffer(ctx, 4 * n)
        algo = float(lens.astype(np.float64).sum()) + 21.0 * n
        kernel = (lambda: ctx.batch_device(d_desc, n, img, d_out))
        stripes = np.maximum(lens.astype(np.int64) - 127, 0) // 1024
        pats = [(p, g, float(stripes.sum()) * 1024.0 if p == 11016 else float(total)) for p, g in ZIPF_PATTERNS]
    else:
        nfiles = 1024 * bench.FILES_PER_BLOCK
        img, desc, expected, total = bench.build_headline(ctx, 1024, bench.rank_blocks(1024, 1, 0), 0)
        n = nfiles
        d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
        d_ok = crc.DeviceBuffer(ctx, n)
        algo = float(n) * bench.ALGO_BYTES_PER_FILE
        kernel = (lambda: ctx.verify_device(d_desc, n, img, None, d_ok, None))
        pats = []
        for p, g in VERIFY_PATTERNS:
            if p % 1000 == 0:
                nb = total
            else:
                run = p % 1000
                nb = n * ((bench.FILE_SIZE - 127) // (64 * run)) * 64 * run
            pats.append((p, g, float(nb)))
    res = {"kernel": [], **{"p%d_g%d" % (p, g): [] for p, g, _ in pats}}
    for _ in range(rounds):
        res["kernel"].append(algo / (timed(ctx, kernel) / 1e3) / 1e9)
        for p, g, nb in pats:
            ms = timed(mctx, lambda: mctx.membench_device(p, img, d_desc, n, total, out, grid=g))
            res["p%d_g%d" % (p, g)].append(nb / (ms / 1e3) / 1e9)
    print(json.dumps({"tool": "ceilings", "mode": mode, "rounds": rounds,
                      "GBs_median": {k: sorted(v)[len(v) // 2] for k, v in res.items()}, "GBs_all": res}))


if __name__ == "__main__":
    main()
