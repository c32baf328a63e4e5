#!/usr/bin/env python3
"""One streaming-copy calibration kernel of the measurement build over a fixed
byte count, alone in its process (measurement only): the dense-copy reference
the device compaction (compact_pipe_kernel) is compared with, in a form a
rocprofv3 --pmc pass can isolate.

  python tools/copy_probe.py PATTERN [GRID] [GIB] [REPS]

PATTERN: launch_membench ids (tfs_crc_kernels.hip), e.g. 53104 (wave-contiguous
64 KiB chunks, nt stores), 53101 (16 KiB chunks), 52114 (grid-stride).  GIB
defaults to the compact_device line's live bytes (349,184 records x 65,572 B).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tfs_amd.crc as crc  # noqa: E402


def main():
    pat = int(sys.argv[1])
    grid = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    nb = int(float(sys.argv[3]) * 2**30) if len(sys.argv) > 3 else 349184 * 65572
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    nb = nb // 65536 * 65536
    ctx = crc.Context(0, measure=True)
    src = crc.DeviceBuffer(ctx, nb + 4096)
    dst = crc.DeviceBuffer(ctx, nb + 4096)
    ctx.synth_fill_device(src, nb, 7, 0)
    ctx.membench_device(pat, src, None, 0, nb, dst, grid=grid)
    e0, e1 = crc.Event(ctx), crc.Event(ctx)
    e0.record()
    for _ in range(reps):
        ctx.membench_device(pat, src, None, 0, nb, dst, grid=grid)
    e1.record()
    ctx.sync()
    ms = e0.elapsed_ms(e1) / reps
    print(json.dumps({"tool": "copy_probe", "pattern": pat, "grid": grid, "bytes": nb, "ms": ms,
                      "GBs_rw": 2 * nb / (ms / 1e3) / 1e9, "frac_8TBs": 2 * nb / (ms / 1e3) / 1e9 / 8000.0}))


if __name__ == "__main__":
    main()
