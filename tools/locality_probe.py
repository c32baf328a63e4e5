"""Measurement probe (not product, not a test): does the headline kernel's
wave-per-file access pattern lose HBM bandwidth to address spread?

The verify kernel runs 4,096 waves, each streaming its own 64 KiB file, so the
reads in flight at any moment spread over a 256 MiB window.  A grid-stride
stream of the same image keeps them inside a few MiB and reads faster
(DESIGN.md §4 calibration).  This probe runs the same wave-per-descriptor
pattern (`membench_kernel`, 1 KiB stripes, 16 B per lane, non-temporal) over
one 64 GiB image cut into contiguous segments of S bytes -- S = 64 KiB is the
headline geometry; smaller S is what splitting each file over several waves
(segment chains combined by a CRC shift) would give -- and the grid-stride
stream beside it.  Output: one JSON line, GB/s per segment size."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfs_amd.crc as crc  # noqa: E402

ctx = crc.Context(0, measure=True)  # calibration kernels: measurement build
TOTAL = 64 << 30
img = crc.DeviceBuffer(ctx, TOTAL + 4096)
ctx.synth_fill_device(img, TOTAL, 7, 0)
out = crc.DeviceBuffer(ctx, 64)
res = {}


def timed(pattern, d_desc, n, nbytes, grid=0, reps=5):
    ctx.membench_device(pattern, img, d_desc, n, TOTAL, out, grid=grid)
    e0, e1 = crc.Event(ctx), crc.Event(ctx)
    e0.record()
    for _ in range(reps):
        ctx.membench_device(pattern, img, d_desc, n, TOTAL, out, grid=grid)
    e1.record()
    ctx.sync()
    return nbytes / (e0.elapsed_ms(e1) / reps / 1e3) / 1e9


for rnd in range(2):  # two interleaved rounds: box noise shows as round-to-round spread
    res.setdefault("grid_stride_GBs", []).append(timed(1000, None, 0, TOTAL))
    for seg in (65536, 32768, 16384, 8192, 4096):
        n = TOTAL // seg
        desc = np.zeros(n, crc.DESC_DTYPE)
        desc["offset"] = np.arange(n, dtype=np.uint64) * seg
        desc["len"] = seg + 16  # (len - 15) // 1024 == seg // 1024 whole stripes from a 16-aligned start
        d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
        res.setdefault("wave_per_%dKiB_GBs" % (seg >> 10), []).append(timed(1016, d_desc, n, TOTAL))
        d_desc.free()
# Occupancy: the same patterns at 1, 2 and 4 workgroups of 16 waves per CU
# (the CRC kernel is held to 1 by its 128 KiB of LDS tables).
seg = 65536
n = TOTAL // seg
desc = np.zeros(n, crc.DESC_DTYPE)
desc["offset"] = np.arange(n, dtype=np.uint64) * seg
desc["len"] = seg + 16
d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
for grid in (256, 512, 1024):
    res["wave_per_64KiB_grid%d_GBs" % grid] = timed(1016, d_desc, n, TOTAL, grid=grid)
    res["grid_stride_grid%d_GBs" % grid] = timed(1000, None, 0, TOTAL, grid=grid)
d_desc.free()
print(json.dumps({"locality_probe": res}), flush=True)
img.free()
out.free()
ctx.close()
