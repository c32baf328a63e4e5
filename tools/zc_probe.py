"""Measurement probe (not product, not a test): GPU-initiated reads/writes of
pinned host memory (zero-copy) vs DMA copies, to size the compaction path."""
import json
import os
import sys
import time


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfs_amd.crc as crc  # noqa: E402

ctx = crc.Context(0, measure=True)  # calibration kernels: measurement build
N = 1 << 30
h = crc.PinnedBuffer(ctx, N)
h2 = crc.PinnedBuffer(ctx, N)
h.array[:] = 1
d = crc.DeviceBuffer(ctx, N)
out = crc.DeviceBuffer(ctx, 64)
res = {}


def t(fn, reps=3):
    fn()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.sync()
    return (time.perf_counter() - t0) / reps


for grid in (256, 1024, 2048, 4096):
    for pat in (0, 1000):
        s = t(lambda: ctx.membench_device(pat, h.ptr, None, 0, N, out, grid=grid))
        res["zc_read_p%d_g%d_GBs" % (pat, grid)] = N / s / 1e9
for grid in (256, 2048):
    for pat in (52004, 52114):  # grid-stride copies: plain, and nt loads + stores
        s = t(lambda: ctx.membench_device(pat, h.ptr, None, 0, N // 2, h2.ptr, grid=grid))
        res["zc_host2host_copy_p%d_g%d_GBs_each_way" % (pat, grid)] = (N // 2) / s / 1e9
        s = t(lambda: ctx.membench_device(pat, d.ptr, None, 0, N, h2.ptr, grid=grid))
        res["zc_write_from_dev_p%d_g%d_GBs" % (pat, grid)] = N / s / 1e9
s = t(lambda: crc.lib().tfs_crc32_memcpy(ctx.handle, d.ptr, h.ptr, N, None))
res["dma_h2d_GBs"] = N / s / 1e9
s = t(lambda: crc.lib().tfs_crc32_memcpy(ctx.handle, h2.ptr, d.ptr, N, None))
res["dma_d2h_GBs"] = N / s / 1e9
print(json.dumps(res, indent=1))
