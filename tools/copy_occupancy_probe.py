#!/usr/bin/env python3
"""Copy ceilings by occupancy (measurement only): the wave-contiguous chunk copy
(membench 53104: 64 KiB per wave, nt stores) and the grid-stride copy (52114) of
the device compaction's 21.3 GiB at 1, 2 and 4 workgroups of 16 waves per CU, all
interleaved in one process -- does the record kernel's one workgroup per CU
(held there by its 140 KiB of LDS tables) cost its copy form anything?

  python tools/copy_occupancy_probe.py [ROUNDS]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tfs_amd.crc as crc  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    ctx = crc.Context(0, measure=True)  # calibration kernels: measurement build
    nbytes = 349184 * 65572 // 16 * 16
    src = crc.DeviceBuffer(ctx, nbytes + 4096)
    dst = crc.DeviceBuffer(ctx, nbytes + 4096)
    ctx.synth_fill_device(src, nbytes, 0xC0FE, 0)
    cases = [(53104, 256), (53104, 512), (53104, 1024), (52114, 256), (52114, 512), (52114, 2048)]
    times = {c: [] for c in cases}
    for _ in range(rounds):
        for pat, grid in cases:
            ctx.membench_device(pat, src, None, 0, nbytes, dst, grid=grid)
            e0, e1 = crc.Event(ctx), crc.Event(ctx)
            e0.record()
            for _ in range(3):
                ctx.membench_device(pat, src, None, 0, nbytes, dst, grid=grid)
            e1.record()
            ctx.sync()
            times[(pat, grid)].append(e0.elapsed_ms(e1) / 3)
    res = {}
    for (pat, grid), v in times.items():
        v = sorted(v)
        med = v[len(v) // 2]
        res["p%d_g%d" % (pat, grid)] = {"median_ms": med, "frac_8TBs_rw": 2.0 * nbytes / (med / 1e3) / 1e9 / 8000.0}
    print(json.dumps({"tool": "copy_occupancy_probe", "bytes": nbytes, "rounds": rounds, "copy": res}))
    src.free()
    dst.free()
    ctx.close()


if __name__ == "__main__":
    main()
