#!/usr/bin/env python3
"""Copy ceilings of the device compaction's bytes (measurement only): the
runtime's own device-to-device copy (hipMemcpyAsync D2D through torch's
`copy_`, the ROCm blit kernel) beside the measurement build's copy kernels of
the same byte count (membench 53104: wave-contiguous 64 KiB chunks, nt stores;
52114: grid-stride, 4 chunks in flight), interleaved round by round in one
process.  Is there a copy of these bytes faster than the one the record kernel
matches (`compact_vs_copy`)?

  python tools/copy_ceiling_probe.py [ROUNDS] [GIB]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import tfs_amd.crc as crc  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    gib = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    nbytes = int(gib * 2**30) // 65536 * 65536 if gib else 349184 * 65572 // 65536 * 65536
    ctx = crc.Context(0, measure=True)
    src = crc.DeviceBuffer(ctx, nbytes + 4096)
    dst = crc.DeviceBuffer(ctx, nbytes + 4096)
    ctx.synth_fill_device(src, nbytes, 0xC0FE, 0)
    ctx.sync()
    tsrc = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    tdst = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    tsrc.fill_(7)
    torch.cuda.synchronize()
    ours = [(53104, 256), (53104, 512), (53116, 256), (52114, 2048), (52114, 8192), (52004, 2048)]
    times = {"hipMemcpyD2D_torch": []}
    for pat, grid in ours:
        times["p%d_g%d" % (pat, grid)] = []
    for _ in range(rounds):
        tdst.copy_(tsrc)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            tdst.copy_(tsrc)
        e1.record()
        torch.cuda.synchronize()
        times["hipMemcpyD2D_torch"].append(e0.elapsed_time(e1) / 3)
        for pat, grid in ours:
            ctx.membench_device(pat, src, None, 0, nbytes, dst, grid=grid)
            e0, e1 = crc.Event(ctx), crc.Event(ctx)
            e0.record()
            for _ in range(3):
                ctx.membench_device(pat, src, None, 0, nbytes, dst, grid=grid)
            e1.record()
            ctx.sync()
            times["p%d_g%d" % (pat, grid)].append(e0.elapsed_ms(e1) / 3)
        print("round done", file=sys.stderr, flush=True)
    res = {}
    for k, v in times.items():
        v = sorted(v)
        med = v[len(v) // 2]
        res[k] = {"median_ms": med, "min_ms": v[0], "frac_8TBs_rw": 2.0 * nbytes / (med / 1e3) / 1e9 / 8000.0}
    print(json.dumps({"tool": "copy_ceiling_probe", "bytes": nbytes, "rounds": rounds, "copy": res}))


if __name__ == "__main__":
    main()
