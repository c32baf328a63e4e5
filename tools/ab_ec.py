#!/usr/bin/env python3
"""Same-process A/B of erasure-code kernel forms (measurement only).

Builds the ec line's members (k = 5 data + m = 3 parity of 1,536 MiB, device
resident), then interleaves, round by round, encodes through the product
library and through measurement-build forms selected by TFS_EC_VARIANT
(tfs_ec_kernels.hip: 1-3 chunked tiles, 4 / 6 striding grids; 20 / 21 the
5-read : 3-write copy ceiling of the same tile walk -- one member ahead as the
product, or all five members' loads in flight -- with one XOR per dword instead
of the bitmatrix, not an erasure code), each timed with HIP events.  (Round 5's form 7, every source member's loads in flight at once, was
measured and deleted: DESIGN.md §4.2.)

  python tools/ab_ec.py VARIANTS [ROUNDS] [MIB]     e.g. python tools/ab_ec.py 1,4 8
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tfs_amd.crc as crc  # noqa: E402
from tfs_amd.ec import ErasureCode  # noqa: E402


def main():
    variants = [int(v) for v in sys.argv[1].split(",") if v]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    size = (int(sys.argv[3]) if len(sys.argv) > 3 else 1536) << 20
    k, m = 5, 3
    ctx = crc.Context(0)
    d = [crc.DeviceBuffer(ctx, size + 64) for _ in range(k + m)]
    for i in range(k):
        ctx.synth_fill_device(d[i], size, 0xEC0 + i, 0)
    ctx.sync()
    forms = {"product": (ctx, ErasureCode(ctx, k, m))}
    mctx = {}
    for v in variants:
        os.environ["TFS_EC_VARIANT"] = str(v)
        c = crc.Context(0, measure=True)
        forms["v%d" % v] = (c, ErasureCode(c, k, m))
        mctx[v] = c
    os.environ.pop("TFS_EC_VARIANT", None)
    times = {name: [] for name in forms}
    for _ in range(rounds):
        for name, (c, e) in forms.items():
            e.encode_device(d, size)
            e0, e1 = crc.Event(c), crc.Event(c)
            e0.record()
            for _ in range(3):
                e.encode_device(d, size)
            e1.record()
            c.sync()
            times[name].append(e0.elapsed_ms(e1) / 3)
    res = {}
    for name, t in times.items():
        t = sorted(t)
        med = t[len(t) // 2]
        res[name] = {"median_ms": med, "min_ms": t[0], "max_ms": t[-1],
                     "frac_8TBs": (k + m) * size / (med / 1e3) / 1e9 / 8000.0}
    print(json.dumps({"tool": "ab_ec", "k": k, "m": m, "member_bytes": size, "rounds": rounds, "ab": res}))


if __name__ == "__main__":
    main()
