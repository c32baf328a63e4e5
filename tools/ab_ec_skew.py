#!/usr/bin/env python3
"""Member placement A/B of the erasure-code kernel (VERDICT r4
weak item 9; measurement only).

The kernel reads unit u of every data member and writes unit u of every parity
member in one wave, so the 8 addresses a wave touches at once differ by the
members' base distances.  bench.py allocates each 1.5 GiB member on its own
(hipMalloc places them one after another), which makes those distances nearly
the same multiple of a large power of two for every member.  This times
ErasureCode encode (k=5, m=3, the same kernel and launch) with the members
carved from one allocation at base + i * (size + skew) for several skews,
interleaved round by round with the separately allocated members, HIP events
around REPS encodes each.  The parity bytes of every placement are checked
against the separately allocated members' at three offsets first.

  python tools/ab_ec_skew.py [ROUNDS] [MIB]      (AB_SKEWS=0,4096,... bytes)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tfs_amd.crc as crc  # noqa: E402
from tfs_amd.ec import ErasureCode  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 1536
    skews = [int(x) for x in os.environ.get("AB_SKEWS", "0,4096,12288,69632,266240,2166784").split(",") if x]
    reps = 3
    k, m = 5, 3
    size = mib << 20
    ctx = crc.Context(0)
    enc = ErasureCode(ctx, k, m)
    sep = [crc.DeviceBuffer(ctx, size + 64) for _ in range(k + m)]
    for i in range(k):
        ctx.synth_fill_device(sep[i], size, 0xEC0 + i, 0)
    smax = max(skews)
    big = crc.DeviceBuffer(ctx, (k + m) * (size + smax) + 4096)
    places = {"separate": [b.ptr for b in sep]}
    for s in skews:
        places["skew%d" % s] = [big.ptr + i * (size + s) for i in range(k + m)]
    if enc.encode_device(sep, size) != 0:
        raise SystemExit("ab_ec_skew: encode failed")
    ctx.sync()
    probe = [0, size // 2 + 4096, size - 65536]
    want = {(i, o): sep[i].download(np.uint8, 65536, o) for i in range(k, k + m) for o in probe}
    for name, ptrs in places.items():
        if name == "separate":
            continue
        base_skew = int(name[4:])
        # fill the carved data members with the same bytes (synth_fill writes from a buffer's start)
        for i in range(k):
            off = i * (size + base_skew)
            ctx.synth_fill_device(big.ptr + off, size, 0xEC0 + i, 0)
        if enc.encode_device(ptrs, size) != 0:
            raise SystemExit("ab_ec_skew: encode failed on %s" % name)
        ctx.sync()
        for (i, o), w in want.items():
            got = big.download(np.uint8, 65536, i * (size + base_skew) + o)
            if not (got == w).all():
                raise SystemExit("ab_ec_skew: %s parity member %d differs at %d" % (name, i, o))
    times = {k_: [] for k_ in places}
    for r in range(rounds):
        for name, ptrs in places.items():
            enc.encode_device(ptrs, size)
            e0, e1 = crc.Event(ctx), crc.Event(ctx)
            e0.record()
            for _ in range(reps):
                enc.encode_device(ptrs, size)
            e1.record()
            ctx.sync()
            times[name].append(e0.elapsed_ms(e1) / reps)
        print("round %d done" % r, file=sys.stderr, flush=True)
    algo = float(k + m) * size
    res = {}
    for name, v in times.items():
        v = sorted(v)
        med = v[len(v) // 2]
        res[name] = {"median_ms": med, "min_ms": v[0], "max_ms": v[-1], "frac_8TBs": algo / (med / 1e3) / 1e9 / 8000.0,
                     "member_bases_mod_2MiB": [int(p % (2 << 20)) for p in places[name]]}
    print(json.dumps({"tool": "ab_ec_skew", "k": k, "m": m, "member_bytes": size, "rounds": rounds, "reps": reps,
                      "algo_bytes_per_launch": algo, "ab": res}))


if __name__ == "__main__":
    main()
