#!/usr/bin/env python3
"""configs[0] loopback throughput against the CloseBatcher's batch size
(measurement only): the bench's loopback (1,024 x 64 KiB through the harness,
page-locked block images) with 8 and 64 closing threads, for each max_batch,
interleaved round by round in one process; plus the close latency at 1/8/64
leases.

  python tools/loopback_probe.py [ROUNDS]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tfs_amd.crc as crc  # noqa: E402
import tfs_amd.dataserver as ds  # noqa: E402
from tfs_amd.synth import synth_bytes  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ctx = crc.Context(0)
    n, L = 1024, 65536
    pay = synth_bytes(0x9E3779B97F4A7C15, n * L)
    client = ctx.batch(pay, np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint32))
    pool = ds.BlockImagePool(ctx, 2, n * (L + 36) + 4096)
    cases = [(8, 8, 8, 0), (8, 4, 8, 0), (8, 2, 8, 0), (8, 1, 8, 0), (64, 16, 8, 0), (64, 8, 8, 0), (64, 4, 8, 0),
             (64, 2, 8, 0)]
    if os.environ.get("LB_CASES"):
        # "threads:batch[:in_flight[:pool]],..." (in_flight: batches in use at once, 1-16; pool 1: the
        # DataFile buffers from a page-locked LeaseBufferPool, checked in place)
        cases = [tuple(int(v) for v in (c.split(":") + ["8", "0"])[:4]) for c in os.environ["LB_CASES"].split(",")]
    lease_pool = ds.LeaseBufferPool(ctx, 128)
    batchers = {c: ds.CloseBatcher(ctx, max_batch=c[1], max_wait_us=100, in_flight=c[2],
                                   pool=lease_pool if c[3] else None) for c in cases}

    def key(c):
        return "%d_threads_batch_%d%s%s" % (c[0], c[1], "_inflight_%d" % c[2] if c[2] != 8 else "",
                                          "_pool" if c[3] else "")
    times = {key(c): [] for c in cases}
    for _ in range(2):  # warm-up
        for c in cases:
            blk = ds.LogicBlock(1, pool=pool)
            assert ds.loopback_block(ctx, pay, n, L, client, c[0], blk, batchers[c]) == 0
            blk.free()
    for r in range(rounds):
        for c in cases:
            t0 = time.perf_counter()
            for _ in range(4):
                blk = ds.LogicBlock(1, pool=pool)
                assert ds.loopback_block(ctx, pay, n, L, client, c[0], blk, batchers[c]) == 0
                blk.free()
            times[key(c)].append((time.perf_counter() - t0) / 4)
        print("round %d" % r, file=sys.stderr, flush=True)
    res = {k: {"GiBs_median": n * L / sorted(v)[len(v) // 2] / 2**30, "GiBs_best": n * L / min(v) / 2**30}
           for k, v in times.items()}
    lat = {}
    for leases in (1, 8, 64, 1):
        us = ds.close_latency(ctx, leases, 200 if leases < 64 else 40)
        lat["close_%d_leases%s" % (leases, "_again" if "close_%d_leases" % leases in lat else "")] = {"p50_us": float(np.percentile(us, 50)),
                                           "p99_us": float(np.percentile(us, 99))}
    print(json.dumps({"tool": "loopback_probe", "rounds": rounds, "loopback": res, "latency": lat}))


if __name__ == "__main__":
    main()
