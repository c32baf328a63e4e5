#!/usr/bin/env python3
"""Same-process A/B of the packet CRC path (VERDICT r4 item 6;
measurement only).  Builds bench.py's packet workload once (1 M device-resident
V1 frames carrying 64 KiB WriteDataMessages, sealed on the device), then
interleaves, round by round:

  one_pass   tfs_packet_verify_device, the product (packet_files_kernel: the
             header parsed by the wave that checksums the body)
  three      the same call through the three-launch form (TFS_CRC_VARIANT=51:
             parse, crc_files_kernel, finish)
  verify     tfs_crc32_verify_device over the same frames' bodies (descriptors
             built on the host, expected = the bodies' seed-0 CRCs): the headline kernel
             on exactly these bytes, no packet work at all

each timed with HIP events around REPS launches on its own context's stream.

  python tools/ab_packet.py [ROUNDS] [NBLOCKS]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import tfs_amd.crc as crc  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    nblocks = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    reps = 3
    ctx = crc.Context(0)
    os.environ["TFS_CRC_VARIANT"] = "51"
    c3 = crc.Context(0, measure=True)
    os.environ["TFS_CRC_VARIANT"] = "0"
    body = 32 + 4 + 6 * 8 + bench.FILE_SIZE
    frame = 24 + body
    n = nblocks * bench.FILES_PER_BLOCK
    total = n * frame
    img = crc.DeviceBuffer(ctx, (total + 4095) // 4096 * 4096)
    ctx.synth_fill_device(img, (total + 7) // 8 * 8, 0x5EED, 0)
    off = np.arange(n, dtype=np.uint64) * frame
    blen = np.full(n, body, np.uint32)
    d_off = crc.DeviceBuffer(ctx, off.nbytes).upload(off)
    d_blen = crc.DeviceBuffer(ctx, blen.nbytes).upload(blen)
    ctx.write_packet_headers_device(img, d_off, d_blen, n, pcode=9, version=2, first_id=1)
    pd = np.zeros(n, crc.PACKET_DESC_DTYPE)
    pd["offset"], pd["len"] = off, frame
    d_pd = crc.DeviceBuffer(ctx, pd.nbytes).upload(pd)
    d_crc = crc.DeviceBuffer(ctx, 4 * n)
    d_st = crc.DeviceBuffer(ctx, 4 * n)
    d_bad = crc.DeviceBuffer(ctx, 4)
    ctx.packet_seal_device(d_pd, n, img, d_crc, d_st)
    ctx.sync()
    sealed = d_crc.download(np.uint32, n)
    # verify checks Func::crc(0, body) (seed 0, as for a FileInfo payload): its
    # expected values are the bodies' zero-seeded CRCs, computed on the device
    vd = np.zeros(n, crc.DESC_DTYPE)
    vd["offset"], vd["len"] = off + 24, body
    d_vd = crc.DeviceBuffer(ctx, vd.nbytes).upload(vd)
    d_z = crc.DeviceBuffer(ctx, 4 * n)
    ctx.batch_device(d_vd, n, img, d_z)
    ctx.sync()
    vd["aux"] = d_z.download(np.uint32, n)
    d_vd.upload(vd)
    d_ok = crc.DeviceBuffer(ctx, n)
    # every form agrees before timing: no bad frame, the same CRCs
    for name, c in (("one_pass", ctx), ("three", c3)):
        d_bad.zero()
        c.packet_verify_device(d_pd, n, img, d_crc, d_st, d_bad)
        c.sync()
        if int(d_bad.download(np.uint32)[0]) != 0 or not (d_crc.download(np.uint32, n) == sealed).all():
            raise SystemExit("ab_packet: %s disagrees" % name)
    d_bad.zero()
    ctx.verify_device(d_vd, n, img, None, d_ok, d_bad)
    ctx.sync()
    if int(d_bad.download(np.uint32)[0]) != 0:
        raise SystemExit("ab_packet: verify of the bodies disagrees")
    cases = {"one_pass": lambda: ctx.packet_verify_device(d_pd, n, img, d_crc, d_st, d_bad),
             "three": lambda: c3.packet_verify_device(d_pd, n, img, d_crc, d_st, d_bad),
             "verify": lambda: ctx.verify_device(d_vd, n, img, None, d_ok, d_bad)}
    owner = {"one_pass": ctx, "three": c3, "verify": ctx}
    times = {k: [] for k in cases}
    for r in range(rounds):
        for k, fn in cases.items():
            c = owner[k]
            fn()
            e0, e1 = crc.Event(c), crc.Event(c)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            c.sync()
            times[k].append(e0.elapsed_ms(e1) / reps)
        print("round %d done" % r, file=sys.stderr, flush=True)
    algo = float(n) * (frame + 16 + 4 + 4)
    res = {}
    for k, v in times.items():
        v = sorted(v)
        med = v[len(v) // 2]
        res[k] = {"median_ms": med, "min_ms": v[0], "max_ms": v[-1], "frac_8TBs": algo / (med / 1e3) / 1e9 / 8000.0}
    res["one_pass_over_verify"] = res["one_pass"]["median_ms"] / res["verify"]["median_ms"]
    res["three_over_verify"] = res["three"]["median_ms"] / res["verify"]["median_ms"]
    print(json.dumps({"tool": "ab_packet", "frames": n, "frame_bytes": frame, "rounds": rounds, "reps": reps,
                      "algo_bytes_per_launch": algo, "ab": res}))


if __name__ == "__main__":
    main()
