#!/usr/bin/env python3
"""Same-process A/B of the device compaction kernel (measurement
only).  Builds bench.py's compact_device workload once (1,024 resident blocks,
341 of every 1,024 records live, one job per live record), then interleaves, round
by round, launches of

  * kernel variants on the packed destination (AB_VARIANTS: 26 the product
    without its payload CRC steps; 67 / 68 the record list through the chunk
    copy's loop, dynamic / static order; 94-99 the round-5 occupancy forms), and
  * the product kernel on destinations congruent to the source mod 128 (whole
    destination lines per stripe),

each timed with HIP events on its own context's stream.  The streaming-copy
ceilings of the same bytes (membench 52114 grid-stride, 53104/53116/53004/53016
wave-contiguous chunks) are timed in the same rounds.  Verify-on-read of every
resident record (tfs_blocks_verify_device) is timed for the product.

  python tools/ab_compact.py [ROUNDS] [NBLOCKS]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import tfs_amd.crc as crc  # noqa: E402


def ctx_for(variant):
    os.environ["TFS_CRC_VARIANT"] = str(variant)
    c = crc.Context(0, measure=True)  # variants: measurement build
    os.environ["TFS_CRC_VARIANT"] = "0"
    return c


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    nblocks = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    ctx = crc.Context(0, measure=True)  # calibration kernels: measurement build
    nfiles, rec = bench.FILES_PER_BLOCK, bench.FILEINFO + bench.FILE_SIZE
    blk = nfiles * rec
    total = nblocks * blk
    img = crc.DeviceBuffer(ctx, (total + 4095) // 4096 * 4096)
    ctx.synth_fill_device(img, (total + 7) // 8 * 8, 0xC0DE, 0)
    n = nblocks * nfiles
    desc = np.zeros(n, crc.DESC_DTYPE)
    rec_off = np.arange(n, dtype=np.uint64) * rec
    desc["offset"], desc["len"] = rec_off + bench.FILEINFO, bench.FILE_SIZE
    d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
    d_crc = crc.DeviceBuffer(ctx, 4 * n)
    ctx.batch_device(d_desc, n, img, d_crc)
    d_roff = crc.DeviceBuffer(ctx, rec_off.nbytes).upload(rec_off)
    d_len = crc.DeviceBuffer(ctx, 4 * n).upload(np.full(n, bench.FILE_SIZE, np.uint32))
    ctx.write_headers_device(img, d_roff, d_len, d_crc, 1, n)
    ctx.sync()
    for b in (d_desc, d_roff, d_len, d_crc):
        b.free()
    # AB_LIVE=all: every record live (a dense source, the copy's read shape)
    live1 = (np.arange(nfiles) if os.environ.get("AB_LIVE") == "all"
             else np.nonzero(bench._fragmented_flags(nfiles) == 0)[0])
    nl = live1.size
    bidx = np.repeat(np.arange(nblocks, dtype=np.uint64), nl)
    soff = bidx * blk + np.tile(live1.astype(np.uint64) * rec, nblocks)
    k = np.arange(nblocks * nl, dtype=np.uint64)
    # AB_ALIGNED=1 adds "aligned64k": the same number of jobs over a dense, 64 KiB-aligned
    # record list (src = dest = j * 65,536, size 65,536) -- the dense copy's own layout
    # through the record kernel (timing only: the FileInfo checks fail)
    dsts = {"packed": k * rec,                                   # the product workload (contiguous new blocks)
            "dst128": k * 65664 + (soff & np.uint64(127))}       # delta == 0 mod 128: whole lines per stripe
    d_dst = crc.DeviceBuffer(ctx, int(k.size) * 65664 + 256)
    d_bad = crc.DeviceBuffer(ctx, 4)
    jobsets = {}
    for name, do in dsts.items():
        j = np.zeros(k.size, crc.COMPACT_JOB_DTYPE)
        j["src_offset"], j["dest_offset"] = soff, do
        j["file_id"] = 1 + bidx * nfiles + np.tile(live1.astype(np.uint64), nblocks)
        j["size"] = rec
        j["new_offset"] = (do % np.uint64(1 << 31)).astype(np.int32)
        jobsets[name] = crc.DeviceBuffer(ctx, j.nbytes).upload(j)
    # AB_PARTS=1: the product on the first half and the first quarter of the packed job
    # list too (same buffers, one launch each): a fixed per-launch cost shows as a
    # higher time per record in the shorter launches
    parts = {}
    if os.environ.get("AB_PARTS"):
        for nm, den in (("half", 2), ("quarter", 4)):
            parts[nm] = int(k.size) // den
    if os.environ.get("AB_ALIGNED"):
        j = np.zeros(k.size, crc.COMPACT_JOB_DTYPE)
        j["src_offset"] = j["dest_offset"] = k * np.uint64(65536)
        j["file_id"], j["size"] = 1, 65536
        jobsets["aligned64k"] = crc.DeviceBuffer(ctx, j.nbytes).upload(j)
    want = [int(x) for x in os.environ.get("AB_VARIANTS", "26,68").split(",") if x]
    ctxs = {0: ctx}
    for v in want:
        ctxs[v] = ctx_for(v)
    # 67/68: the record list through the chunk copy's loop -- destinations congruent mod 128 only
    cases = ([(0, "packed")] + [(v, "packed") for v in want if v not in (67, 68)] + [(0, "dst128")] +
             [(v, "dst128") for v in want if v in (67, 68)])
    if os.environ.get("AB_ALIGNED"):
        # every requested variant on the dense layout too: where the kernel trails
        # the chunk copy of the same layout
        cases += [(0, "aligned64k")] + [(v, "aligned64k") for v in want]
    cases += [(0, nm) for nm in parts]
    # AB_SEG=S[,S...]: the segmented compaction (tfs_crc32_set_compact_segment) on the
    # product context itself, toggled around its rounds (no second context's placement);
    # the other cases run it with whole records (set_compact_segment 0)
    segs = [int(x) for x in os.environ.get("AB_SEG", "").split(",") if x]
    cases += [("seg%d" % S, "packed") for S in segs]
    d_st = crc.DeviceBuffer(ctx, 4 * max([int(k.size)] + [getattr(b, "njobs", 0) for b in jobsets.values()]))
    # verify-on-read of every record of the resident blocks (tfs_blocks_verify_device)
    allj = np.zeros(n, crc.COMPACT_JOB_DTYPE)
    allj["src_offset"], allj["file_id"], allj["size"] = rec_off, 1 + np.arange(n, dtype=np.uint64), rec
    d_allj = crc.DeviceBuffer(ctx, allj.nbytes).upload(allj)
    d_vst = crc.DeviceBuffer(ctx, 4 * n)
    vcases = [0] + [v for v in want if v == 50]
    nj = int(k.size)
    live_bytes = float(nj) * rec
    algo = 2 * live_bytes + nj * (40 + 4)
    # correctness of the product cases (the diagnostic variants 26 and 30 compute
    # no CRCs / skip stores)
    def ctx_of(v):
        if isinstance(v, str):
            ctx.set_compact_segment(int(v[3:]))
            return ctx
        ctx.set_compact_segment(0)
        return ctxs[v]

    for v, js in cases:
        if v in (26, 67, 68) or js == "aligned64k" or js in parts:
            continue
        d_bad.zero()
        c = ctx_of(v)
        c.compact_jobs_device(img, total, jobsets[js], nj, d_dst, None, d_st, d_bad)
        c.sync()
        if int(d_bad.download(np.uint32, 1)[0]) != 0:
            raise SystemExit("ab_compact: variant %s on %s reports bad records" % (v, js))
    times = {"%s_%s" % c: [] for c in cases}
    times["copy_52114"] = []
    # wave-contiguous chunks: nt / plain stores, 64 / 256 KiB (256 workgroups); AB_COPIES
    # adds "pattern:grid[:dskew[:sskew]]" (e.g. 52114:8192, the grid-stride copy over 8,192
    # workgroups; skews: bytes added to the destination / source pointers, multiples of 16)
    copies = [(53104, 0, 0, 0), (53116, 0, 0, 0), (53004, 0, 0, 0), (53016, 0, 0, 0)]
    for x in os.environ.get("AB_COPIES", "").split(","):
        if x:
            pg = [int(v) for v in x.split(":")] + [0, 0, 0]
            copies.append(tuple(pg[:4]))

    def cname(pat, grid, dsk, ssk):
        return "copy_%d%s%s%s" % (pat, "_g%d" % grid if grid else "", "_d%d" % dsk if dsk else "",
                                  "_s%d" % ssk if ssk else "")
    for c in copies:
        times[cname(*c)] = []
    for v in vcases:
        d_bad.zero()
        ctxs[v].blocks_verify_device(img, total, d_allj, n, None, d_vst, d_bad)
        ctxs[v].sync()
        if int(d_bad.download(np.uint32, 1)[0]) != 0:
            raise SystemExit("ab_compact: verify variant %d reports bad records" % v)
        times["verify_%d" % v] = []
    cb = int(live_bytes) // 16 * 16
    reps = int(os.environ.get("AB_REPS", "3"))  # back-to-back launches per timing (sustained load: 16)
    for r in range(rounds):
        for v, js in cases:
            c = ctx_of(v)
            e0, e1 = crc.Event(c), crc.Event(c)
            nn = parts.get(js, getattr(jobsets.get(js), "njobs", nj))
            jb = jobsets["packed"] if js in parts else jobsets[js]
            c.compact_jobs_device(img, total, jb, nn, d_dst, None, d_st, d_bad)
            e0.record()
            for _ in range(reps):
                c.compact_jobs_device(img, total, jb, nn, d_dst, None, d_st, d_bad)
            e1.record()
            c.sync()
            times["%s_%s" % (v, js)].append(e0.elapsed_ms(e1) / reps)
        ctx.set_compact_segment(0)
        for v in vcases:
            c = ctxs[v]
            e0, e1 = crc.Event(c), crc.Event(c)
            c.blocks_verify_device(img, total, d_allj, n, None, d_vst, d_bad)
            e0.record()
            for _ in range(3):
                c.blocks_verify_device(img, total, d_allj, n, None, d_vst, d_bad)
            e1.record()
            c.sync()
            times["verify_%d" % v].append(e0.elapsed_ms(e1) / 3)
        e0, e1 = crc.Event(ctx), crc.Event(ctx)
        ctx.membench_device(52114, img, None, 0, cb, d_dst)
        e0.record()
        for _ in range(3):
            ctx.membench_device(52114, img, None, 0, cb, d_dst)
        e1.record()
        ctx.sync()
        times["copy_52114"].append(e0.elapsed_ms(e1) / 3)
        for pat, grid, dsk, ssk in copies:
            e0, e1 = crc.Event(ctx), crc.Event(ctx)
            nb = cb - max(dsk, ssk) // 16 * 16
            ctx.membench_device(pat, img.ptr + ssk, None, 0, nb, d_dst.ptr + dsk, grid=grid)
            e0.record()
            for _ in range(reps):
                ctx.membench_device(pat, img.ptr + ssk, None, 0, nb, d_dst.ptr + dsk, grid=grid)
            e1.record()
            ctx.sync()
            times[cname(pat, grid, dsk, ssk)].append(e0.elapsed_ms(e1) / reps * cb / nb)
        print("round %d done" % r, file=sys.stderr, flush=True)
    res = {}
    for name, v in times.items():
        v = sorted(v)
        med = v[len(v) // 2]
        by = 2.0 * cb if name.startswith("copy") else (n * (rec + 40 + 8) if name.startswith("verify") else algo)
        for nm, cnt in parts.items():
            if name == "0_" + nm:
                by = algo * cnt / nj
        res[name] = {"median_ms": med, "min_ms": v[0], "max_ms": v[-1], "GBs": by / (med / 1e3) / 1e9,
                     "frac_8TBs": by / (med / 1e3) / 1e9 / 8000.0}
    print(json.dumps({"tool": "ab_compact", "rounds": rounds, "nblocks": nblocks, "records": nj,
                      "algo_bytes": algo, "ab": res}))


if __name__ == "__main__":
    main()
