"""bench.py --workload packet."""
import ctypes
import os
import time

import numpy as np

from benchlines.common import *  # noqa: F401,F403


def bench_packet(args):
    """Receive-side packet CRC (BasePacket::decode, base_packet.cpp:117-148) over
    device-resident V1 frames carrying 64 KiB WriteDataMessages.
    Frames are sealed on the device first (the send side), then decoded K times."""
    import tfs_amd.crc as crc
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    # WriteDataMessage body: WriteDataInfo 32 B | vint64 ds_ (3 servers + lease triple: 4 + 6*8) | 64 KiB data
    body = 32 + 4 + 6 * 8 + FILE_SIZE
    frame = 24 + body
    n = args.blocks * FILES_PER_BLOCK
    total = n * frame
    img = crc.DeviceBuffer(ctx, (total + 4095) // 4096 * 4096)
    ctx.synth_fill_device(img, (total + 7) // 8 * 8, 0x5EED + rank, 0)
    off = np.arange(n, dtype=np.uint64) * frame
    blen = np.full(n, body, np.uint32)
    d_off = crc.DeviceBuffer(ctx, off.nbytes).upload(off)
    d_blen = crc.DeviceBuffer(ctx, blen.nbytes).upload(blen)
    ctx.write_packet_headers_device(img, d_off, d_blen, n, pcode=9, version=2, first_id=1 + rank * n)
    pd = np.zeros(n, crc.PACKET_DESC_DTYPE)
    pd["offset"], pd["len"] = off, frame
    d_pd = crc.DeviceBuffer(ctx, pd.nbytes).upload(pd)
    d_crc = crc.DeviceBuffer(ctx, 4 * n)
    d_st = crc.DeviceBuffer(ctx, 4 * n)
    d_bad = crc.DeviceBuffer(ctx, 4)
    ctx.packet_seal_device(d_pd, n, img, d_crc, d_st)  # send side: header crc_ = Func::crc(FLAG_V1, body)
    d_bad.zero()
    for _ in range(max(1, args.warmup)):
        ctx.packet_verify_device(d_pd, n, img, d_crc, d_st, d_bad)
    ctx.sync()
    if int(d_bad.download(np.uint32, 1)[0]) != 0:
        raise SystemExit("packet: sealed frames failed to verify")
    # parity spot check against the oracle (test infrastructure)
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_crc.restype = ctypes.c_uint32
    ora.oracle_crc.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int32]
    got = d_crc.download(np.uint32, n)
    for i in np.linspace(0, n - 1, 24).astype(np.int64):
        b = img.download(np.uint8, body, int(off[i]) + 24).tobytes()
        if ora.oracle_crc(0x4E534654, b, body) != int(got[i]):
            raise SystemExit("packet: GPU CRC disagrees with oracle at frame %d" % i)
    ev = [(crc.Event(ctx), crc.Event(ctx)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record()
        ctx.packet_verify_device(d_pd, n, img, d_crc, d_st, d_bad)
        ev[k][1].record()
    ctx.sync()
    if dist:
        dist.barrier()
    el = _max_over_ranks(dist, time.perf_counter() - t0)
    kms = float(np.mean([a.elapsed_ms(b) for a, b in ev]))
    # algorithmic bytes per frame of the one-pass decode (packet_files_kernel, round 5):
    # the frame (24-B header + body) and its 16-B PacketDesc read, the 4-B crc and
    # 4-B status written; the wave that checksums the body parses the header itself.
    algo = n * (float(frame) + 16 + 4 + 4)
    p_traffic, p_src = _pmc_traffic("profiles/r06/pmc/packet/pmc_summary.json", PACKET_KERNEL, n == 1048576)
    res = {
        "metric": "GiB/s packet bytes CRC-verified (BasePacket::decode), device-resident V1 frames",
        "value": world * args.steps * n * frame / el / 2**30, "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64) WriteDataMessage bodies, headers sealed on the GPU",
        "config": {"workload": "SURVEY §8 f1: %d V1 frames x %d B (64 KiB write + message fields)" % (n, frame),
                   "frames_per_gpu": n},
        "roofline": {"bound": "hbm", "achieved": algo / (kms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": algo / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, "traffic": p_traffic,
                     "traffic_source": p_src, "traffic_measured_in_this_run": False, "traffic_note": TRAFFIC_NOTE, "algorithmic_bytes_per_launch": algo,
                     "kernel": "packet_files_kernel<1> (one pass: header parse + body CRC + status)", "kernel_ms_avg": kms,
                     "kernel_ms_min": float(min(a.elapsed_ms(b) for a, b in ev))},
    }
    if rank == 0 and not args.no_cpu:
        # BasePacket::decode's CRC on the host: Func::crc(TFS_PACKET_FLAG_V1, body) over sampled bodies
        idx = np.linspace(0, n - 1, min(n, 1024)).astype(np.int64)
        sample = np.zeros(len(idx) * body, np.uint8)
        for j, i in enumerate(idx):
            sample[j * body:(j + 1) * body] = img.download(np.uint8, body, int(off[i]) + 24)
        cb = cpu_baseline(sample, np.arange(len(idx)) * body, np.full(len(idx), body), got[idx],
                          args.cpu_seconds, "%d-B WriteDataMessage bodies" % body, seed=0x4E534654)
        cb["unit"] = "GiB/s of body bytes"
        res["cpu_baseline"] = cb
    if dist and not args.no_cpu:
        dist.barrier()
    emit(rank, res)
    del ev
    for b in (img, d_off, d_blen, d_pd, d_crc, d_st, d_bad):
        b.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()

