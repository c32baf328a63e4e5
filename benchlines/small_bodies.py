"""bench.py --workload small_bodies: per-call latency of the drop-in on small RPC
bodies.

A dataserver checks the CRC of every RPC body (BasePacket::decode,
src/common/base_packet.cpp:141; seed TFS_PACKET_FLAG_V1).  Most bodies are
small control messages; a lone frame decoded on its own goes through the scalar
drop-in tfs_crc32_e, which is one GPU round trip, while the
reference's byte loop (src/common/func.cpp:426-435) takes a few ns per byte on a
host core.  This line times, for bodies of 32 B .. 64 KiB:

  scalar_us   tfs_crc32_e on a pageable body (a lone frame), p50 / p99 over
              `iters` calls
  frame_us    tfs_packet_verify of one sealed V1 frame (the frame's own header
              check, host form), p50 / p99; called through ctypes with its
              descriptor and output arrays made once, as tfs_crc32_e is
  batch_us    tfs_packet_verify of 64 such frames in one call (one connection
              read, PacketDecoder), per frame at the p50 of the call
  cpu_us      the reference Func::crc (oracle/_ref, the reference's own text; or
              the oracle restatement) on one host core, per call, timed inside one C
              loop over 200,000 calls (no Python in the loop)

and reports the body size at which one GPU round trip costs as much as the
host loop (`crossover_bytes`).  Latencies include the ctypes call (~1 us of
Python per call, measured: `python_call_us`)."""
import ctypes
import os
import time

import numpy as np

from benchlines.common import *  # noqa: F401,F403
from benchlines.common import _ref_crc_fn

SIZES = (32, 80, 256, 1024, 4096, 16384, 65536)


def _pcts(us):
    us = np.sort(np.asarray(us))
    return {"p50": float(us[len(us) // 2]), "p99": float(us[min(len(us) - 1, int(0.99 * len(us)))]),
            "min": float(us[0])}


def bench_small_bodies(args):
    import tfs_amd.crc as crc
    from tfs_amd import packet as pk
    from tfs_amd.synth import synth_bytes
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    crc.lib().tfs_crc32_set_default_ctx(ctx.handle)
    iters = max(200, args.steps * 50)
    L = crc.lib()
    err = ctypes.c_int()
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_crc_batch_mt_fn.restype = ctypes.c_int
    ora.oracle_crc_batch_mt_fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int]
    fn, kind = _ref_crc_fn()
    # the ctypes overhead of one call that does nothing on the GPU (len 0 returns the seed)
    t0 = time.perf_counter()
    for _ in range(20000):
        L.tfs_crc32_e(7, b"", 0, ctypes.byref(err))
    py_us = (time.perf_counter() - t0) / 20000 * 1e6
    rows = {}
    for size in SIZES:
        body = synth_bytes(0x5B0D + size, size).tobytes()
        seed = pk.TFS_PACKET_FLAG_V1
        for _ in range(20):
            L.tfs_crc32_e(seed, body, size, ctypes.byref(err))
        us = []
        for _ in range(iters):
            a = time.perf_counter()
            c = L.tfs_crc32_e(seed, body, size, ctypes.byref(err))
            us.append((time.perf_counter() - a) * 1e6)
        if err.value != 0:
            raise SystemExit("small_bodies: tfs_crc32_e failed: %d" % err.value)
        # one sealed V1 frame, and a read of 64 of them
        frame = np.frombuffer(pk.frame_v1(body, pid=size, crc=int(c)), np.uint8).copy()

        def verify_call(buf, nfr):
            # tfs_packet_verify through ctypes on arrays made once (no numpy work per call)
            pd = np.zeros(nfr, crc.PACKET_DESC_DTYPE)
            pd["offset"], pd["len"] = np.arange(nfr) * frame.size, frame.size
            oc, os_, ob = np.zeros(nfr, np.uint32), np.zeros(nfr, np.int32), np.zeros(1, np.uint32)
            args = (ctx.handle, pd.ctypes.data, nfr, buf.ctypes.data, buf.size, oc.ctypes.data, os_.ctypes.data,
                    ob.ctypes.data)
            keep = (pd, oc, os_, ob, buf)  # the arrays the pointers name stay alive with the call

            def call(keep=keep):
                return L.tfs_packet_verify(*args)
            return call, os_, ob
        fcall, fst, fbad = verify_call(frame, 1)
        fus = []
        for _ in range(20):
            fcall()
        for _ in range(iters):
            a = time.perf_counter()
            rc = fcall()
            fus.append((time.perf_counter() - a) * 1e6)
        if fbad[0] or rc != 0 or fst[0] != 0:
            raise SystemExit("small_bodies: sealed frame failed to verify")
        read = np.tile(frame, 64)
        bcall, bst, bbad = verify_call(read, 64)
        bus = []
        for _ in range(max(50, iters // 4)):
            a = time.perf_counter()
            rc = bcall()
            bus.append((time.perf_counter() - a) * 1e6 / 64)
        if bbad[0] or rc != 0 or bst.any():
            raise SystemExit("small_bodies: batch failed to verify")
        # the reference byte loop on one core: 200,000 calls of this body inside one C loop
        ncall = 200000 if size <= 4096 else 20000
        buf = np.frombuffer(body, np.uint8).copy()
        d = np.zeros(ncall, crc.DESC_DTYPE)
        d["len"], d["aux"] = size, seed
        out = np.zeros(ncall, np.uint32)
        a = time.perf_counter()
        ora.oracle_crc_batch_mt_fn(fn, d.ctypes.data, ncall, buf.ctypes.data, out.ctypes.data, 1)
        cpu_us = (time.perf_counter() - a) / ncall * 1e6
        if not (out == np.uint32(c)).all():
            raise SystemExit("small_bodies: reference CRC differs from the GPU's")
        rows[str(size)] = {"scalar_us": _pcts(us), "frame_us": _pcts(fus), "batch_us_per_frame": _pcts(bus),
                           "cpu_us": cpu_us}
    # crossover: the body size at which the host loop (linear in size) costs as much as one
    # GPU call, the call's p50 interpolated linearly between the measured sizes (bodies of up
    # to 80 bytes ride in the resident ring's unit and cost less than the larger ones)
    per_byte = rows["65536"]["cpu_us"] / 65536
    cross = None
    for a, b in zip(SIZES, SIZES[1:]):
        ga, gb = rows[str(a)]["scalar_us"]["p50"], rows[str(b)]["scalar_us"]["p50"]
        da, db = per_byte * a - ga, per_byte * b - gb  # host minus GPU at both ends
        if da < 0 <= db:
            cross = int(a + (b - a) * (-da) / (db - da))
            break
    res = {
        "metric": "us per call, RPC body CRC (BasePacket::decode) through the drop-in, 32 B - 64 KiB bodies",
        "value": rows["4096"]["scalar_us"]["p50"], "unit": "us (p50, 4 KiB body, tfs_crc32_e)", "n_gpus": world,
        "steps": iters, "warmup": 20, "ms_per_step": rows["4096"]["scalar_us"]["p50"] / 1e3,
        "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic bodies, seed TFS_PACKET_FLAG_V1", "config": {"workload": "small RPC bodies", "sizes": SIZES},
        "sizes": rows, "python_call_us": py_us,
        "cpu_kind": kind, "cpu_ns_per_byte": per_byte * 1e3,
        "crossover_bytes": cross,
        # where the resident ring (and the bodies of up to 16 KiB) lived for these calls
        "resident_ring": {1: "device memory", 0: "host memory"}.get(ctx.resident_ring_in_device_memory(), "not set up"),
        "note": "scalar/frame/batch include ~python_call_us of ctypes per call; cpu_us is per call inside one C loop "
                "on one core.  Below crossover_bytes a lone body is cheaper on the host loop than one GPU round "
                "trip; batched reads (batch_us_per_frame) amortise the round trip over the frames of a read.",
    }
    emit(rank, res)
    crc.lib().tfs_crc32_set_default_ctx(None)
    ctx.close()
    if dist:
        dist.destroy_process_group()
