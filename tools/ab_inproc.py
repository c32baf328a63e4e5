#!/usr/bin/env python3
"""Same-process A/B of two builds of libtfs_crc.so on the headline workload
(measurement only).  Both libraries are loaded into one process (RTLD_LOCAL;
they share the HIP runtime and the device), the resident 1 M x 64 KiB block set
is built once with the product library, and verify passes of the two builds are
interleaved round by round, each timed with its own HIP events on its own
context's stream.  Process-to-process placement noise (+-3 % on this pool)
drops out.

  python tools/ab_inproc.py OTHER_SO[,OTHER_SO...] [ROUNDS] [mode]   mode: verify (default) | zipf

Two more entries: "product_nosplit" is the product library's SAME context with
file splitting switched off (tfs_crc32_set_split 0) for its rounds, so split on
vs off shares one stream and one scratch set and the per-context placement
noise (up to +-2 % between two contexts of one library) drops out of that pair.
(Round 3's "appended" split form was deleted in round 5.)  OTHER_SO "-" compares
only those.
AB_VARIANTS=v[,v...] adds measurement-build contexts running kernel variant v
(TFS_CRC_VARIANT) as entries "v<v>".
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import tfs_amd.crc as crc  # noqa: E402


def bind(path):
    L = ctypes.CDLL(path, mode=os.RTLD_LOCAL)
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    L.tfs_crc32_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.tfs_crc32_verify_device.argtypes = [vp, vp, u32, vp, vp, vp, vp, vp]
    L.tfs_crc32_batch_device.argtypes = [vp, vp, u32, vp, vp, vp]
    L.tfs_crc32_event_create.argtypes = [vp, ctypes.POINTER(vp)]
    L.tfs_crc32_event_record.argtypes = [vp, vp, vp]
    L.tfs_crc32_event_elapsed_ms.argtypes = [vp, vp, vp, ctypes.POINTER(ctypes.c_float)]
    L.tfs_crc32_sync.argtypes = [vp]
    h = vp()
    assert L.tfs_crc32_ctx_create(0, ctypes.byref(h)) == 0
    return L, h


def main():
    other = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    mode = sys.argv[3] if len(sys.argv) > 3 else "verify"
    ctx = crc.Context(0)
    prod = bind(crc.LIB_PATH)
    prod[0].tfs_crc32_set_split.argtypes = [ctypes.c_void_p, ctypes.c_int]
    libs = {"product": prod, "product_nosplit": prod}
    for i, o in enumerate(x for x in other.split(",") if x and x != "-"):
        libs["other%d" % i] = bind(os.path.abspath(o))
    if mode == "zipf":
        blocks = bench.zipf_sizes(42, 1024)
        offs, lens = [], []
        for b, L in enumerate(blocks):
            rec = np.concatenate([[0], np.cumsum(36 + L)[:-1]])
            offs.append(b * (64 << 20) + rec + 36)
            lens.append(L)
        offs = np.concatenate(offs).astype(np.uint64)
        lens = np.concatenate(lens).astype(np.uint32)
        n = len(lens)
        total = 1024 * (64 << 20) + 8192
        img = crc.DeviceBuffer(ctx, total)
        ctx.synth_fill_device(img, total, 0xC0FFEE, 0)
        d = np.zeros(n, crc.DESC_DTYPE)
        d["offset"], d["len"] = offs, lens
        algo = float(lens.astype(np.float64).sum()) + 21.0 * n
    else:
        n = 1024 * 1024
        rec = 65572
        total = n * rec
        img = crc.DeviceBuffer(ctx, (total + 4095) // 4096 * 4096)
        ctx.synth_fill_device(img, (total + 7) // 8 * 8, 0x9E3779B97F4A7C15, 0)
        d = np.zeros(n, crc.DESC_DTYPE)
        d["offset"] = np.arange(n, dtype=np.uint64) * rec + 36
        d["len"] = 65536
        algo = n * 65557.0
    d_desc = crc.DeviceBuffer(ctx, d.nbytes).upload(d)
    out = crc.DeviceBuffer(ctx, 4 * n)
    ctx.batch_device(d_desc, n, img, out)
    ctx.sync()
    d["aux"] = out.download(np.uint32)
    d_vdesc = crc.DeviceBuffer(ctx, d.nbytes).upload(d)
    ok = crc.DeviceBuffer(ctx, n)
    only = [x for x in os.environ.get("AB_ONLY", "").split(",") if x]  # e.g. AB_ONLY=product,product_ao
    if only:
        libs = {k: v for k, v in libs.items() if k in only}
    keep = []  # the variant contexts stay alive for the run
    for v in [int(x) for x in os.environ.get("AB_VARIANTS", "").split(",") if x]:
        os.environ["TFS_CRC_VARIANT"] = str(v)
        vc = crc.Context(0, measure=True)
        os.environ["TFS_CRC_VARIANT"] = "0"
        keep.append(vc)
        libs["v%d" % v] = (vc.L, vc.handle)
    times = {k: [] for k in libs}
    for r in range(rounds):
        for name, (L, h) in libs.items():
            if name in ("product", "product_nosplit"):  # split on / off (tfs_crc32_set_split)
                assert L.tfs_crc32_set_split(h, {"product": 1, "product_nosplit": 0}[name]) == 0
            e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
            L.tfs_crc32_event_create(h, ctypes.byref(e0))
            L.tfs_crc32_event_create(h, ctypes.byref(e1))
            if mode == "zipf":
                run = lambda: L.tfs_crc32_batch_device(h, d_desc.ptr, n, img.ptr, out.ptr, None)  # noqa: E731
            else:
                run = lambda: L.tfs_crc32_verify_device(h, d_vdesc.ptr, n, img.ptr, None, ok.ptr, None, None)  # noqa
            assert run() == 0
            L.tfs_crc32_event_record(h, e0, None)
            for _ in range(3):
                assert run() == 0
            L.tfs_crc32_event_record(h, e1, None)
            ms = ctypes.c_float()
            L.tfs_crc32_event_elapsed_ms(h, e0, e1, ctypes.byref(ms))
            times[name].append(ms.value / 3)
            if mode != "zipf":
                assert (ok.download(np.uint8, n) == 1).all(), name
    res = {}
    for k, v in times.items():
        v = sorted(v)
        res[k] = {"median_ms": v[len(v) // 2], "min_ms": v[0], "max_ms": v[-1],
                  "frac_at_median": algo / (v[len(v) // 2] / 1e3) / 1e9 / 8000.0}
    print(json.dumps({"mode": mode, "rounds": rounds, "other": other, "ab": res}))


if __name__ == "__main__":
    main()
