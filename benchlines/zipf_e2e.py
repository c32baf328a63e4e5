"""bench.py --workload zipf_e2e, and the `end_to_end` leg of --workload zipf:
BASELINE configs[2]'s compute-on-write path starting in host memory.

The write path's bytes arrive in the dataserver's socket receive buffer
(dataservice.cpp:1182-1287, write_data_message.cpp:44-49) and are checksummed at
close (DataFile::get_crc via DataManagement::close_write_file,
data_file.cpp:183-190, data_management.cpp:197).  Here a receive buffer is a
page-locked 64 MiB host region holding one 64 MiB block's worth of Zipf-sized
payloads (zipf_sizes: 4 KiB-1 MiB, most bytes in files over the 128 KiB split
size) at arbitrary byte offsets (a random 0-127 byte gap before each payload, the
framing between messages).  Each buffer is one tfs_crc32_batch call (the wide
in-place path: the throughput kernel reads the payloads over PCIe where they lie,
descriptors and CRCs in the slot's page-locked words, split plan for the long
files); `inflight` dataserver threads each issue their own calls, so that many
batches are in flight on the context.
"""
import ctypes
import os
import threading
import time

import numpy as np

from benchlines.common import *  # noqa: F401,F403

RECV_GAP = 128  # payload i starts after a U[0, 128) byte gap (message framing): arbitrary alignment


def recv_buffers(ctx, nbuf, seed):
    """nbuf page-locked receive buffers: [(pinned, desc, payload bytes, span bytes)], filled
    with the splitmix64 stream on the device and copied down."""
    import tfs_amd.crc as crc
    blocks = zipf_sizes(seed, nbuf)
    rng = np.random.default_rng(seed + 7)
    out = []
    lay = []
    for L in blocks:
        gap = rng.integers(0, RECV_GAP, L.size)
        offs = np.cumsum(gap) + np.concatenate([[0], np.cumsum(L)[:-1]])
        span = int(offs[-1] + L[-1])
        lay.append((offs, L, span))
    big = max(s for _, _, s in lay)
    d = crc.DeviceBuffer(ctx, (big + 4095) // 4096 * 4096)
    for b, (offs, L, span) in enumerate(lay):
        nb = (span + 7) // 8 * 8
        ctx.synth_fill_device(d, nb, 0x2EC0 + seed * 131 + b, 0)
        ctx.sync()
        p = crc.PinnedBuffer(ctx, nb)
        ctx._check(ctx.L.tfs_crc32_memcpy(ctx.handle, p.ptr, d.ptr, nb, None), "memcpy")
        desc = np.zeros(L.size, crc.DESC_DTYPE)
        desc["offset"], desc["len"] = offs, L
        out.append((p, desc, float(L.sum()), span))
    d.free()
    return out


def oracle_crcs(bufs):
    """Test infrastructure: every distinct buffer's CRCs from the oracle (pthreads)."""
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle_crc.so"))
    ora.oracle_crc_batch_mt.restype = ctypes.c_int
    ora.oracle_crc_batch_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int]
    exp = []
    for p, desc, _, _ in bufs:
        e = np.zeros(desc.size, np.uint32)
        if ora.oracle_crc_batch_mt(desc.ctypes.data, desc.size, p.ptr, e.ctypes.data, _cpu_budget(shared=True)):
            raise SystemExit("zipf_e2e: oracle failed")
        exp.append(e)
    return exp


def zipf_e2e_leg(ctx, dist, world, rank, nsub, inflight=3, ndistinct=16, seed=4242):
    """Time nsub receive-buffer checksums (tfs_crc32_batch, `inflight` threads) between
    barriers, max over ranks.  Every submission's CRCs are compared with the oracle's
    for its buffer.  Returns the `end_to_end` dict."""
    bufs = recv_buffers(ctx, ndistinct, seed + rank)
    exp = oracle_crcs(bufs)
    L = ctx.L
    fn = L.tfs_crc32_batch
    order = [i % ndistinct for i in range(nsub)]
    outs = [np.zeros(bufs[i][1].size, np.uint32) for i in order]
    errs = []

    def worker(t, go, idx):
        go.wait()
        for k in idx:
            p, desc, _, span = bufs[order[k]]
            rc = fn(ctx.handle, desc.ctypes.data, desc.size, p.ptr, span, outs[k].ctypes.data)
            if rc != 0:
                errs.append((k, rc))
                return

    def run(idx_sets):
        go = threading.Barrier(len(idx_sets) + 1)
        ts = [threading.Thread(target=worker, args=(t, go, idx)) for t, idx in enumerate(idx_sets)]
        for t in ts:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in ts:
            t.join()
        return time.perf_counter() - t0

    # warmup: every distinct buffer once through `inflight` threads (slots, plans, streams)
    run([list(range(t, ndistinct, inflight)) for t in range(inflight)])
    if dist:
        dist.barrier()
    el_local = run([list(range(t, nsub, inflight)) for t in range(inflight)])
    el = _max_over_ranks(dist, el_local)
    if errs:
        raise SystemExit("zipf_e2e: tfs_crc32_batch failed: %s (%s)" % (
            errs[:4], L.tfs_crc32_last_error(ctx.handle).decode()))
    mism = sum(int((outs[k] != exp[order[k]]).sum()) for k in range(nsub))
    files = sum(bufs[order[k]][1].size for k in range(nsub))
    if mism:
        raise SystemExit("zipf_e2e: %d of %d CRCs disagree with the oracle" % (mism, files))
    payload = sum(bufs[order[k]][2] for k in range(nsub))
    nfiles = sum(b[1].size for b in bufs)
    big = sum(int((b[1]["len"] > 131072).sum()) for b in bufs)
    big_bytes = sum(float(b[1]["len"][b[1]["len"] > 131072].sum()) for b in bufs)
    ceil = pcie_ceiling(ctx, dist=dist)
    pcie = float(world) * payload / el / 1e9
    ranks = {"payload_GiBs": per_rank(dist, world, el_local, payload),
             "pcie_GBs": per_rank(dist, world, el_local, payload, 1e9)}
    for b in bufs:
        b[0].free()
    return {
        "value": float(world) * payload / el / 2**30, "unit": "GiB/s", "pcie_GBs": pcie,
        "ms_per_buffer": el / nsub * 1e3, "n_buffers": nsub, "inflight": inflight,
        "workload": "%d page-locked 64 MiB receive buffers per GPU (%d distinct, cycled), each one block of Zipf "
                    "payloads (%d files in the %d distinct buffers, mean %.1f KiB, %d files > 128 KiB holding "
                    "%.0f%% of the bytes) at arbitrary byte offsets (U[0,%d) gaps); one tfs_crc32_batch per "
                    "buffer (wide in-place path: payloads read over PCIe where they lie), %d caller threads" % (
                        nsub, ndistinct, nfiles, ndistinct, sum(b[2] for b in bufs) / nfiles / 1024, big,
                        100.0 * big_bytes / sum(b[2] for b in bufs), RECV_GAP, inflight),
        "distinct_note": "%d distinct buffers (%d MiB of page-locked host memory per GPU) are cycled: every byte "
                         "still crosses PCIe on every call (the GPU holds no copy of a receive buffer), and the "
                         "set is far above every GPU cache" % (ndistinct, sum(b[3] for b in bufs) >> 20),
        "per_rank": ranks,
        "parity": {"files_checked": files, "mismatches": mism,
                   "method": "every submission's CRCs against the oracle's CRCs of its buffer (pthreads, computed "
                             "once per distinct buffer over the page-locked bytes)"},
        "roofline": {"bound": "pcie", "achieved": pcie / world, "peak": ceil["h2d_GBs"], "unit": "GB/s (per GPU)",
                     "frac": pcie / world / ceil["h2d_GBs"], "peak_source": ceil["source"],
                     "traffic": "payload bytes host->device (descriptors 16 B and CRCs 4 B per file besides)"},
    }


def bench_zipf_e2e(args):
    """The configs[2] compute-on-write path from host memory, as its own line."""
    import tfs_amd.crc as crc
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    nsub = args.e2e_blocks if args.e2e_blocks > 0 else 128
    leg = zipf_e2e_leg(ctx, dist, world, rank, nsub)
    res = {
        "metric": "GiB/s CRC32 compute-on-write from page-locked receive buffers (PCIe included), Zipf files",
        "value": leg["value"], "unit": "GiB/s", "n_gpus": world, "steps": nsub, "warmup": 16,
        "ms_per_step": leg["ms_per_buffer"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (splitmix64), Zipf(1.1) k in 1..255, len = 4096k + U[0,4095]",
        "config": {"workload": "BASELINE configs[2] from host memory: " + leg["workload"]},
        "pcie_GBs": leg["pcie_GBs"], "per_rank": leg["per_rank"], "parity": leg["parity"],
        "roofline": leg["roofline"], "distinct_note": leg["distinct_note"],
    }
    emit(rank, res)
    ctx.close()
    if dist:
        dist.destroy_process_group()
