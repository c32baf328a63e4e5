"""bench.py --workload e2e."""


from benchlines.common import *  # noqa: F401,F403


def bench_e2e(args):
    """Verify-on-read starting in host memory: pinned block images -> (read over PCIe in place) ->
    verify -> verdicts back, several blocks in flight (submit/wait)."""
    import tfs_amd.crc as crc
    world, rank, local, dist = _dist_init()
    ctx = crc.Context(local)
    nsub, inflight = args.compact_blocks, 3
    cpu_res = {}

    def cpu(arr, offs, lens, exp):
        # the same verify of one page-locked block image on the host CPU
        cpu_res["v"] = cpu_baseline(arr, offs, lens, exp, args.cpu_seconds,
                                    "64 KiB payloads of a page-locked block image")
    gibs, pcie, el, ranks = e2e_blocks(ctx, dist, world, rank, nsub, inflight,
                                       cpu if rank == 0 and not args.no_cpu else None)
    res = {
        "metric": "GiB/s CRC32 verify end-to-end from pinned host block images (H2D included)",
        "value": gibs, "unit": "GiB/s", "n_gpus": world, "steps": nsub, "warmup": 2,
        "ms_per_step": el / nsub * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic 64 KiB files, 1024 per 64 MiB block",
        "config": {"workload": "pinned host blocks -> GPU verify, %d in flight, %d blocks" % (inflight, nsub)},
        "pcie_GBs": pcie,
        "per_rank": ranks,
    }
    ceil = pcie_ceiling(ctx, dist=dist)
    res["roofline"] = {"bound": "pcie", "achieved": pcie / world, "peak": ceil["h2d_GBs"], "unit": "GB/s (per GPU)",
                       "frac": pcie / world / ceil["h2d_GBs"], "peak_source": ceil["source"], "traffic": None}
    if "v" in cpu_res:
        res["cpu_baseline"] = cpu_res["v"]
    if dist and not args.no_cpu:
        dist.barrier()
    emit(rank, res)
    ctx.close()
    if dist:
        dist.destroy_process_group()

