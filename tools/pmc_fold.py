#!/usr/bin/env python3
"""Fold the counter passes of tools/pmc_passes.sh into one summary per kernel
(measurement only).

  python tools/pmc_fold.py PASSDIR [--bytes B] [--kernel SUBSTR] [--out JSON]

PASSDIR is OUTDIR/NAME of pmc_passes.sh (trace/ + pmc_<group>/ subdirectories).
For every kernel whose name contains SUBSTR: the median of each counter over its
dispatches, the kernel-trace average duration, and derived ratios -- the share
of wave time issuing / waiting, instructions per KiB of algorithmic bytes (B per
launch), translation misses per MiB, write requests that are full 64 B, DRAM
credit stalls per cycle.  HBM bytes use the gfx950 correction of
MI355X_MICROARCH.md (FETCH_SIZE x 2; TCC_EA0_RDREQ x 128 B cross-check).
"""
import argparse
import csv
import glob
import json
import os
import statistics


def short(name):
    n = name[5:] if name.startswith("void ") else name
    return n.split("(")[0].replace("tfscrc::", "").replace("tfsec::", "")


def load(passdir, sub):
    per = {}
    for f in glob.glob(os.path.join(passdir, "pmc_*", "*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                if sub and sub not in k:
                    continue
                per.setdefault(k, {}).setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"] + f, 0.0)
                per[k][r["Counter_Name"]][r["Dispatch_Id"] + f] += float(r["Counter_Value"])
    out = {}
    for k, cs in per.items():
        out[k] = {c: statistics.median(v.values()) for c, v in cs.items()}
    return out


def trace_ms(passdir, sub):
    res = {}
    for f in glob.glob(os.path.join(passdir, "trace", "*kernel_stats.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Name"])
                if not sub or sub in k:
                    res[k] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                              "min_ms": float(r["MinNs"]) / 1e6}
    return res


def derive(c, algo):
    d = {}
    g = lambda k: c.get(k)  # noqa: E731
    if g("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM"):
            if g(k) is not None:
                d[k.lower() + "_per_wave_cycle"] = g(k) / g("SQ_WAVE_CYCLES")
    if g("GRBM_GUI_ACTIVE") and g("SQ_BUSY_CYCLES"):
        d["sq_busy_per_gui_cycle"] = g("SQ_BUSY_CYCLES") / g("GRBM_GUI_ACTIVE")
    if algo:
        kib = algo / 1024.0
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU",
                  "SQ_INSTS_SMEM", "SQ_LDS_BANK_CONFLICT"):
            if g(k) is not None:
                d[k.lower() + "_per_KiB"] = g(k) / kib
        if g("TCP_UTCL1_TRANSLATION_MISS_sum") is not None:
            d["utcl1_miss_per_MiB"] = g("TCP_UTCL1_TRANSLATION_MISS_sum") / (algo / 2**20)
    if g("FETCH_SIZE") is not None:
        d["read_bytes_corrected"] = g("FETCH_SIZE") * 1024.0 * 2.0
    if g("TCC_EA0_RDREQ_sum"):
        d["read_bytes_rdreq_x128"] = g("TCC_EA0_RDREQ_sum") * 128.0
        if g("TCC_EA0_RDREQ_DRAM_sum") is not None:
            d["rdreq_dram_share"] = g("TCC_EA0_RDREQ_DRAM_sum") / g("TCC_EA0_RDREQ_sum")
    if g("WRITE_SIZE") is not None:
        d["write_bytes"] = g("WRITE_SIZE") * 1024.0
    if g("TCC_EA0_WRREQ_sum"):
        d["wrreq_64B_share"] = (g("TCC_EA0_WRREQ_64B_sum") or 0.0) / g("TCC_EA0_WRREQ_sum")
    if algo and "read_bytes_corrected" in d:
        d["traffic_over_algorithmic"] = (d["read_bytes_corrected"] + d.get("write_bytes", 0.0)) / algo
    gui = g("GRBM_GUI_ACTIVE")
    if gui:
        for k in ("TCP_PENDING_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum", "TCC_EA0_WRREQ_STALL_sum",
                  "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum", "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "TCC_BUSY_sum"):
            if g(k) is not None:
                d[k.lower() + "_per_gui_cycle"] = g(k) / gui
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("passdir")
    ap.add_argument("--bytes", type=float, default=0.0, help="algorithmic bytes per launch")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--out")
    a = ap.parse_args()
    cnt = load(a.passdir, a.kernel)
    tr = trace_ms(a.passdir, a.kernel)
    res = {"source": a.passdir, "algorithmic_bytes_per_launch": a.bytes or None, "kernels": {}}
    for k, c in cnt.items():
        res["kernels"][k] = {"trace": tr.get(k), "counters_median": c, "derived": derive(c, a.bytes)}
    s = json.dumps(res, indent=1)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as fh:
            fh.write(s)
    print(s)


if __name__ == "__main__":
    main()
