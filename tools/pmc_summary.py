#!/usr/bin/env python3
"""tools/pmc_summary.py TAG -- summarise gpurun_out/prof_TAG into profiles/TAG/
(kernel stats csv, per-counter medians for the verify kernel, corrected HBM
traffic per launch) and point profiles/pmc_latest.json at it."""
import collections
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
dst = os.path.join(ROOT, "profiles", tag)
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
bench_line = open(os.path.join(src, "bench_trace.json")).read().strip().splitlines()[-1]
open(os.path.join(dst, "bench_under_rocprof.json"), "w").write(bench_line + "\n")
vals = collections.defaultdict(list)
kname = None
for f in glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv")):
    grp = os.path.basename(os.path.dirname(f))
    shutil.copy(f, os.path.join(dst, grp + ".csv"))
    for r in csv.DictReader(open(f)):
        if "crc_files_kernel<1" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            kname = r["Kernel_Name"].split("(")[0]
med = {k: statistics.median(v) for k, v in vals.items()}
stats = {}
for r in csv.DictReader(open(os.path.join(dst, "kernel_stats.csv"))):
    if "crc_files_kernel<1" in r["Name"]:
        stats = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                 "max_ns": float(r["MaxNs"])}
nfiles = 1048576
algo = nfiles * (65536 + 21)
rd = med.get("FETCH_SIZE", 0.0) * 1024 * 2
wr = med.get("WRITE_SIZE", 0.0) * 1024
summ = {
    "kernel": kname, "tag": tag,
    "launch_work": "1,048,576 files x 64 KiB payload (block images, FileInfo|payload)",
    "rocprof_kernel_stats": stats,
    "counters_median": med,
    "read_bytes_corrected": rd,
    "read_bytes_from_rdreq_x128": med.get("TCC_EA0_RDREQ_sum", 0.0) * 128,
    "write_bytes": wr,
    "traffic_bytes_per_launch": rd + wr,
    "algorithmic_bytes_per_launch": algo,
    "traffic_over_algorithmic": (rd + wr) / algo if rd else None,
    "achieved_GBs_algorithmic_at_rocprof_avg": algo / (stats["avg_ns"] * 1e-9) / 1e9 if stats else None,
    "correction": "gfx950 FETCH_SIZE reports half the bytes of a wide coalesced stream (MI355X_MICROARCH.md §HBM): x2; "
                  "cross-checked by TCC_EA0_RDREQ x 128 B",
    "effective_clock_GHz": med["GRBM_GUI_ACTIVE"] / 8 / (stats["avg_ns"] * 1e-9) / 1e9
    if stats and "GRBM_GUI_ACTIVE" in med else None,
}
json.dump(summ, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
json.dump(dict(summ, source="profiles/%s/pmc_summary.json" % tag),
          open(os.path.join(ROOT, "profiles", "pmc_latest.json"), "w"), indent=1)
print(json.dumps(summ, indent=1))
