#!/usr/bin/env python3
"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes of a multi-kernel step (the
packet decode pipeline: parse + CRC + finish) into one summary: per-kernel
medians summed, with the gfx950 FETCH_SIZE x2 correction (MI355X_MICROARCH.md
§HBM).  Measurement only.

  python tools/pmc_pipeline.py PASSDIR --kernel NAME --part tag=SUBSTR ... --algo-bytes B --tag T --work W --out JSON
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("passdir")
    ap.add_argument("--kernel", required=True, help="name the bench line matches (pmc['kernel'])")
    ap.add_argument("--part", action="append", required=True, help="tag=substring of one kernel of the step")
    ap.add_argument("--algo-bytes", type=float, required=True)
    ap.add_argument("--tag", required=True)
    ap.add_argument("--work", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    parts = [p.split("=", 1) for p in a.part]
    vals = {t: {} for t, _ in parts}
    for f in glob.glob(os.path.join(a.passdir, "pmc_*", "*counter_collection.csv")):
        with open(f) as fh:
            per = {}
            for r in csv.DictReader(fh):
                for t, sub in parts:
                    if sub in r["Kernel_Name"]:
                        key = (t, r["Counter_Name"], r["Dispatch_Id"])
                        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
            for (t, c, _), v in per.items():
                vals[t].setdefault(c, []).append(v)
    med = {t: {c: statistics.median(v) for c, v in cs.items()} for t, cs in vals.items()}
    stats = {}
    for f in glob.glob(os.path.join(a.passdir, "trace", "*kernel_stats.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                for t, sub in parts:
                    if sub in r["Name"]:
                        stats[t] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    read = sum(m.get("FETCH_SIZE", 0.0) for m in med.values()) * 1024.0 * 2.0
    write = sum(m.get("WRITE_SIZE", 0.0) for m in med.values()) * 1024.0
    step_ns = sum(s["avg_ns"] for s in stats.values())
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {"kernel": a.kernel, "tag": a.tag, "launch_work": a.work, "counters_median_per_kernel": med,
           "rocprof_kernel_stats": stats, "read_bytes_corrected": read, "write_bytes": write,
           "traffic_bytes_per_launch": read + write, "algorithmic_bytes_per_launch": a.algo_bytes,
           "traffic_over_algorithmic": (read + write) / a.algo_bytes,
           "achieved_GBs_algorithmic_at_rocprof_avg": a.algo_bytes / (step_ns * 1e-9) / 1e9 if step_ns else None,
           "correction": "gfx950 FETCH_SIZE x2 (MI355X_MICROARCH.md §HBM); the kernels of one step summed",
           "source": os.path.relpath(os.path.abspath(a.out), root)}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: res[k] for k in ("traffic_bytes_per_launch", "traffic_over_algorithmic",
                                            "achieved_GBs_algorithmic_at_rocprof_avg")}))


if __name__ == "__main__":
    main()
