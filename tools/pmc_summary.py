#!/usr/bin/env python3
"""Fold rocprofv3 passes of one kernel into a PMC summary JSON (and, with
--latest, profiles/pmc_latest.json, which bench.py reads for roofline.traffic).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE (KiB)
reports half the bytes of a wide coalesced stream, so read bytes = FETCH_SIZE x
1024 x 2, cross-checked by TCC_EA0_RDREQ x 128 B; WRITE_SIZE (KiB) as is.
Counter values are medians over the kernel's dispatches."""
import argparse
import csv
import json
import os
import statistics


def counters(paths, kernel):
    vals = {}
    for p in paths:
        with open(p) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["Kernel_Name"]:
                    vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def kernel_stats(path, kernel):
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if kernel in row["Name"]:
                return {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                        "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"])}
    raise SystemExit("kernel %r not in %s" % (kernel, path))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="crc_files_kernel<1, 4, 3>")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--algo-bytes", type=float, default=1048576.0 * 65557)
    ap.add_argument("--stats", required=True, help="kernel_stats.csv of rocprofv3 --stats on the same command")
    ap.add_argument("--out", required=True)
    ap.add_argument("--latest", action="store_true")
    ap.add_argument("--work", default="1,048,576 files x 64 KiB payload (block images, FileInfo|payload)")
    ap.add_argument("--trace", help="kernel_trace.csv of the same command: also report the timed dispatches")
    ap.add_argument("--skip", type=int, default=0, help="dispatches before the timed ones (warm-up)")
    ap.add_argument("--count", type=int, default=0, help="timed dispatches")
    ap.add_argument("csvs", nargs="+", help="counter_collection.csv of each --pmc pass")
    a = ap.parse_args()
    c = counters(a.csvs, a.kernel)
    ks = kernel_stats(a.stats, a.kernel)
    if a.trace and a.count:
        # The --stats average includes the cold first dispatches; the bench line's
        # HIP events time only the steps after its warm-up.
        with open(a.trace) as fh:
            d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(fh)
                 if a.kernel in r["Kernel_Name"]]
        timed = d[a.skip:a.skip + a.count]
        ks["timed_dispatches"] = {"skip": a.skip, "count": len(timed), "avg_ns": sum(timed) / len(timed),
                                  "all_ns": d}
    read = c["FETCH_SIZE"] * 1024.0 * 2.0
    write = c.get("WRITE_SIZE", 0.0) * 1024.0
    res = {
        "kernel": a.kernel, "tag": a.tag,
        "launch_work": a.work,
        "rocprof_kernel_stats": ks, "counters_median": c,
        "read_bytes_corrected": read,
        "read_bytes_from_rdreq_x128": c["TCC_EA0_RDREQ_sum"] * 128.0 if "TCC_EA0_RDREQ_sum" in c else None,
        "write_bytes": write, "traffic_bytes_per_launch": read + write,
        "algorithmic_bytes_per_launch": a.algo_bytes,
        "traffic_over_algorithmic": (read + write) / a.algo_bytes,
        "achieved_GBs_algorithmic_at_rocprof_avg": a.algo_bytes / (ks["avg_ns"] * 1e-9) / 1e9,
        "achieved_GBs_algorithmic_at_rocprof_timed_avg": (a.algo_bytes / (ks["timed_dispatches"]["avg_ns"] * 1e-9) / 1e9
                                                          if "timed_dispatches" in ks else None),
        "correction": "gfx950 FETCH_SIZE reports half the bytes of a wide coalesced stream "
                      "(MI355X_MICROARCH.md §HBM): x2; cross-checked by TCC_EA0_RDREQ x 128 B",
        "source": os.path.relpath(a.out, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
    }
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    if a.latest:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        with open(os.path.join(root, "profiles", "pmc_latest.json"), "w") as fh:
            json.dump(res, fh, indent=1)
    print(json.dumps({k: res[k] for k in ("traffic_bytes_per_launch", "traffic_over_algorithmic",
                                            "achieved_GBs_algorithmic_at_rocprof_avg")}))


if __name__ == "__main__":
    main()
