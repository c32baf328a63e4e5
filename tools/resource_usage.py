#!/usr/bin/env python3
"""Per-kernel register / LDS / scratch / occupancy table of a gfx950 build
(hipcc -Rpass-analysis=kernel-resource-usage), demangled names shortened.

  python tools/resource_usage.py [-DTFS_CRC_MEASURE] [--src=tfs_amd/csrc/tfs_ec_kernels.hip] [FILTER]
"""
import re
import subprocess
import sys

SRC = "tfs_amd/csrc/tfs_crc_kernels.hip"


def main():
    defs = [a for a in sys.argv[1:] if a.startswith("-D")]
    srcs = [a[6:] for a in sys.argv[1:] if a.startswith("--src=")]
    filt = [a for a in sys.argv[1:] if not a.startswith("-D") and not a.startswith("--src=")]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", srcs[0] if srcs else SRC, "-o", "/tmp/ru_k.o",
           "-Rpass-analysis=kernel-resource-usage", *defs]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (?:.*?)(Function Name|VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|"
                      r"Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k.split()[0]] = v
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    for r, n in zip(rows, names):
        n = re.sub(r"\(.*\)$", "", n).replace("tfscrc::", "").replace("tfsec::", "")
        if filt and not any(f in n for f in filt):
            continue
        print("%4s v %3s a %4s s %5s scr %6s lds occ %2s  %s" % (r.get("VGPRs"), r.get("AGPRs"), r.get("TotalSGPRs"),
                                                              r.get("ScratchSize"), r.get("LDS"), r.get("Occupancy"), n))


if __name__ == "__main__":
    main()
