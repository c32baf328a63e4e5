#!/bin/bash
# Round 6 GPU pass 21: landing slots of 64 KiB (abtmp/land64) against 16 KiB (the
# product, abtmp/cur), swapped in turn under the latency probe (3 rounds) and the
# loopback line (2 rounds).
set -o pipefail
O=${1:-gpurun_out/r06/pass21}
mkdir -p $O
bash tools/ab_swap.sh 3 cur,land64 tools/latency_probe 400 > $O/ab_latency.log 2>&1 &&
bash tools/ab_swap.sh 2 cur,land64 python -u bench.py --workload loopback --no-cpu > $O/ab_loopback.log 2>&1
