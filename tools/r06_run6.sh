#!/bin/bash
# Round 6 GPU pass 6: same-box A/B of the resident ring protocol -- this tree's
# library (units polled by tag, tiny bodies in one load) against the round-5
# closing tree's (abtmp/r05, built from commit c37a82d), alternating processes.
set -o pipefail
mkdir -p gpurun_out/r06/latency_ab
O=gpurun_out/r06/latency_ab
for r in 1 2 3; do
  timeout -k 10 120 tools/latency_probe 400 > $O/new_$r.json 2> $O/new_$r.err &&
  timeout -k 10 120 tools/latency_probe_r05 400 > $O/r05_$r.json 2> $O/r05_$r.err || exit 1
done
