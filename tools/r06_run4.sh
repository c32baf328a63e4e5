#!/bin/bash
# Round 6 GPU pass 4: the close path with and without prefaulted block
# reservations (TFS_DS_PREFAULT), alternating on one box.
set -o pipefail
mkdir -p gpurun_out/r06
O=gpurun_out/r06
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload loopback --no-cpu > $O/loopback_pf1_$i.json 2> $O/loopback_pf1_$i.err &&
  TFS_DS_PREFAULT=0 timeout -k 10 300 python -u bench.py --workload loopback --no-cpu > $O/loopback_pf0_$i.json 2> $O/loopback_pf0_$i.err || exit 1
done
