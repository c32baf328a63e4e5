#!/usr/bin/env bash
# Round 5, run 3: the pruned product on the default and device-compaction lines;
# the compaction occupancy A/B (97, 98) against the product and the copies on
# another box; the host-compaction direction probe.
set -u
O=gpurun_out/r05/run3
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/default.json 2> $O/default.err || exit 5
timeout -k 10 300 python -u bench.py --workload compact_device > $O/compact_device.json 2> $O/compact_device.err || exit 6
AB_VARIANTS=97,98,26,68 timeout -k 10 400 python -u tools/ab_compact.py 6 > $O/ab.json 2> $O/ab.err || exit 7
timeout -k 10 400 python -u tools/compact_direction_probe.py 64 4 > $O/direction.json 2> $O/direction.err || exit 8
echo ALLDONE
