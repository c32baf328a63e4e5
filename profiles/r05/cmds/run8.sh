#!/usr/bin/env bash
# Round 5, run 8: erasure-code member placement (tools/ab_ec_skew.py); the
# compaction A/B over a dense source (every record live, AB_LIVE=all) beside the
# 64 KiB-aligned list, to split the record list's cost into density and alignment;
# host compaction at 16..256 blocks per launch.
set -u
O=gpurun_out/r05/run8
mkdir -p $O
timeout -k 10 400 python -u tools/ab_ec_skew.py 6 > $O/ec_skew.json 2> $O/ec_skew.err || exit 5
AB_LIVE=all AB_ALIGNED=1 AB_VARIANTS=68 timeout -k 10 500 python -u tools/ab_compact.py 4 > $O/ab_compact_dense.json 2> $O/ab_compact_dense.err || exit 6
CG_GROUPS=16,64,128,256 timeout -k 10 400 python -u tools/compact_group_probe.py 1024 3 > $O/group.json 2> $O/group.err || exit 7
echo ALLDONE
