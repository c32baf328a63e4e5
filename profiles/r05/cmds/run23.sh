#!/usr/bin/env bash
# Round 5, run 23: the measurement tools after membench's shape check -- the compaction
# A/B (copies 52114 / 53xxx) and the verify read ceilings, one round each.
set -u
O=gpurun_out/r05/run23
mkdir -p $O
AB_VARIANTS= timeout -k 10 400 python -u tools/ab_compact.py 1 > $O/ab_compact.json 2> $O/ab_compact.err || exit 5
timeout -k 10 400 python -u tools/ceilings.py verify 2 > $O/ceilings.json 2> $O/ceilings.err || exit 6
echo ALLDONE
