#!/usr/bin/env bash
# Round 5, run 15: device compaction time per record against launch length in one
# process (the packed job list whole, its first half and first quarter), twice.
set -u
O=gpurun_out/r05/run15
mkdir -p $O
AB_PARTS=1 AB_VARIANTS= timeout -k 10 400 python -u tools/ab_compact.py 5 > $O/parts_a.json 2> $O/parts_a.err || exit 5
AB_PARTS=1 AB_VARIANTS= timeout -k 10 400 python -u tools/ab_compact.py 5 > $O/parts_b.json 2> $O/parts_b.err || exit 6
echo ALLDONE
