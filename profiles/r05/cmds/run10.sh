#!/usr/bin/env bash
# Round 5, run 10: device compaction time against its record count, sparse (341 of
# 1,024 live; 256..2048 resident blocks) and dense (every record live; 342 and 1024
# blocks), to separate a fixed per-launch cost from a per-record one.
set -u
O=gpurun_out/r05/run10
mkdir -p $O
for nb in 256 512 1024 2048; do
  AB_VARIANTS= timeout -k 10 300 python -u tools/ab_compact.py 3 $nb > $O/sparse_$nb.json 2> $O/sparse_$nb.err || exit 5
done
for nb in 342 1024; do
  AB_LIVE=all AB_VARIANTS= timeout -k 10 300 python -u tools/ab_compact.py 3 $nb > $O/dense_$nb.json 2> $O/dense_$nb.err || exit 6
done
echo ALLDONE
