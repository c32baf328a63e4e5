#!/usr/bin/env bash
# Round 5, run 18: the N = 2 line at full size with both ranks on the one GPU of the
# box (TFS_BENCH_SHARE_DEVICE=1; each rank holds its own 1,024 resident blocks): the
# per-rank attribution fields of an N > 1 line at full size.  Not a scaling figure.
set -u
O=gpurun_out/r05/run18
mkdir -p $O
TFS_BENCH_SHARE_DEVICE=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 8 --warmup 2 > $O/n2_shared.json 2> $O/n2_shared.err || exit 5
echo ALLDONE
