#!/usr/bin/env bash
# Round 5, run 19: process-to-process spread of the headline on one box -- the
# default line (driver arguments, no CPU legs) in four separate processes.
set -u
O=gpurun_out/r05/run19
mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-blocks 0 > $O/default_$i.json 2> $O/default_$i.err || exit 5
done
echo ALLDONE
