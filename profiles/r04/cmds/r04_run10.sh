#!/usr/bin/env bash
# Round 4: where the 8 % between the record kernel and the chunk copy of the same
# dense layout goes -- the kernel, the kernel reduced to a copy (64), without CRC
# steps (26), static order (60), and the probe copies over the job list (67 tickets,
# 68 static) on the dense 64 KiB layout, beside the chunk copy, one process.
set -eu
mkdir -p gpurun_out/r04/run10
AB_ALIGNED=1 AB_VARIANTS=${AB_VARIANTS:-64,67,68,26,60} timeout -k 10 400 python tools/ab_compact.py 5 > gpurun_out/r04/run10/ab${TAG:-}.json 2> gpurun_out/r04/run10/ab${TAG:-}.err
echo ALLDONE
