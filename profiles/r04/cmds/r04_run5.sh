#!/usr/bin/env bash
# Round 4: the record kernel over a dense, 64 KiB-aligned record list (where does
# the gap to the dense copy come from?), then every bench line at full size.
set -u
mkdir -p gpurun_out/r04/run5
AB_VARIANTS="" AB_ALIGNED=1 timeout -k 10 600 python tools/ab_compact.py 3 \
  > gpurun_out/r04/run5/ab_aligned.json 2> gpurun_out/r04/run5/ab_aligned.err || exit 1
bash tools/all_lines.sh gpurun_out/r04/run5/lines
echo ALLDONE
