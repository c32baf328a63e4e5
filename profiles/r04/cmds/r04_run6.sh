#!/usr/bin/env bash
# Round 4: is the device-compaction line slower than the in-process A/B of the same
# kernel?  The line, the A/B (whole records, 32 KiB segments, store-policy / PF
# variants), the line again -- one box, one call.
set -eu
mkdir -p gpurun_out/r04/run6
timeout -k 10 300 python bench.py --workload compact_device --no-cpu > gpurun_out/r04/run6/line1.json 2> gpurun_out/r04/run6/line1.err
AB_VARIANTS="25,35,75,76" AB_SEG=32768 timeout -k 10 600 python tools/ab_compact.py 4 \
  > gpurun_out/r04/run6/ab.json 2> gpurun_out/r04/run6/ab.err
timeout -k 10 300 python bench.py --workload compact_device --no-cpu > gpurun_out/r04/run6/line2.json 2> gpurun_out/r04/run6/line2.err
echo ALLDONE
