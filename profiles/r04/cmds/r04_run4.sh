#!/usr/bin/env bash
# Round 4: do partial-line writes cost a dense copy?  The 64 KiB wave-chunk copy
# (53104) beside the same copy with one / two 16-byte holes per chunk and with
# its ends written as byte stores, interleaved with the compaction kernel (whole
# records and 32 KiB segments) in one process.
set -eu
mkdir -p gpurun_out/r04/run4
AB_VARIANTS="" AB_SEG=32768 AB_COPIES="53204:256,53304:256,53404:256" timeout -k 10 600 python tools/ab_compact.py 5 \
  > gpurun_out/r04/run4/ab_holes.json 2> gpurun_out/r04/run4/ab_holes.err
O=gpurun_out/r04/run4/pmc
PMC_GROUPS=tccw,tccs,write tools/pmc_passes.sh $O hole2 "membench_copy_chunk" -- python tools/copy_probe.py 53304 256
PMC_GROUPS=tccw,tccs,write tools/pmc_passes.sh $O hole3 "membench_copy_chunk" -- python tools/copy_probe.py 53404 256
echo ALLDONE
