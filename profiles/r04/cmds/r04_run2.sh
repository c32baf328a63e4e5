#!/usr/bin/env bash
# Round 4, second GPU call: counter passes of the device compaction (f3) beside
# dense copies of the same byte count, and of the erasure-code kernel (f4); the
# segment-split probe of the compaction kernel.
set -eu
O=gpurun_out/r04/pmc
mkdir -p gpurun_out/r04
tools/pmc_passes.sh $O compact "compact_pipe_kernel<true, true, false" -- python bench.py --workload compact_device --no-cpu --steps 2 --warmup 1
PMC_GROUPS=sq1,tcp,tccw,fetch,write,tccs tools/pmc_passes.sh $O copy53104 "membench_copy_chunk" -- python tools/copy_probe.py 53104 256
PMC_GROUPS=sq1,tcp,tccw,fetch,write,tccs tools/pmc_passes.sh $O copy53101 "membench_copy_chunk" -- python tools/copy_probe.py 53101 2048
tools/pmc_passes.sh $O ec "ec_apply_kernel" -- python bench.py --workload ec --no-cpu --steps 2 --warmup 1
AB_VARIANTS="" AB_SEG=8192,16384,32768 AB_SPLIT=16384 timeout -k 10 600 python tools/ab_compact.py 4 > gpurun_out/r04/ab_compact_split.json 2> gpurun_out/r04/ab_compact_split.err
timeout -k 10 300 python tools/ab_ec.py 7,6 8 > gpurun_out/r04/ab_ec.json 2> gpurun_out/r04/ab_ec.err
AB_ONLY=product,product_ao PMC_GROUPS=tcp,sq1,tccs tools/pmc_passes.sh $O zipf_forms "crc_files_kernel<0" -- python tools/ab_inproc.py - 2 zipf
echo ALLDONE
