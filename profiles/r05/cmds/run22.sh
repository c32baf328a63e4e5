#!/usr/bin/env bash
# Round 5, run 22: does the physical layout of the 64 GiB image set the headline's
# process-to-process spread?  The default line (driver arguments, no CPU legs) in
# alternating processes: hipMalloc (the product), physical chunks of 1 GiB and of
# 256 MiB mapped back to back (TFS_CRC_DEV_VMM), three processes each.
set -u
O=gpurun_out/r05/run22
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-blocks 0 > $O/malloc_$i.json 2> $O/malloc_$i.err || exit 5
  TFS_CRC_DEV_VMM=1024 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-blocks 0 > $O/vmm1024_$i.json 2> $O/vmm1024_$i.err || exit 6
  TFS_CRC_DEV_VMM=256 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-blocks 0 > $O/vmm256_$i.json 2> $O/vmm256_$i.err || exit 7
done
echo ALLDONE
