#!/usr/bin/env bash
# Round 6: rocprofv3 kernel trace + PMC passes (FETCH_SIZE, WRITE_SIZE, TCC EA
# requests) of the other device-resident lines' dominant kernels at full size
# (the headline's are in tools/r06_final4.sh).  Raw CSVs under gpurun_out/r06/pmc/<line>/;
# tools/pmc_summary.py folds them into profiles/r06/pmc/<line>/pmc_summary.json.
set -u
O=gpurun_out/r06/pmc
mkdir -p $O
export PMC_GROUPS=fetch,write,tccw
tools/pmc_passes.sh $O zipf "crc_files_kernel<0, 4, 3>" -- python bench.py --workload zipf --no-cpu --steps 4 --warmup 1 --e2e-blocks 0 || exit 3
tools/pmc_passes.sh $O packet "packet_files_kernel<1>" -- python bench.py --workload packet --no-cpu --steps 4 --warmup 1 || exit 4
tools/pmc_passes.sh $O compact_device "compact_pipe_kernel<true, false, 12, 5, 1, 0, false, 2" -- \
  python bench.py --workload compact_device --no-cpu --steps 4 --warmup 1 || exit 5
tools/pmc_passes.sh $O block_verify_device "compact_pipe_kernel<true, true, 12, 5, 4, 3" -- \
  python bench.py --workload block_verify_device --no-cpu --steps 4 --warmup 1 || exit 6
tools/pmc_passes.sh $O ec "ec_apply_kernel<3" -- python bench.py --workload ec --no-cpu --steps 4 --warmup 1 || exit 7
echo PMCDONE
