#!/usr/bin/env bash
# Round 4: the -m gpu suite and smoke on this tree, then rocprofv3 kernel-trace +
# FETCH/WRITE passes of the erasure-code, device block-verify and packet lines
# (their roofline.traffic summaries move to round-4 profiles).
set -u
O=gpurun_out/r04/run9
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/gputests.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
PMC_GROUPS=fetch,write tools/pmc_passes.sh $O/prof ec "ec_apply_kernel" -- python bench.py --workload ec --no-cpu --steps 4 --warmup 1 || exit 4
PMC_GROUPS=fetch,write tools/pmc_passes.sh $O/prof bvd "compact_pipe_kernel<true, true, true" -- python bench.py --workload block_verify_device --no-cpu --steps 4 --warmup 1 || exit 5
PMC_GROUPS=fetch,write tools/pmc_passes.sh $O/prof packet "packet_|crc_files_kernel" -- python bench.py --workload packet --no-cpu --steps 4 --warmup 1 || exit 6
echo ALLDONE
