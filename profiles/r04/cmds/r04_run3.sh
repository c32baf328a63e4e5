#!/usr/bin/env bash
# Round 4, third GPU call: the whole -m gpu suite, then the default line and the
# Zipf / device-compaction / EC lines at full size, then the headline and Zipf
# rocprofv3 kernel-trace + FETCH/WRITE passes of this tree.
set -u
mkdir -p gpurun_out/r04/run3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04/run3/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -3 gpurun_out/r04/run3/gputests.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/run3/smoke.log 2>&1 || exit 3
for w in default zipf compact_device ec; do
  if [[ $w == default ]]; then args=(); else args=(--workload $w); fi
  timeout -k 10 300 python bench.py "${args[@]}" > gpurun_out/r04/run3/$w.json 2> gpurun_out/r04/run3/$w.err || exit 4
  echo "$w done"
done
O=gpurun_out/r04/run3/prof
PMC_GROUPS=fetch,write tools/pmc_passes.sh $O verify "crc_files_kernel<1" -- python bench.py --steps 8 --warmup 2 --no-cpu --e2e-blocks 0 --parity-every 1024
PMC_GROUPS=fetch,write tools/pmc_passes.sh $O zipf "crc_files_kernel<0" -- python bench.py --workload zipf --no-cpu --steps 4 --warmup 1
PMC_GROUPS=fetch,write tools/pmc_passes.sh $O compact "compact_pipe_kernel<true, true, false" -- python bench.py --workload compact_device --no-cpu --steps 4 --warmup 1
echo ALLDONE
