#!/usr/bin/env bash
# Round 4: the device compaction product switched to whole records in the hybrid
# order (kCompactHS) -- the GPU suite and smoke, kernel-trace + FETCH/WRITE passes of
# the compaction line (its new kernel), the compaction and default lines, and the
# in-process A/B against the former default (32 KiB segments).
set -u
O=gpurun_out/r04/run19
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/gputests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
PMC_GROUPS=fetch,write tools/pmc_passes.sh $O/prof compact "compact_pipe_kernel<true, true, false" -- python bench.py --workload compact_device --no-cpu --steps 4 --warmup 1 || exit 4
timeout -k 10 300 python bench.py --workload compact_device > $O/compact_device.json 2> $O/compact_device.err || exit 5
timeout -k 10 300 python bench.py > $O/default.json 2> $O/default.err || exit 6
AB_SEG=32768 AB_VARIANTS=88 timeout -k 10 400 python tools/ab_compact.py 8 > $O/ab.json 2> $O/ab.err || exit 7
echo ALLDONE
