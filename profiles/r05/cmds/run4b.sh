#!/usr/bin/env bash
# Round 5, run 4b: the rest of run 4 (group / ds / block store / error paths /
# split / streams tests after the per-rank fix), the configs[3] line and the
# direction probe with grouped zero-copy host compaction, then run 5's
# small-body latency line and the verify / packet kernel traces.
set -u
O=gpurun_out/r05/run4b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_group.py tests/test_ds_harness.py tests/test_block_store.py \
  tests/test_error_paths.py tests/test_split_files.py tests/test_scalar_and_streams.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --workload compact > $O/compact.json 2> $O/compact.err || exit 5
timeout -k 10 400 python -u tools/compact_direction_probe.py 64 4 > $O/direction.json 2> $O/direction.err || exit 8
bash profiles/r05/cmds/run5.sh || exit 9
echo ALLDONE
