#!/usr/bin/env bash
# Round 5, run 4: grouped zero-copy host compaction (runs of 16 page-locked blocks
# per launch) -- its parity tests and every compaction / group / ds test, then the
# configs[3] line and the direction probe on the same box; the N=2 lines.
set -u
O=gpurun_out/r05/run4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_compaction_kernels.py tests/test_group.py \
  tests/test_ds_harness.py tests/test_block_store.py tests/test_error_paths.py tests/test_split_files.py \
  tests/test_scalar_and_streams.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --workload compact > $O/compact.json 2> $O/compact.err || exit 5
timeout -k 10 400 python -u tools/compact_direction_probe.py 64 4 > $O/direction.json 2> $O/direction.err || exit 8
echo ALLDONE
