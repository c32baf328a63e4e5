#!/usr/bin/env bash
# Round 5, run 11: wide page-locked host batches read in place by the throughput
# kernel, block verify with metas and verdicts in page-locked words: the pinned /
# block-verify parity tests, the same-process A/B against the staged forms
# (TFS_CRC_VARIANT=52), then the e2e, host block verify and default lines.
set -u
O=gpurun_out/r05/run11
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "pinned or block_verify or submit" -m gpu -x -v \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 500 python -u tools/ab_host_paths.py 5 128 > $O/ab_host.json 2> $O/ab_host.err || exit 5
timeout -k 10 300 python -u bench.py --workload e2e > $O/e2e.json 2> $O/e2e.err || exit 6
timeout -k 10 300 python -u bench.py --workload block_verify > $O/block_verify.json 2> $O/block_verify.err || exit 7
timeout -k 10 300 python -u bench.py > $O/default.json 2> $O/default.err || exit 8
echo ALLDONE
