#!/usr/bin/env bash
# Round 5, run 20: the page-locked batch tests, with wide batches from four threads.
set -u
O=gpurun_out/r05/run20
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pinned" -m gpu -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
exit $rc
