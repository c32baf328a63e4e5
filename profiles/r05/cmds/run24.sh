#!/usr/bin/env bash
# Round 5, run 24: the wide page-locked batch tests, with the 65,536-file limit.
set -u
O=gpurun_out/r05/run24
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "wide_pinned" -m gpu -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
exit $rc
