#!/usr/bin/env bash
# Round 5, run 21: every other in-flight wide page-locked block on a second stream
# (variant 53): the wide-pinned test, then the host-path A/B (product, staged, two streams).
set -u
O=gpurun_out/r05/run21
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "wide_pinned" -m gpu -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 500 python -u tools/ab_host_paths.py 6 128 > $O/ab_host.json 2> $O/ab_host.err || exit 5
echo ALLDONE
