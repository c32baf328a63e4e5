#!/usr/bin/env bash
# Round 5, run 16: erasure-code forms -- plain parity stores (8), plain member loads (9),
# two members in flight (10) -- parity, then an 8-round A/B against the product.
set -u
O=gpurun_out/r05/run16
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ec.py -k "kernel_forms" -m gpu -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 500 python -u tools/ab_ec.py 8,9,10 8 > $O/ab_ec.json 2> $O/ab_ec.err || exit 5
echo ALLDONE
