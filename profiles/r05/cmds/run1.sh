#!/usr/bin/env bash
# Round 5, run 1: two workgroups per CU for the record kernel (variants 94-99:
# LdsLayout<2> tables, 10/12/16-wave workgroups) -- oracle parity of the jobs
# forms, then the same-process A/B against the product and the copy ceilings.
set -u
O=gpurun_out/r05/run1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_compaction_kernels.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "94 or 95 or 96 or 97 or 98 or 99" > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
AB_VARIANTS=94,95,96,97,98,99 timeout -k 10 500 python -u tools/ab_compact.py 6 > $O/ab.json 2> $O/ab.err || exit 7
echo ALLDONE
