#!/usr/bin/env bash
# Round 5, run 2: the pruned tree (measurement forms cut, partial split, shared
# foreign-stream plan) -- the whole GPU suite, then the same-process A/B of the
# round-5 occupancy forms (94-99) against the product and the copy ceilings.
set -u
O=gpurun_out/r05/run2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/gputests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
AB_VARIANTS=94,95,96,97,98,99,26,68 timeout -k 10 500 python -u tools/ab_compact.py 6 > $O/ab.json 2> $O/ab.err || exit 7
echo ALLDONE
