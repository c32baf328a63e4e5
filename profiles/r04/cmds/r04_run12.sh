#!/usr/bin/env bash
# Round 4: the hybrid record order (86-88: static for the first n - (n >> HS)
# records, tickets for the rest) -- parity over every compaction variant, then the
# in-process A/B against the product and the static / ticketed probe copies.
set -eu
O=gpurun_out/r04/run12
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_compaction_kernels.py -m gpu > $O/test.log 2>&1
AB_ALIGNED=1 AB_VARIANTS=86,87,88,79,67,68 timeout -k 10 400 python tools/ab_compact.py 5 > $O/ab.json 2> $O/ab.err
echo ALLDONE
