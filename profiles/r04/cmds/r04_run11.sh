#!/usr/bin/env bash
# Round 4: compaction parity over every measurement variant (77/78 W slots,
# 81-83 cross-record ring / wide head loads), then the in-process A/B of 81-83
# against the product and the chunk copy of the same bytes.
set -eu
O=gpurun_out/r04/run11
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_compaction_kernels.py -m gpu > $O/test.log 2>&1
AB_VARIANTS=81,82,83,77 timeout -k 10 400 python tools/ab_compact.py 6 > $O/ab.json 2> $O/ab.err
echo ALLDONE
