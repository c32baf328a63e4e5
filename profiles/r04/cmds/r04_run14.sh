#!/usr/bin/env bash
# Round 4: the hybrid unit order on the segmented product form (90) against the
# segmented product (AB_SEG 32768), whole records with the hybrid order (88) and
# whole records, interleaved in one process; parity of the hybrid forms first.
set -eu
O=gpurun_out/r04/run14
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_compaction_kernels.py -m gpu -k "hybrid or vctx or statuses" > $O/test${TAG:-}.log 2>&1
AB_SEG=32768 AB_VARIANTS=88,90 timeout -k 10 400 python tools/ab_compact.py 8 > $O/ab${TAG:-}.json 2> $O/ab${TAG:-}.err
echo ALLDONE
