#!/usr/bin/env bash
# Round 4: hybrid record order, half / three quarters static (89 / 88), against the
# product on the real workload, interleaved in one process.
set -eu
O=gpurun_out/r04/run13
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_compaction_kernels.py -m gpu -k hybrid > $O/test${TAG:-}.log 2>&1
AB_VARIANTS=88,89 timeout -k 10 400 python tools/ab_compact.py 8 > $O/ab${TAG:-}.json 2> $O/ab${TAG:-}.err
echo ALLDONE
