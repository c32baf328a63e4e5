#!/usr/bin/env bash
# Round 4: the hybrid chunk order on the headline verify (91-93: the first 3/4,
# 1/2, 7/8 of the 4-file chunks static, tickets after) -- parity on 1 M files, then
# the in-process A/B against the product on the resident 1 M x 64 KiB set.
set -eu
O=gpurun_out/r04/run15
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "million and (91 or 92 or 93 or 42)" > $O/test${TAG:-}.log 2>&1
AB_ONLY=product AB_VARIANTS=91,92,93 timeout -k 10 400 python tools/ab_inproc.py - 8 > $O/ab${TAG:-}.json 2> $O/ab${TAG:-}.err
echo ALLDONE
