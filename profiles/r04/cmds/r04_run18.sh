#!/usr/bin/env bash
# Round 4: the erasure-code narrow form (9: 4 bytes per lane, 46 VGPRs, 8 waves per
# SIMD) against the product (88 VGPRs, 5 waves) and the wide form (8) -- parity
# over every form, then two in-process A/Bs.
set -eu
O=gpurun_out/r04/run18${TAG:-}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ec.py -m gpu > $O/test_ec.log 2>&1
timeout -k 10 300 python tools/ab_ec.py ${EC_V:-9,8} 8 > $O/ab_ec.json 2> $O/ab_ec.err
timeout -k 10 300 python tools/ab_ec.py ${EC_V2:-9} 8 > $O/ab_ec2.json 2> $O/ab_ec2.err
echo ALLDONE
