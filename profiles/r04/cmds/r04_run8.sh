#!/usr/bin/env bash
# Round 4: the erasure-code wide form (16 bytes per lane) against the product and
# the no-math form, and the EC tests over every kernel form.
set -eu
mkdir -p gpurun_out/r04/run8
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ec.py -m gpu > gpurun_out/r04/run8/test_ec.log 2>&1
timeout -k 10 300 python tools/ab_ec.py 8,7 8 > gpurun_out/r04/run8/ab_ec.json 2> gpurun_out/r04/run8/ab_ec.err
timeout -k 10 300 python tools/ab_ec.py 8 8 > gpurun_out/r04/run8/ab_ec2.json 2> gpurun_out/r04/run8/ab_ec2.err
echo ALLDONE
