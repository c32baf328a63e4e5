#!/usr/bin/env bash
# Round 4: sustained load.  The compaction kernel and the dense copy timed over 3
# and over 16 back-to-back launches in one process, beside the line itself.
set -eu
mkdir -p gpurun_out/r04/run7
AB_VARIANTS="" AB_SEG=32768 AB_REPS=3 timeout -k 10 600 python tools/ab_compact.py 3 > gpurun_out/r04/run7/ab_reps3.json 2> gpurun_out/r04/run7/ab_reps3.err
AB_VARIANTS="" AB_SEG=32768 AB_REPS=16 timeout -k 10 600 python tools/ab_compact.py 3 > gpurun_out/r04/run7/ab_reps16.json 2> gpurun_out/r04/run7/ab_reps16.err
timeout -k 10 300 python bench.py --workload compact_device --no-cpu > gpurun_out/r04/run7/line.json 2> gpurun_out/r04/run7/line.err
timeout -k 10 300 python bench.py --workload block_verify_device --no-cpu > gpurun_out/r04/run7/bvd.json 2> gpurun_out/r04/run7/bvd.err
timeout -k 10 300 python tools/ab_ec.py 8,7 8 > gpurun_out/r04/run7/ab_ec.json 2> gpurun_out/r04/run7/ab_ec.err
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ec.py -m gpu > gpurun_out/r04/run7/test_ec.log 2>&1
echo ALLDONE
