#!/usr/bin/env bash
# Round 5, run 14: the small-body line with tfs_packet_verify timed through ctypes on
# arrays made once; the GPU tests of the files whose imports changed.
set -u
O=gpurun_out/r05/run14
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_abi.py tests/test_read_path.py tests/test_headline_parity.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload small_bodies > $O/small_bodies.json 2> $O/small_bodies.err || exit 5
echo ALLDONE
