#!/usr/bin/env bash
# Round 5, run 17: the host block verify line with its timed loop calling the C ABI
# directly (arrays made once), twice; the resident tests (order-robust grid check).
set -u
O=gpurun_out/r05/run17
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_resident.py tests/test_bench_contract.py -m gpu -x -q --timeout 250 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload block_verify > $O/block_verify_1.json 2> $O/block_verify_1.err || exit 5
timeout -k 10 300 python -u bench.py --workload block_verify --no-cpu > $O/block_verify_2.json 2> $O/block_verify_2.err || exit 6
echo ALLDONE
