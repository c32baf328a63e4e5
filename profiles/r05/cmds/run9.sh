#!/usr/bin/env bash
# Round 5, run 9: the erasure-code form with every source member in flight (variant
# 7: parity, then a same-process A/B against the product); translation and issue
# counters of device compaction over the sparse live records (341 of 1,024, the
# product workload) and over a dense source (every record live).
set -u
O=gpurun_out/r05/run9
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ec.py -k "kernel_forms" -m gpu -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 400 python -u tools/ab_ec.py 7 8 > $O/ab_ec.json 2> $O/ab_ec.err || exit 5
K="compact_pipe_kernel<true, false, 12, 5, 1, 0, false, 2, 16, 1, 1>"
PMC_GROUPS=tcp,sq1 AB_VARIANTS= tools/pmc_passes.sh $O cd_sparse "$K" -- python tools/ab_compact.py 1 || exit 6
PMC_GROUPS=tcp,sq1 AB_LIVE=all AB_VARIANTS= tools/pmc_passes.sh $O cd_dense "$K" -- python tools/ab_compact.py 1 || exit 7
echo ALLDONE
