#!/bin/bash
# Round 6 GPU pass 9: wide in-place launches of synchronous calls on per-slot
# streams -- parity, then the configs[2] receive-buffer leg against the context-
# stream form (TFS_CRC_VARIANT=53, measurement build), alternating.
set -o pipefail
mkdir -p gpurun_out/r06/wide_streams
O=gpurun_out/r06/wide_streams
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "wide" > $O/tests.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --workload zipf_e2e --e2e-blocks 128 > $O/new_$r.json 2> $O/new_$r.err &&
  TFS_CRC_VARIANT=53 timeout -k 10 200 python -u bench.py --workload zipf_e2e --e2e-blocks 128 > $O/ctx_$r.json 2> $O/ctx_$r.err || exit 1
done
