#!/bin/bash
# Round 6 GPU pass 10: async wide submissions on per-slot streams too, and the
# latency form's shift levels bounded by the distance -- parity, the small-call
# floor, and the configs[4] end-to-end leg against the context-stream form.
set -o pipefail
mkdir -p gpurun_out/r06/pass10
O=gpurun_out/r06/pass10
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_latency_form.py tests/test_resident.py tests/test_scalar_and_streams.py tests/test_packet.py > $O/tests.log 2>&1 &&
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
timeout -k 10 120 tools/floor_probe 400 > $O/floor_probe.json 2> $O/floor_probe.err &&
timeout -k 10 200 python -u bench.py --workload small_bodies > $O/small_bodies.json 2> $O/small_bodies.err &&
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --workload e2e --compact-blocks 256 --no-cpu > $O/e2e_new_$r.json 2> $O/e2e_new_$r.err &&
  TFS_CRC_VARIANT=53 timeout -k 10 200 python -u bench.py --workload e2e --compact-blocks 256 --no-cpu > $O/e2e_ctx_$r.json 2> $O/e2e_ctx_$r.err || exit 1
done
