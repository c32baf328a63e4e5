#!/bin/bash
# Round 6, first GPU pass: ADVICE r5 fixes, tfs_crc32_stats, the zipf end-to-end
# leg, the EC 5:3 copy ceiling, the small-call floor and the close-path tail.
set -o pipefail
mkdir -p gpurun_out/r06
O=gpurun_out/r06
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_compaction_kernels.py tests/test_scalar_and_streams.py tests/test_resident.py \
  tests/test_ds_harness.py > $O/t1.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload zipf_e2e --e2e-blocks 128 > $O/zipf_e2e.json 2> $O/zipf_e2e.err &&
timeout -k 10 200 python -u tools/ab_ec.py 20,21 6 > $O/ab_ec_copy.json 2> $O/ab_ec_copy.err &&
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
timeout -k 10 120 tools/floor_probe 400 > $O/floor_probe.json 2> $O/floor_probe.err &&
timeout -k 10 300 python -u bench.py --workload loopback > $O/loopback.json 2> $O/loopback.err
