#!/bin/bash
# Round 6 GPU pass 2 (the suite of pass 1 passed: gpurun_out/r06/t1.log): the zipf
# end-to-end leg, the EC 5:3 copy ceiling, the small-call floor, the close-path tail
# and the LDS-DMA compaction A/B.
set -o pipefail
mkdir -p gpurun_out/r06
O=gpurun_out/r06
timeout -k 10 200 python -u bench.py --workload zipf_e2e --e2e-blocks 128 > $O/zipf_e2e.json 2> $O/zipf_e2e.err &&
timeout -k 10 200 python -u tools/ab_ec.py 20,21 6 > $O/ab_ec_copy.json 2> $O/ab_ec_copy.err &&
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
timeout -k 10 120 tools/floor_probe 400 > $O/floor_probe.json 2> $O/floor_probe.err &&
timeout -k 10 300 python -u bench.py --workload loopback > $O/loopback.json 2> $O/loopback.err &&
AB_VARIANTS=97,120,121 timeout -k 10 300 python -u tools/ab_compact.py 6 > $O/ab_compact_lds.json 2> $O/ab_compact_lds.err
