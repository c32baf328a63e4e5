#!/bin/bash
# Round 6 GPU pass 19: the resident ring in fine-grained device memory written
# through the BAR (TFS_CRC_RESIDENT_VRAM=1) against the ring in host memory, one
# library.  The resident tests (both placements), the full GPU suite with the
# device ring, the floor probe with it, a NUMA-bound latency A/B (3 rounds
# alternating), and the loopback line both ways.
set -o pipefail
O=${1:-gpurun_out/r06/pass19}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_resident.py -m gpu > $O/resident_tests.log 2>&1 &&
TFS_CRC_RESIDENT_VRAM=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > $O/gpu_tests_vram.log 2>&1 &&
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
TFS_CRC_RESIDENT_VRAM=1 timeout -k 10 200 tools/floor_probe 400 > $O/floor_probe_vram.json 2> $O/floor_probe_vram.err &&
for r in 1 2 3; do
  if [ $r = 2 ]; then
    timeout -k 10 120 tools/latency_probe 400 > $O/host_$r.json 2> $O/host_$r.err &&
    TFS_CRC_RESIDENT_VRAM=1 timeout -k 10 120 tools/latency_probe 400 > $O/vram_$r.json 2> $O/vram_$r.err || exit 1
  else
    TFS_CRC_RESIDENT_VRAM=1 timeout -k 10 120 tools/latency_probe 400 > $O/vram_$r.json 2> $O/vram_$r.err &&
    timeout -k 10 120 tools/latency_probe 400 > $O/host_$r.json 2> $O/host_$r.err || exit 1
  fi
done &&
for r in 1 2; do
  TFS_CRC_RESIDENT_VRAM=1 timeout -k 10 300 python -u bench.py --workload loopback --no-cpu > $O/loopback_vram_$r.json 2> $O/loopback_vram_$r.err &&
  timeout -k 10 300 python -u bench.py --workload loopback --no-cpu > $O/loopback_host_$r.json 2> $O/loopback_host_$r.err || exit 1
done
