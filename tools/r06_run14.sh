#!/bin/bash
# Round 6 GPU pass 14: bodies of <= 80 bytes in the ring unit itself.  Full GPU
# suite, the floor probe (stamps), then a NUMA-bound latency A/B against the
# previous commit's library (abtmp/r06b), 3 rounds alternating, and the
# small_bodies line.
set -o pipefail
O=${1:-gpurun_out/r06/pass14}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 &&
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
timeout -k 10 120 tools/floor_probe 400 > $O/floor_probe.json 2> $O/floor_probe.err &&
for r in 1 2 3; do
  if [ $r = 2 ]; then
    timeout -k 10 120 tools/latency_probe_r06b 400 > $O/old_$r.json 2> $O/old_$r.err &&
    timeout -k 10 120 tools/latency_probe 400 > $O/new_$r.json 2> $O/new_$r.err || exit 1
  else
    timeout -k 10 120 tools/latency_probe 400 > $O/new_$r.json 2> $O/new_$r.err &&
    timeout -k 10 120 tools/latency_probe_r06b 400 > $O/old_$r.json 2> $O/old_$r.err || exit 1
  fi
done &&
timeout -k 10 300 python -u bench.py --workload small_bodies > $O/small_bodies.json 2> $O/small_bodies.err
