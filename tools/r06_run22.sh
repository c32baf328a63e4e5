#!/bin/bash
# Round 6 GPU pass 22: tail shift tables in the latency form (one table round for a
# body's tail).  Full GPU suite, the floor probe with the fenced form as a second pass
# (TFS_FLOOR_FENCE=1: its cost, and that no result changes), then a NUMA-bound
# latency A/B against the previous commit's library (abtmp/r06d), 3 rounds
# alternating, and the loopback line (64 KiB closes through the ring).
set -o pipefail
O=${1:-gpurun_out/r06/pass22}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 &&
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
TFS_FLOOR_FENCE=1 timeout -k 10 200 tools/floor_probe 400 > $O/floor_probe.json 2> $O/floor_probe.err &&
for r in 1 2 3; do
  if [ $r = 2 ]; then
    timeout -k 10 120 tools/latency_probe_r06d 400 > $O/old_$r.json 2> $O/old_$r.err &&
    timeout -k 10 120 tools/latency_probe 400 > $O/new_$r.json 2> $O/new_$r.err || exit 1
  else
    timeout -k 10 120 tools/latency_probe 400 > $O/new_$r.json 2> $O/new_$r.err &&
    timeout -k 10 120 tools/latency_probe_r06d 400 > $O/old_$r.json 2> $O/old_$r.err || exit 1
  fi
done &&
mkdir -p abtmp/cur && cp tfs_amd/libtfs_crc.so abtmp/cur/ &&
bash tools/ab_swap.sh 2 cur,r06d python -u bench.py --workload small_bodies > $O/ab_swap.log 2>&1
