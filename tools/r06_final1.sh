#!/bin/bash
# Round 6 closing pass 1: the driver's sequence on this tree (GPU suite, smoke,
# the headline line with the driver's arguments), the small-call floor, and the
# threaded host block verify against one caller thread.
set -o pipefail
O=gpurun_out/r06/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err &&
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
timeout -k 10 120 tools/floor_probe 400 > $O/floor_probe.json 2> $O/floor_probe.err &&
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --workload block_verify --no-cpu > $O/block_verify_t3_$r.json 2> $O/block_verify_t3_$r.err &&
  timeout -k 10 200 python -u bench.py --workload block_verify --no-cpu --verify-threads 1 > $O/block_verify_t1_$r.json 2> $O/block_verify_t1_$r.err || exit 1
done
