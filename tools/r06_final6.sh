#!/bin/bash
# Round 6 closing pass 6 (the committed final tree): the driver's sequence
# (GPU suite, smoke, the headline with the driver's arguments), then the ring's
# lines -- small bodies, loopback -- and the latency and floor probes.
set -o pipefail
O=gpurun_out/r06/final6
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 400 python bench.py --workload small_bodies > $O/small_bodies.json 2> $O/small_bodies.err &&
timeout -k 10 400 python bench.py --workload loopback > $O/loopback.json 2> $O/loopback.err &&
timeout -k 10 120 tools/latency_probe 400 > $O/latency_probe.json 2> $O/latency_probe.err &&
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
timeout -k 10 200 tools/floor_probe 400 > $O/floor_probe.json 2> $O/floor_probe.err
