#!/bin/bash
# Round 6 GPU pass 5: the resident ring polled by unit tag (no separate unit
# read) and tiny bodies in one load -- the full GPU suite, the small-call floor,
# small bodies and the close path.
set -o pipefail
mkdir -p gpurun_out/r06
O=gpurun_out/r06
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > $O/t5.log 2>&1 &&
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
timeout -k 10 120 tools/floor_probe 400 > $O/floor_probe3.json 2> $O/floor_probe3.err &&
timeout -k 10 200 python -u bench.py --workload small_bodies > $O/small_bodies3.json 2> $O/small_bodies3.err &&
timeout -k 10 300 python -u bench.py --workload loopback > $O/loopback3.json 2> $O/loopback3.err
