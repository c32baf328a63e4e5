#!/bin/bash
# Round 6 GPU pass 11: the latency form issues only the stripes a file has --
# parity of the latency and resident forms, then the small-call floor.
set -o pipefail
mkdir -p gpurun_out/r06/pass11
O=gpurun_out/r06/pass11
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_latency_form.py \
  tests/test_resident.py tests/test_scalar_and_streams.py tests/test_packet.py tests/test_gpu_parity.py > $O/tests.log 2>&1 &&
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
timeout -k 10 120 tools/floor_probe 400 > $O/floor_probe.json 2> $O/floor_probe.err &&
timeout -k 10 200 python -u bench.py --workload small_bodies > $O/small_bodies.json 2> $O/small_bodies.err &&
timeout -k 10 120 tools/latency_probe 400 > $O/latency_new.json 2> $O/latency_new.err &&
timeout -k 10 120 tools/latency_probe_r05 400 > $O/latency_r05.json 2> $O/latency_r05.err
