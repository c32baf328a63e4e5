#!/bin/bash
# Round 6 GPU pass 3: the small-call floor with the fence / load split and a
# no-fence pass, and the close-path tail after prefaulting block reservations.
set -o pipefail
mkdir -p gpurun_out/r06
O=gpurun_out/r06
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
timeout -k 10 120 tools/floor_probe 400 > $O/floor_probe2.json 2> $O/floor_probe2.err &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ds_harness.py \
  tests/test_resident.py > $O/t3.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload loopback > $O/loopback2.json 2> $O/loopback2.err
