#!/bin/bash
# Round 6 GPU pass 7: the resident kernel's acquire fence -- its cost, staleness
# without it (default page-locked staging), and fine-grained staging without it.
set -o pipefail
mkdir -p gpurun_out/r06
O=gpurun_out/r06
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
TFS_FLOOR_NOFENCE=1 timeout -k 10 200 tools/floor_probe 400 > $O/floor_probe4.json 2> $O/floor_probe4.err
