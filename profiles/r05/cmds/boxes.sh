#!/usr/bin/env bash
# Round 5: the driver's headline command on whatever box this call lands on (run once
# per call, several calls: the box-to-box spread), plus the box's PCIe ceilings.
set -u
O=gpurun_out/r05/boxes/${BOX_TAG:-x}
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 4
rocm-smi --showproductname --showserial > $O/smi.txt 2>&1 || true
echo ALLDONE
