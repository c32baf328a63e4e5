#!/usr/bin/env bash
# tools/variance_pmc.sh N OUT -- the headline line in N separate processes, each
# under one rocprofv3 PMC pass (address translation, read latency and DRAM-side
# read counters of the verify kernel), to see what differs between a fast and a
# slow process placement (measurement only).
set -euo pipefail
N=${1:-5}
OUT=${2:-gpurun_out/variance}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
CTRS="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum"
for i in $(seq 1 "$N"); do  # env passes through (e.g. TFS_CRC_DEV_CONTIG)
  timeout -s KILL 200 rocprofv3 --pmc $CTRS --kernel-include-regex "crc_files_kernel<1" -d "$OUT/run$i" -o run \
    --output-format csv -- python bench.py --steps 6 --warmup 2 --no-cpu --e2e-blocks 0 --parity-every 1024 \
    > "$OUT/run$i.json" 2> "$OUT/run$i.err"
done
echo "variance_pmc done"
