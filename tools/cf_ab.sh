#!/usr/bin/env bash
# tools/cf_ab.sh OUT -- on the GPU box: chunked tickets (TFS_CRC_VARIANT 39/40/42/
# 43/45 = 2 / 4 / 4 with the last n/8 single / 4 with the last n/4 single / 3
# consecutive files per ticket) against the product (0): interleaved in-process
# A/B on the headline, Zipf, packet, device compaction and device block-verify
# lines, then one rocprofv3 PMC pass per variant (address translation, DRAM reads).
set -euo pipefail
OUT=${1:-gpurun_out/cf_ab}
VS=${2:-0,50,40,47,48}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu --e2e-blocks 0 --ab $VS --ab-rounds 8 \
  > "$OUT/verify_ab.json" 2> "$OUT/verify_ab.err"
timeout -k 10 300 python bench.py --workload zipf --steps 4 --warmup 1 --no-cpu --ab $VS --ab-rounds 8 \
  > "$OUT/zipf_ab.json" 2> "$OUT/zipf_ab.err"
AB_VARIANTS=${VS#0,} timeout -k 10 400 python tools/ab_compact.py 6 > "$OUT/compact_ab.json" 2> "$OUT/compact_ab.err"
if [ "${PMC:-1}" = 1 ]; then
CTRS="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum"
for v in ${VS//,/ }; do
  TFS_CRC_VARIANT=$v timeout -s KILL 200 rocprofv3 --pmc $CTRS --kernel-include-regex "crc_files_kernel<1" \
    -d "$OUT/pmc_v$v" -o run --output-format csv -- python bench.py --steps 6 --warmup 2 --no-cpu --e2e-blocks 0 \
    --parity-every 1024 > "$OUT/pmc_v$v.json" 2> "$OUT/pmc_v$v.err"
done
fi
echo "cf_ab done"
