#!/usr/bin/env bash
# tools/variant_pmc.sh V... -- on the GPU box: kernel time and HBM read counters of
# the headline verify kernel for each TFS_CRC_VARIANT given (one rocprofv3 pass
# per counter group, never combined with other trace domains).
set -euo pipefail
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for v in "$@"; do
  OUT=gpurun_out/variant_pmc/v$v
  mkdir -p "$OUT"
  export TFS_CRC_VARIANT=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python bench.py --steps 6 --warmup 1 --no-cpu --e2e-blocks 0 > "$OUT/bench.json" 2> "$OUT/trace.err"
  for grp in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    name=$(echo "$grp" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "crc_files_kernel<1" -d "$OUT/pmc_$name" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --e2e-blocks 0 > "$OUT/pmc_$name.json" 2> "$OUT/pmc_$name.err"
  done
done
unset TFS_CRC_VARIANT
echo "variant pmc done"
