#!/usr/bin/env bash
# tools/profile.sh TAG -- rocprofv3 passes over the headline bench command, run
# on the GPU box (gpurun).  Kernel trace + stats in one pass; each PMC group in
# its own pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a
# pass; counters never combined with other trace domains).  Outputs under
# gpurun_out/prof_TAG/; tools/pmc_summary.py turns them into profiles/.
set -euo pipefail
TAG=${1:?tag}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
CMD=(python bench.py --steps 8 --warmup 2 --no-cpu --e2e-blocks 0)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- "${CMD[@]}" > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  name=$(echo "$grp" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "crc_files_kernel<1" -d "$OUT/pmc_$name" -o run \
    --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --e2e-blocks 0 > "$OUT/pmc_$name.json" 2> "$OUT/pmc_$name.err"
done
echo "profile $TAG done"
