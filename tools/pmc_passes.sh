#!/usr/bin/env bash
# tools/pmc_passes.sh OUTDIR NAME KERNEL_REGEX -- CMD...   (run on the GPU box via gpurun)
#
# One rocprofv3 kernel-trace + stats pass of CMD, then every counter group below
# in a run of its own (rocprofv3 does not split counters over passes; per-block
# limits: 8 SQ, 4 TCC, 4 TCP, 2 TA, 2 GRBM; counters never combined with other
# trace domains).  Raw CSVs land under OUTDIR/NAME/; tools/pmc_fold.py folds them.
# PMC_GROUPS=sq1,sq2,tcp,tccw,fetch,write,tccs selects groups (default: all).
set -euo pipefail
OUT=$1; NAME=$2; KRE=$3; shift 3
[[ ${1:-} == "--" ]] && shift
D="$OUT/$NAME"
mkdir -p "$D"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
declare -A G=(
  [sq1]="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
  [sq2]="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  [tcp]="TCP_UTCL1_TRANSLATION_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_REQUEST_sum TA_BUSY_avr GRBM_GUI_ACTIVE"
  [tccw]="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
  [fetch]="FETCH_SIZE"
  [write]="WRITE_SIZE"
  [tccs]="TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum"
)
PGROUPS=${PMC_GROUPS:-sq1,sq2,tcp,tccw,fetch,write,tccs}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$D/trace" -o run --output-format csv -- "$@" \
  > "$D/trace.out" 2> "$D/trace.err"
for g in ${PGROUPS//,/ }; do
  timeout -s KILL 150 rocprofv3 --pmc ${G[$g]} --kernel-include-regex "$KRE" -d "$D/pmc_$g" -o run \
    --output-format csv -- "$@" > "$D/pmc_$g.out" 2> "$D/pmc_$g.err"
  echo "$NAME $g done"
done
