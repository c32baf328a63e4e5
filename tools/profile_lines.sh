#!/usr/bin/env bash
# tools/profile_lines.sh -- rocprofv3 passes for a round's profiles (run on the
# GPU box through gpurun): kernel trace + stats of each bench command, then each
# PMC group in its own pass (FETCH_SIZE and WRITE_SIZE cannot share one; counters
# never combined with other trace domains).  Outputs under OUTDIR;
# tools/pmc_summary.py folds them into profiles/rNN/.
# Usage: tools/profile_lines.sh [all|compact|verify|bverify|zipf|packet|ec] OUTDIR
set -euo pipefail
PART=${1:-all}
OUT=${2:-gpurun_out/prof_r02}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
run_trace() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$name/trace" -o run --output-format csv -- \
    python bench.py "$@" > "$OUT/$name/bench_trace.json" 2> "$OUT/$name/trace.err"
}
run_pmc() {  # name, counters, kernel regex, bench args...
  local name=$1 ctrs=$2 kre=$3; shift 3
  local tag
  tag=$(echo "$ctrs" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "$kre" -d "$OUT/$name/pmc_$tag" -o run \
    --output-format csv -- python bench.py "$@" > "$OUT/$name/pmc_$tag.json" 2> "$OUT/$name/pmc_$tag.err"
}
mkdir -p "$OUT/verify" "$OUT/compact" "$OUT/bverify"
H=(--steps 8 --warmup 2 --no-cpu --e2e-blocks 0 --parity-every 1024)
if [[ $PART == all || $PART == verify ]]; then
run_trace verify "${H[@]}"
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  run_pmc verify "$grp" "crc_files_kernel<1" --steps 2 --warmup 1 --no-cpu --e2e-blocks 0 --parity-every 1024
done
fi
# the record kernel's product instantiations carry DIAG = kCompactDiag (12)
if [[ $PART == all || $PART == compact ]]; then
C=(--workload compact_device --no-cpu --steps 4 --warmup 1)
run_trace compact "${C[@]}"
for grp in FETCH_SIZE WRITE_SIZE; do run_pmc compact "$grp" "compact_pipe_kernel<true, true, false, 12, 5, 1, 0" --workload compact_device --no-cpu --steps 1 --warmup 1; done
fi
if [[ $PART == all || $PART == bverify ]]; then
B=(--workload block_verify_device --no-cpu --steps 4 --warmup 1)
run_trace bverify "${B[@]}"
for grp in FETCH_SIZE WRITE_SIZE; do run_pmc bverify "$grp" "compact_pipe_kernel<true, true, true, 12, 5, 4, 3" --workload block_verify_device --no-cpu --steps 1 --warmup 1; done
fi
mkdir -p "$OUT/zipf" "$OUT/packet" "$OUT/ec"
if [[ $PART == all || $PART == zipf ]]; then
Z=(--workload zipf --no-cpu --steps 4 --warmup 1)
run_trace zipf "${Z[@]}"
for grp in FETCH_SIZE WRITE_SIZE; do run_pmc zipf "$grp" "crc_files_kernel<0" --workload zipf --no-cpu --steps 1 --warmup 1; done
fi
if [[ $PART == all || $PART == packet ]]; then
P=(--workload packet --no-cpu --steps 4 --warmup 1)
run_trace packet "${P[@]}"
for grp in FETCH_SIZE WRITE_SIZE; do run_pmc packet "$grp" "packet_parse_kernel|crc_files_kernel<1|packet_finish_kernel" --workload packet --no-cpu --steps 1 --warmup 1; done
fi
if [[ $PART == all || $PART == ec ]]; then
E=(--workload ec --no-cpu --steps 4 --warmup 1)
run_trace ec "${E[@]}"
for grp in FETCH_SIZE WRITE_SIZE; do run_pmc ec "$grp" "ec_apply_kernel<3>" --workload ec --no-cpu --steps 1 --warmup 1; done
fi
echo "profile_lines done"
