#!/usr/bin/env bash
# tools/all_lines.sh OUTDIR -- every bench.py line at its default (full) size,
# one after another on one GPU; JSON lines into OUTDIR (under gpurun_out/).
set -uo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed rc=$?"; return 1; }
}
run default && run zipf --workload zipf && run zipf_e2e --workload zipf_e2e && run packet --workload packet && run compact_device --workload compact_device \
  && run block_verify_device --workload block_verify_device && run compact --workload compact \
  && run block_verify --workload block_verify && run e2e --workload e2e && run ec --workload ec \
  && run compact_files --workload compact_files \
  && run loopback --workload loopback && run small_bodies --workload small_bodies
echo "all_lines done"
