#!/usr/bin/env bash
# tools/ab_lib.sh OLD_SO ROUNDS [bench args...] -- same-box A/B of two builds of
# libtfs_crc.so: the product build (tfs_amd/libtfs_crc.so) and OLD_SO (an older
# commit built into abtmp/), alternated ROUNDS times in separate processes on
# one GPU.  Output: one JSON line per run under gpurun_out/ab_lib/.
set -euo pipefail
OLD=${1:?old so}; ROUNDS=${2:-3}; shift 2
OUT=gpurun_out/ab_lib
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  timeout -k 10 200 python bench.py "$@" > "$OUT/new_$r.json" 2> "$OUT/new_$r.err"
  TFS_CRC_LIB="$OLD" timeout -k 10 200 python bench.py "$@" > "$OUT/old_$r.json" 2> "$OUT/old_$r.err"
done
echo "ab_lib done"
