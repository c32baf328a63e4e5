#!/usr/bin/env bash
# tools/ab_libs.sh ROUNDS LIB1,LIB2,... [bench args...] -- same-box A/B of several
# builds of libtfs_crc.so ("product" = tfs_amd/libtfs_crc.so), alternated ROUNDS
# times in separate processes on one GPU.  One JSON line per run in gpurun_out/ab_libs/.
set -euo pipefail
ROUNDS=${1:?rounds}; LIBS=${2:?libs}; shift 2
OUT=gpurun_out/ab_libs
mkdir -p "$OUT"
IFS=',' read -ra L <<< "$LIBS"
for r in $(seq 1 "$ROUNDS"); do
  for lib in "${L[@]}"; do
    tag=$(basename "$lib" .so)
    if [ "$lib" = product ]; then
      timeout -k 10 200 python bench.py "$@" > "$OUT/${tag}_$r.json" 2> "$OUT/${tag}_$r.err"
    else
      TFS_CRC_LIB="$lib" timeout -k 10 200 python bench.py "$@" > "$OUT/${tag}_$r.json" 2> "$OUT/${tag}_$r.err"
    fi
  done
done
echo "ab_libs done"
