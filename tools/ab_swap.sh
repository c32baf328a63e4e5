#!/usr/bin/env bash
# tools/ab_swap.sh ROUNDS TAG1,TAG2,... CMD... -- same-box A/B of builds of
# libtfs_crc.so that the dataserver library (tfs_amd/ds/libtfs_ds.so, linked to
# tfs_amd/libtfs_crc.so) must load too: abtmp/TAG/libtfs_crc.so is copied over the
# product file before each run, TAGs alternated ROUNDS times in separate
# processes; the product file is restored at the end.  CMD's stdout goes to
# gpurun_out/ab_swap/<CMD as a name>/TAG_ROUND.json.  Measurement only (the GPU
# box's scratch copy).
set -euo pipefail
ROUNDS=${1:?rounds}; TAGS=${2:?tags}; shift 2
OUT="gpurun_out/ab_swap/$(echo "$*" | tr -c 'A-Za-z0-9' '_' | cut -c1-60)"
mkdir -p "$OUT"
cp tfs_amd/libtfs_crc.so abtmp/.product.so
trap 'cp abtmp/.product.so tfs_amd/libtfs_crc.so' EXIT
IFS=',' read -ra T <<< "$TAGS"
for r in $(seq 1 "$ROUNDS"); do
  for tag in "${T[@]}"; do
    cp "abtmp/$tag/libtfs_crc.so" tfs_amd/libtfs_crc.so
    timeout -k 10 200 "$@" > "$OUT/${tag}_$r.json" 2> "$OUT/${tag}_$r.err"
  done
done
echo "ab_swap done"
