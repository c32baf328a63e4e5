#!/usr/bin/env bash
# tools/combine_probe.sh -- on the GPU box: product vs no-combine diagnostic build
# of libtfs_crc.so, alternating in one call (both built here beforehand:
# abtmp/diag/libtfs_crc.so from -DTFS_DIAG_SKIP_COMBINE).  Restores the product .so.
set -euo pipefail
OUT=gpurun_out/combine_probe
mkdir -p "$OUT"
cp tfs_amd/libtfs_crc.so "$OUT/product.so"
for r in 1 2 3; do
  cp "$OUT/product.so" tfs_amd/libtfs_crc.so
  timeout -k 10 120 python tools/combine_probe.py product >> "$OUT/probe.jsonl"
  cp abtmp/diag/libtfs_crc.so tfs_amd/libtfs_crc.so
  timeout -k 10 120 python tools/combine_probe.py no_combine >> "$OUT/probe.jsonl"
done
cp "$OUT/product.so" tfs_amd/libtfs_crc.so
rm -f "$OUT/product.so"
echo "combine probe done"
