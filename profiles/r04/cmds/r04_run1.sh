#!/usr/bin/env bash
# Round 4, first GPU call: the Zipf production-launch parity tests and the split
# tests under both unit orders, the segmented-compaction tests, then the
# SQ/TCP/TCC counter passes of the headline and Zipf.
set -u
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_zipf_parity.py tests/test_split_files.py \
  tests/test_compaction_kernels.py::test_product_segmented_compaction_toggle \
  > gpurun_out/r04/tests1b.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python tools/ab_inproc.py - 6 zipf > gpurun_out/r04/ab_zipf_forms.json 2> gpurun_out/r04/ab_zipf_forms.err
timeout -k 10 300 python tools/ab_inproc.py - 6 verify > gpurun_out/r04/ab_verify_forms.json 2> gpurun_out/r04/ab_verify_forms.err
bash tools/diag_r04a.sh
