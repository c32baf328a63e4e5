#!/usr/bin/env bash
# Round 4, first GPU call: the new Zipf production-launch parity tests and the
# split/stream tests, then the SQ/TCP/TCC counter passes of the headline and Zipf.
set -u
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_zipf_parity.py tests/test_split_files.py tests/test_scalar_and_streams.py \
  tests/test_compaction_kernels.py::test_jobs_device_statuses_and_split_records \
  tests/test_compaction_kernels.py::test_jobs_device_many_blocks_shuffled \
  > gpurun_out/r04/tests1.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
bash tools/diag_r04a.sh
