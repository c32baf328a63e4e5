#!/usr/bin/env bash
# Round 5, run 13: resident units cut into 16 KiB segments (a 64 KiB close read by
# four workgroups at once): the resident and latency tests, then the loopback and
# small-body lines with segments (default) and with whole files
# (TFS_CRC_RESIDENT_SEG_KIB=0), alternating, two processes each.
set -u
O=gpurun_out/r05/run13
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_resident.py tests/test_latency_form.py tests/test_ds_harness.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --workload loopback --no-cpu > $O/loop_seg_$r.json 2> $O/loop_seg_$r.err || exit 5
  TFS_CRC_RESIDENT_SEG_KIB=0 timeout -k 10 300 python -u bench.py --workload loopback --no-cpu > $O/loop_whole_$r.json 2> $O/loop_whole_$r.err || exit 6
  timeout -k 10 300 python -u bench.py --workload small_bodies > $O/small_seg_$r.json 2> $O/small_seg_$r.err || exit 7
  TFS_CRC_RESIDENT_SEG_KIB=0 timeout -k 10 300 python -u bench.py --workload small_bodies > $O/small_whole_$r.json 2> $O/small_whole_$r.err || exit 8
done
echo ALLDONE
