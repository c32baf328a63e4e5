#!/usr/bin/env bash
# Round 5, run 12: host block verify completes on a page-locked flag (the record
# kernel's last workgroup stores it) instead of a stream sync: the whole -m gpu
# suite (the record kernel's signature changed), the host-path A/B, the block
# verify and loopback lines.
set -u
O=gpurun_out/r05/run12
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/gputests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 500 python -u tools/ab_host_paths.py 5 128 > $O/ab_host.json 2> $O/ab_host.err || exit 5
timeout -k 10 300 python -u bench.py --workload block_verify > $O/block_verify.json 2> $O/block_verify.err || exit 6
timeout -k 10 300 python -u bench.py --workload loopback > $O/loopback.json 2> $O/loopback.err || exit 7
echo ALLDONE
