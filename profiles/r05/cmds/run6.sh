#!/usr/bin/env bash
# Round 5, run 6: one-pass packets (packet tests, the same-process A/B against the
# three-launch form and a plain verify of the same bodies, the packet line);
# blocks per launch of zero-copy host compaction; the compaction A/B with the
# dense 64 KiB-aligned layout (where the record list costs).
set -u
O=gpurun_out/r05/run6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_packet.py tests/test_split_files.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 400 python -u tools/ab_packet.py 6 > $O/ab_packet.json 2> $O/ab_packet.err || exit 5
timeout -k 10 300 python -u bench.py --workload packet > $O/packet.json 2> $O/packet.err || exit 6
timeout -k 10 300 python -u bench.py > $O/default.json 2> $O/default.err || exit 7
timeout -k 10 400 python -u tools/compact_group_probe.py 512 3 > $O/group.json 2> $O/group.err || exit 8
AB_ALIGNED=1 AB_VARIANTS=26,68 timeout -k 10 500 python -u tools/ab_compact.py 4 > $O/ab_compact.json 2> $O/ab_compact.err || exit 9
echo ALLDONE
