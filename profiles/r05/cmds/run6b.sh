#!/usr/bin/env bash
# Round 5, run 6b: run 6 after its tests passed (profiles/r05/packet_traces/tests_run6.log)
# and its packet A/B stopped on the seed of the verify leg: the packet A/B, the packet
# and default lines, blocks per launch of host compaction, the aligned compaction A/B.
set -u
O=gpurun_out/r05/run6b
mkdir -p $O
timeout -k 10 400 python -u tools/ab_packet.py 6 > $O/ab_packet.json 2> $O/ab_packet.err || exit 5
timeout -k 10 300 python -u bench.py --workload packet > $O/packet.json 2> $O/packet.err || exit 6
timeout -k 10 300 python -u bench.py > $O/default.json 2> $O/default.err || exit 7
timeout -k 10 400 python -u tools/compact_group_probe.py 512 3 > $O/group.json 2> $O/group.err || exit 8
AB_ALIGNED=1 AB_VARIANTS=26,68 timeout -k 10 500 python -u tools/ab_compact.py 4 > $O/ab_compact.json 2> $O/ab_compact.err || exit 9
echo ALLDONE
