#!/usr/bin/env bash
# Round 5, run 7: host compaction at 64 blocks per launch (the group test at 64 and 8),
# blocks per launch 16..256, then the PMC passes of every device-resident line
# on the pruned kernel set (profiles/r05/cmds/pmc.sh).
# (As run: bash ignores an assignment to GROUPS, so the probe ran its default
# list 1..64; the probe now reads CG_GROUPS.)
set -u
O=gpurun_out/r05/run7
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "blocks_compact" -m gpu -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
GROUPS=16,64,128,256 timeout -k 10 400 python -u tools/compact_group_probe.py 1024 3 > $O/group.json 2> $O/group.err || exit 8
bash profiles/r05/cmds/pmc.sh || exit 9
echo ALLDONE
