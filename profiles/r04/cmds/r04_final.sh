#!/usr/bin/env bash
# Round 4, closing tree: the -m gpu suite, smoke, then every bench line at full
# default size (tools/all_lines.sh) on one box.
set -u
O=gpurun_out/r04/${FINAL_DIR:-final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/gputests.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
tools/all_lines.sh $O/all_lines || exit 4
echo ALLDONE
