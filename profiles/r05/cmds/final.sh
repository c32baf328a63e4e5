#!/usr/bin/env bash
# Round 5, closing tree: the -m gpu suite, smoke, then every bench line at full
# default size (tools/all_lines.sh) on one box.
set -u
O=gpurun_out/r05/${FINAL_DIR:-final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/gputests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
tools/all_lines.sh $O/all_lines || exit 4
echo ALLDONE
