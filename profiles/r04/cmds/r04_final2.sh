#!/usr/bin/env bash
# Round 4, closing tree after the measurement-variant work: the -m gpu suite,
# smoke and the default line.
set -u
O=gpurun_out/r04/${FINAL_DIR:-final2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/gputests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py > $O/default.json 2> $O/default.err || exit 4
timeout -k 10 300 python bench.py --workload compact_device > $O/compact_device.json 2> $O/compact_device.err || exit 5
echo ALLDONE
