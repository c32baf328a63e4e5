#!/usr/bin/env bash
# Round 5: the driver's own round-end sequence on the closing tree -- the -m gpu suite,
# smoke, `python3 bench.py --gpus 1 --steps 20 --warmup 5` -- and the same bench
# command under rocprofv3 --kernel-trace --stats.
set -u
O=gpurun_out/r05/driver_like
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 $O/gputests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_rocprof.json 2> $O/bench_rocprof.err || exit 5
echo ALLDONE
