#!/usr/bin/env bash
# Round 5, run 5: small-body latency; kernel traces of the
# packet and verify lines on one box (where the packet line's time goes, item 6).
set -u
O=${RUN5_OUT:-gpurun_out/r05/run5}
mkdir -p $O
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 python -u bench.py --workload small_bodies > $O/small_bodies.json 2> $O/small_bodies.err || exit 4
for w in verify packet; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$w -o run --output-format csv -- \
    python bench.py --workload $w --steps 8 --warmup 2 --no-cpu --e2e-blocks 0 --parity-every 1024 \
    > $O/trace_$w.json 2> $O/trace_$w.err || exit 5
done
echo ALLDONE
