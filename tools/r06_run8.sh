#!/bin/bash
# Round 6 GPU pass 8: where configs[2]'s host-memory leg loses the last 6 % of
# H2D -- rocprofv3 kernel trace of the zipf_e2e line (launches, durations, gaps).
set -o pipefail
mkdir -p gpurun_out/r06/prof_zipf_e2e
O=gpurun_out/r06/prof_zipf_e2e
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python bench.py --workload zipf_e2e --e2e-blocks 64 > $O/bench.json 2> $O/bench.err
