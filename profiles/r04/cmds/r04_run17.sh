#!/usr/bin/env bash
# Round 4: packet header parse with one 16-byte + one 4-byte load per frame --
# packet parity tests, then the packet line under rocprofv3 kernel-trace stats.
set -eu
O=gpurun_out/r04/run17
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_packet.py -m gpu > $O/test.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --workload packet --no-cpu --steps 8 --warmup 2 > $O/packet.json 2> $O/packet.err
timeout -k 10 300 python bench.py --workload packet > $O/packet_line.json 2> $O/packet_line.err
echo ALLDONE
