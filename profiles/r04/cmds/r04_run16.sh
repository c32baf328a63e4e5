#!/usr/bin/env bash
# Round 4: instruction-fetch counters of the compaction kernel (37 KB of code)
# against the verify kernel (20 KB): which SQC/IFETCH counters the box offers,
# then one --pmc pass per kernel line with those available.
set -u
O=gpurun_out/r04/run16
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
C=""
for c in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQC_ICACHE_REQ SQ_INSTS_VALU; do
  if grep -qw "$c" $O/avail.txt; then C="$C $c"; fi
done
echo "counters:$C"
[[ -n "$C" ]] || exit 0
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex "compact_pipe_kernel<true, true, false" -d $O/compact -o run --output-format csv -- python bench.py --workload compact_device --no-cpu --steps 3 --warmup 1 > $O/compact.out 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex "crc_files_kernel<1" -d $O/verify -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --e2e-blocks 0 --parity-every 1024 > $O/verify.out 2>&1 || exit 5
echo ALLDONE
