#!/bin/bash
# Round 6 GPU pass 13: NUMA-bound latency A/B of three libraries (this tree,
# abtmp/r06a = junk refills, abtmp/r05 = the round-5 closing tree), 4 rounds in
# rotating order, one process each.
set -o pipefail
mkdir -p gpurun_out/r06/pass13
O=gpurun_out/r06/pass13
run() { timeout -k 10 120 tools/latency_probe$2 400 > $O/$1_$3.json 2> $O/$1_$3.err; }
for r in 1 2 3 4; do
  case $r in
    1|4) run new "" $r && run r06a _r06a $r && run r05 _r05 $r ;;
    2) run r06a _r06a $r && run r05 _r05 $r && run new "" $r ;;
    3) run r05 _r05 $r && run new "" $r && run r06a _r06a $r ;;
  esac || exit 1
done
