#!/bin/bash
# Round 6 GPU pass 12: latency form without junk refills -- parity, then the
# same-box latency A/B: this tree, the previous commit (abtmp/r06a: junk refills)
# and the round-5 library (abtmp/r05), alternating.
set -o pipefail
mkdir -p gpurun_out/r06/pass12
O=gpurun_out/r06/pass12
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_latency_form.py \
  tests/test_resident.py tests/test_gpu_parity.py tests/test_packet.py > $O/tests.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 120 tools/latency_probe 400 > $O/new_$r.json 2> $O/new_$r.err &&
  timeout -k 10 120 tools/latency_probe_r06a 400 > $O/r06a_$r.json 2> $O/r06a_$r.err &&
  timeout -k 10 120 tools/latency_probe_r05 400 > $O/r05_$r.json 2> $O/r05_$r.err || exit 1
done
