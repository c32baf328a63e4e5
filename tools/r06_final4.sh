#!/bin/bash
# Round 6 closing pass 4 on the final tree (device-memory ring): the driver's sequence (GPU suite, smoke,
# `python3 bench.py --gpus 1 --steps 20 --warmup 5`), the same bench command under
# rocprofv3 --kernel-trace --stats, the headline kernel's PMC passes (FETCH_SIZE,
# WRITE_SIZE, TCC EA requests; each group in a run of its own), then every line at
# full size (tools/all_lines.sh).
set -o pipefail
O=gpurun_out/r06/final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_rocprof.json 2> $O/bench_rocprof.err &&
PMC_GROUPS=fetch,write,tccw tools/pmc_passes.sh $O/pmc verify "crc_files_kernel<1, 4, 3>" -- python bench.py --steps 4 --warmup 1 --no-cpu --e2e-blocks 0 --parity-every 1024 &&
bash tools/all_lines.sh $O/all_lines &&
g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe &&
timeout -k 10 200 tools/floor_probe 400 > $O/floor_probe.json 2> $O/floor_probe.err &&
timeout -k 10 120 tools/latency_probe 400 > $O/latency_probe.json 2> $O/latency_probe.err
