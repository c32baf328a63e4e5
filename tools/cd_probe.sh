set -e
mkdir -p gpurun_out/r02i
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --workload compact_device --membench --no-cpu > gpurun_out/r02i/cd.json 2> gpurun_out/r02i/cd.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02i/trace -o run --output-format csv -- python bench.py --workload compact_device --no-cpu --blocks 256 --steps 3 > gpurun_out/r02i/cd_trace.json 2> gpurun_out/r02i/cd_trace.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "compact_fused" -d gpurun_out/r02i/pmc_fetch -o run --output-format csv -- python bench.py --workload compact_device --no-cpu --blocks 256 --steps 2 --warmup 1 > gpurun_out/r02i/pmc_fetch.json 2> gpurun_out/r02i/pmc_fetch.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "compact_fused" -d gpurun_out/r02i/pmc_write -o run --output-format csv -- python bench.py --workload compact_device --no-cpu --blocks 256 --steps 2 --warmup 1 > gpurun_out/r02i/pmc_write.json 2> gpurun_out/r02i/pmc_write.err
echo done
