set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python bench.py --steps 8 --warmup 2 --cpu-seconds 5 > gpurun_out/prof/bench_trace.log 2> gpurun_out/prof/bench_trace.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex crc_files_kernel -d gpurun_out/prof/fetch -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/prof/bench_fetch.log 2> gpurun_out/prof/bench_fetch.err || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex crc_files_kernel -d gpurun_out/prof/write -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/prof/bench_write.log 2> gpurun_out/prof/bench_write.err || exit 3
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex crc_files_kernel -d gpurun_out/prof/rdreq -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/prof/bench_rdreq.log 2> gpurun_out/prof/bench_rdreq.err || exit 4
