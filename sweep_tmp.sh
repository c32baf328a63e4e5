set -o pipefail
mkdir -p gpurun_out/w
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu --ab 0,1,2,5 --ab-rounds 5 > gpurun_out/w/ab_verify.log 2> gpurun_out/w/ab_verify.err || exit 2
timeout -k 10 300 python bench.py --workload zipf --steps 4 --warmup 1 --ab 0,2,5 --ab-rounds 5 > gpurun_out/w/ab_zipf.log 2> gpurun_out/w/ab_zipf.err || exit 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "crc_files_kernel<1" -d gpurun_out/w/fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu > /dev/null 2> gpurun_out/w/fetch.err || exit 4
