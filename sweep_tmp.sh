set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 8 --warmup 2 --membench --no-cpu > gpurun_out/bench_v0.log 2> gpurun_out/bench_v0.err || exit 2
for v in 1 2 3 4 5 6; do
  TFS_CRC_VARIANT=$v timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu > gpurun_out/bench_v$v.log 2> gpurun_out/bench_v$v.err || exit 3
done
