set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu --ab 0,1,2,3,5,6 --ab-rounds 6 > gpurun_out/bench_ab.log 2> gpurun_out/bench_ab.err || exit 3
