set -o pipefail
mkdir -p gpurun_out/w



timeout -k 10 300 python bench.py --workload compact --compact-blocks 4096 > gpurun_out/w/compact.log 2> gpurun_out/w/compact.err || exit 4
timeout -k 10 300 python bench.py --workload e2e --compact-blocks 1024 > gpurun_out/w/e2e.log 2> gpurun_out/w/e2e.err || exit 5
TFS_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 8 --warmup 2 --blocks 512 > gpurun_out/w/verify_n2.log 2> gpurun_out/w/verify_n2.err || exit 6
