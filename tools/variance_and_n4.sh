set -euo pipefail
mkdir -p gpurun_out/var
for i in 1 2 3 4; do
  timeout -k 10 200 python bench.py --no-cpu --e2e-blocks 0 --parity-every 1024 > gpurun_out/var/default_$i.json 2> gpurun_out/var/default_$i.err
done
TFS_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 4 --steps 4 --warmup 1 --blocks 256 --e2e-blocks 8 > gpurun_out/var/n4_shared.json 2> gpurun_out/var/n4_shared.err
echo var done
