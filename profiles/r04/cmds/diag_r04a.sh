set -e
O=gpurun_out/r04/pmc
tools/pmc_passes.sh $O verify "crc_files_kernel<1" -- python bench.py --steps 2 --warmup 1 --no-cpu --e2e-blocks 0 --parity-every 1024
tools/pmc_passes.sh $O zipf "crc_files_kernel<0|split_" -- python bench.py --workload zipf --no-cpu --steps 2 --warmup 1
echo ALLDONE
