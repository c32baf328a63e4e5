set -o pipefail
mkdir -p gpurun_out/prof2
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit 1
for v in 0 1 2 3 4 5 6; do
  TFS_CRC_VARIANT=$v timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu > gpurun_out/bench_v$v.log 2> gpurun_out/bench_v$v.err || exit 3
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex "crc_files_kernel<1" -d gpurun_out/prof2/sq1 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu > /dev/null 2> gpurun_out/prof2/sq1.err || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-include-regex "crc_files_kernel<1" -d gpurun_out/prof2/sq2 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu > /dev/null 2> gpurun_out/prof2/sq2.err || exit 5
