set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "blocks_compact" tests/test_compaction_kernels.py > gpurun_out/r06_t1.log 2>&1
