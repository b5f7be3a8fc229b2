set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_sketch_rollup.py tests/test_gpu_partition.py tests/test_gpu_theta.py tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_part_stored.log 2>&1
