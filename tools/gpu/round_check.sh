set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_async_compile.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
SDO_STREAMS=8 timeout -k 10 400 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 0 --workload jmx --coalesce off --duration 20 > gpurun_out/conc_jmx_s8.json 2> gpurun_out/conc_jmx_s8.log
