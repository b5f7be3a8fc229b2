set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
SDO_STREAMS=8 timeout -k 10 400 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 0 --workload jmx --coalesce off --duration 20 > gpurun_out/conc_jmx_s8.json 2> gpurun_out/conc_jmx_s8.log &&
SDO_STREAMS=8 timeout -k 10 500 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 0 --workload jmx --coalesce off --duration 20 --prewarm 208 > gpurun_out/conc_jmx_s8_warm.json 2> gpurun_out/conc_jmx_s8_warm.log
