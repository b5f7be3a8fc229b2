set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
SDO_STREAMS=8 timeout -k 10 500 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 0 --workload jmx --coalesce off --duration 20 --prewarm 208 > gpurun_out/conc_jmx_s8_warm.json 2> gpurun_out/conc_jmx_s8_warm.log &&
SDO_STREAMS=8 timeout -k 10 500 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 100 --workload jmx --coalesce off --duration 20 --prewarm 208 > gpurun_out/conc_jmx_s8_q100.json 2> gpurun_out/conc_jmx_s8_q100.log
