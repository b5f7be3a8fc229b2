# BASELINE config 5, cold start (verdict r5 #1): the reference's JMeter BI plan over the HiveServer2
# endpoint, 64 clients, 8 execution slots, one text per template prewarmed, background compiles on
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
SDO_STREAMS=8 timeout -k 10 540 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 0 --workload jmx \
    --coalesce off --duration 20 --timeline gpurun_out/r6/tl_cold.json \
    > gpurun_out/r6/conc_cold.json 2> gpurun_out/r6/conc_cold.log
