# BASELINE config 5 on one MI355X (verdict r5 #1 / #2): the reference's JMeter BI plan over the
# HiveServer2 endpoint, 64 clients, 8 execution slots, background compiles on (the default).
#   1. cold: one text per template prewarmed, first-seen shapes run on interim plans while they compile
#   2. open loop at 250 QPS, every text prewarmed, with the per-statement phase timeline
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
SDO_STREAMS=8 timeout -k 10 540 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 0 --workload jmx \
    --coalesce off --duration 20 --timeline gpurun_out/r6/tl_cold.json \
    > gpurun_out/r6/conc_cold.json 2> gpurun_out/r6/conc_cold.log &&
SDO_STREAMS=8 timeout -k 10 540 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 250 --workload jmx \
    --coalesce off --duration 20 --prewarm 208 --timeline gpurun_out/r6/tl_q250.json \
    > gpurun_out/r6/conc_q250.json 2> gpurun_out/r6/conc_q250.log
