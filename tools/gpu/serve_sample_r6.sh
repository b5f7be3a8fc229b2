# BASELINE config 5 at 250 QPS with the server threads' sampling profile (host CPU per statement)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
SDO_STREAMS=8 timeout -k 10 500 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps ${Q:-250} --workload jmx \
    --coalesce off --duration 20 --prewarm 208 --settle --timeline gpurun_out/r6/tl_sample$TAG.json \
    --sample gpurun_out/r6/sample_q${Q:-250}$TAG.txt \
    > gpurun_out/r6/conc_sample$TAG.json 2> gpurun_out/r6/conc_sample$TAG.log
