# Fixed-QPS stall attribution (verdict r5 #2): the BI plan at 250 QPS with the per-statement timeline
# (allocator free-everything-and-retry count per statement), default allocator vs expandable segments.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
SDO_STREAMS=8 timeout -k 10 500 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 250 --workload jmx \
    --coalesce off --duration 20 --prewarm 208 --timeline gpurun_out/r6/tl_q250_b.json \
    > gpurun_out/r6/conc_q250_b.json 2> gpurun_out/r6/conc_q250_b.log &&
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True SDO_STREAMS=8 timeout -k 10 500 python -u tools/concurrency_bench.py \
    --sf 100 --clients 64 --qps 250 --workload jmx --coalesce off --duration 20 --prewarm 208 \
    --timeline gpurun_out/r6/tl_q250_exp.json > gpurun_out/r6/conc_q250_exp.json 2> gpurun_out/r6/conc_q250_exp.log
