# BASELINE config 5, open loop (verdict r5 #2): the reference's JMeter BI plan at a fixed aggregate
# rate, every text prewarmed, 8 execution slots, per-statement phase timeline.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
for Q in ${QPS_LIST:-250 400}; do
  SDO_STREAMS=8 timeout -k 10 500 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps $Q --workload jmx \
      --coalesce off --duration 20 --prewarm 208 ${SETTLE---settle} --timeline gpurun_out/r6/tl_q$Q$TAG.json \
      > gpurun_out/r6/conc_q$Q$TAG.json 2> gpurun_out/r6/conc_q$Q$TAG.log || exit $?
done
