# BASELINE config 5, cold start (verdict r5 #1): the reference's JMeter BI plan over the HiveServer2
# endpoint, 64 clients, 8 execution slots, one text per template prewarmed, background compiles on.
# EXTRA="--settle" adds the server's warm-up step (its compiles finish, slot memory presized);
# TAG names the outputs.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
T=${TAG:-cold}
timeout -k 10 540 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 0 --workload jmx \
    --coalesce off --duration 20 --timeline gpurun_out/r6/tl_$T.json $EXTRA \
    > gpurun_out/r6/conc_$T.json 2> gpurun_out/r6/conc_$T.log
