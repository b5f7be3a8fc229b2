# BASELINE config 5 cold start: where the closed loop's first burst of first-seen texts goes.
# The timeline keeps the warm-up seconds; the sampling profile covers them only.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
timeout -k 10 540 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 0 --workload jmx \
    --coalesce off --duration 10 --timeline gpurun_out/r6/tl_burst.json --include-warmup \
    --sample gpurun_out/r6/sample_burst.txt > gpurun_out/r6/conc_burst.json 2> gpurun_out/r6/conc_burst.log
