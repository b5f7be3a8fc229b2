# BASELINE config 5 cold closed loop at several execution-slot counts (SLOTS="8 10 12")
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
for S in ${SLOTS:-10 12}; do
  SDO_STREAMS=$S timeout -k 10 540 python -u tools/concurrency_bench.py --sf 100 --clients 64 --qps 0 --workload jmx \
      --coalesce off --duration 20 --timeline gpurun_out/r6/tl_cold_s$S.json \
      > gpurun_out/r6/conc_cold_s$S.json 2> gpurun_out/r6/conc_cold_s$S.log || exit $?
done
