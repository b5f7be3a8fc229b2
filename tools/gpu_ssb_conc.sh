#!/bin/bash
# GPU box: GPU tests + SSB bench (BASELINE config 4) + closed-loop Thrift concurrency sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python bench.py --model ssb --sf ${SSB_SF:-100} --steps 3 --warmup 1 --verbose \
  > gpurun_out/bench_ssb.json 2> gpurun_out/bench_ssb.log || { tail -30 gpurun_out/bench_ssb.log; exit 1; }
cut -c1-300 gpurun_out/bench_ssb.json
for C in ${CLIENTS_LIST:-1 8 64}; do
  P=$(( C < 16 ? C : 16 ))
  timeout -k 10 150 python tools/concurrency_bench.py --sf ${SF:-10} --clients $C --procs $P --qps 0 --duration ${DUR:-6} --warmup 2 \
    > gpurun_out/conc_closed_c$C.json 2> gpurun_out/conc_closed_c$C.log || { tail -20 gpurun_out/conc_closed_c$C.log; exit 1; }
  cut -c1-300 gpurun_out/conc_closed_c$C.json
done
