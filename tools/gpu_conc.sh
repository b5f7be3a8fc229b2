#!/bin/bash
# GPU box: BASELINE config 5 -- 64 concurrent Thrift clients at several fixed rates + closed loop
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for QPS in ${QPS_LIST:-250 500 1000 0}; do
  timeout -k 10 200 python tools/concurrency_bench.py --sf ${SF:-100} --clients 64 --procs 16 --qps $QPS --duration ${DUR:-20} \
    > gpurun_out/conc_qps$QPS.json 2> gpurun_out/conc_qps$QPS.log || { tail -20 gpurun_out/conc_qps$QPS.log; exit 1; }
  cut -c1-400 gpurun_out/conc_qps$QPS.json
done
