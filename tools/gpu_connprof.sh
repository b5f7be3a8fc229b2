#!/bin/bash
# GPU box: sampling profile of the Thrift server threads under the 64-client closed loop
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/concurrency_bench.py --sf ${SF:-100} --clients 64 --procs 16 --qps 0 --duration 8 --warmup 2 \
  --sample gpurun_out/conc_sample.txt > gpurun_out/conc_sample.json 2> gpurun_out/conc_sample.log || { tail -20 gpurun_out/conc_sample.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/conc_sample.json')); print(d['achieved_qps'], d['p99_ms'], d['server'])"
