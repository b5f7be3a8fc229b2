#!/bin/bash
# GPU box: server-side counters of the 64-client closed loop + cProfile of the headline host path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/concurrency_bench.py --sf 100 --clients 64 --procs 16 --qps 0 --duration 8 --warmup 2 \
  > gpurun_out/conc_closed_stats.json 2> gpurun_out/conc_closed_stats.log || { tail -20 gpurun_out/conc_closed_stats.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/conc_closed_stats.json')); print(d['achieved_qps'], d['p99_ms'], d['server'])"
timeout -k 10 300 python tools/host_profile.py --sf 100 --mode sql --steps 3 > gpurun_out/host_profile_sql.txt 2>&1 || { tail -20 gpurun_out/host_profile_sql.txt; exit 1; }
head -30 gpurun_out/host_profile_sql.txt
