#!/bin/bash
# GPU box: server statement profile; concurrency (fixed / varied, coalescing off) with 4 and 8 streams
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 170 python tools/server_profile.py --sf 10 --iters 40 --top 45 > gpurun_out/server_profile.txt 2>&1 || { tail -30 gpurun_out/server_profile.txt; exit 1; }
grep statements gpurun_out/server_profile.txt
for ST in 4 8; do
for W in fixed varied; do
SDO_STREAMS=$ST timeout -k 10 170 python tools/concurrency_bench.py --sf 100 --clients 64 --procs 8 --qps 0 --duration 12 --warmup 3 --workload $W --coalesce off > gpurun_out/conc_${W}_off_s$ST.json 2> gpurun_out/conc_${W}_off_s$ST.err || { tail -30 gpurun_out/conc_${W}_off_s$ST.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/conc_${W}_off_s$ST.json')); print('$W streams=$ST', d['executions_per_s'], d['p50_ms'], d['p99_ms'], d['server'])"
done
done
