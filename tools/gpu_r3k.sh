#!/bin/bash
# GPU box: server-side cost of one statement (cProfile, 1 executor, 1 client) at SF10, then the
# concurrency bench (fixed texts and the varied workload, coalescing off) at SF100
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 170 python tools/server_profile.py --sf 10 --iters 40 --top 45 > gpurun_out/server_profile.txt 2>&1 || { tail -30 gpurun_out/server_profile.txt; exit 1; }
head -3 gpurun_out/server_profile.txt
timeout -k 10 170 python tools/concurrency_bench.py --sf 100 --clients 64 --procs 8 --qps 0 --duration 12 --warmup 3 --coalesce off > gpurun_out/conc_fixed_off_k.json 2> gpurun_out/conc_fixed_off_k.err || { tail -30 gpurun_out/conc_fixed_off_k.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/conc_fixed_off_k.json')); print('fixed', d['executions_per_s'], d['p50_ms'], d['p99_ms'], d['server'])"
timeout -k 10 170 python tools/concurrency_bench.py --sf 100 --clients 64 --procs 8 --qps 0 --duration 12 --warmup 3 --workload varied --coalesce off > gpurun_out/conc_varied_off_k.json 2> gpurun_out/conc_varied_off_k.err || { tail -30 gpurun_out/conc_varied_off_k.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/conc_varied_off_k.json')); print('varied', d['executions_per_s'], d['p50_ms'], d['p99_ms'], d['server'])"
