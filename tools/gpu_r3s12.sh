#!/bin/bash
# GPU box: concurrency bench on the current tree -- 64 Thrift clients at SF100, identical-statement
# sharing off, fixed benchmark texts and the varied parameterized workload
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/concurrency_bench.py --sf 100 --clients 64 --procs 8 --qps 0 --duration 15 --warmup 3 --coalesce off > gpurun_out/conc_fixed_off_s12.json 2> gpurun_out/conc_fixed_off_s12.err || { tail -30 gpurun_out/conc_fixed_off_s12.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/conc_fixed_off_s12.json')); print('fixed', d['executions_per_s'], d['p50_ms'], d['p99_ms'], d['server'])"
timeout -k 10 200 python tools/concurrency_bench.py --sf 100 --clients 64 --procs 8 --qps 0 --duration 15 --warmup 3 --workload varied --coalesce off > gpurun_out/conc_varied_off_s12.json 2> gpurun_out/conc_varied_off_s12.err || { tail -30 gpurun_out/conc_varied_off_s12.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/conc_varied_off_s12.json')); print('varied', d['executions_per_s'], d['p50_ms'], d['p99_ms'], d['server'])"
