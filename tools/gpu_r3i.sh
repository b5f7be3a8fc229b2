#!/bin/bash
# GPU box: partition tests; Q18/Q13/Q16 at SF100 + kernel trace of Q18 and Q13; concurrency with
# per-execution server CPU accounting (fixed texts, coalescing off; 8 and 16 client processes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_partition.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_partition.log 2>&1 || { tail -60 gpurun_out/pytest_partition.log; exit 1; }
tail -3 gpurun_out/pytest_partition.log
SDO_BENCH_ONLY=Q18,Q13,Q16 timeout -k 10 400 python bench.py --model tpch22 --steps 5 --warmup 2 --verbose > gpurun_out/tpch22_long_i.json 2> gpurun_out/tpch22_long_i.err || { tail -30 gpurun_out/tpch22_long_i.err; exit 1; }
grep "\[bench\] Q" gpurun_out/tpch22_long_i.err
rm -rf gpurun_out/prof_q18i
cd /tmp && export TMPDIR=/tmp
SDO_BENCH_ONLY=Q18,Q13 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_q18i" -o run -- python3 "$R/bench.py" --model tpch22 --steps 3 --warmup 1 \
  > "$R/gpurun_out/prof_q18i.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_q18i.log"; exit 1; }
cd "$R"
DB=$(find gpurun_out/prof_q18i -name "*.db" | head -1)
python tools/rocpd_summary.py "$DB" --tail-ms 70 --top 30 --timeline-ms 1 > gpurun_out/prof_q18i_summary.txt
head -35 gpurun_out/prof_q18i_summary.txt
for PR in 8 16; do
timeout -k 10 200 python tools/concurrency_bench.py --sf 100 --clients 64 --procs $PR --qps 0 --duration 12 --warmup 3 --coalesce off > gpurun_out/conc_fixed_off_p$PR.json 2> gpurun_out/conc_fixed_off_p$PR.err || { tail -30 gpurun_out/conc_fixed_off_p$PR.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/conc_fixed_off_p$PR.json')); print($PR, d['executions_per_s'], d['p50_ms'], d['p99_ms'], d['server'])"
done
