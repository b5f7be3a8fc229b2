#!/bin/bash
# GPU box: kernel trace of TPC-H Q18 at SF100 on the partitioned plan; concurrency bench with the
# fixed texts and coalescing off (server sampling profile), and the varied workload after a prewarm
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rm -rf gpurun_out/prof_q18
cd /tmp && export TMPDIR=/tmp
SDO_BENCH_ONLY=Q18 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_q18" -o run -- python3 "$R/bench.py" --model tpch22 --steps 3 --warmup 1 \
  > "$R/gpurun_out/prof_q18.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_q18.log"; exit 1; }
cd "$R"
DB=$(find gpurun_out/prof_q18 -name "*.db" | head -1)
python tools/rocpd_summary.py "$DB" --tail-ms 60 --top 30 --timeline-ms 40 > gpurun_out/prof_q18_summary.txt
head -45 gpurun_out/prof_q18_summary.txt
timeout -k 10 200 python tools/concurrency_bench.py --sf 100 --clients 64 --procs 8 --qps 0 --duration 15 --warmup 3 --coalesce off --sample gpurun_out/conc_fixed_off_sample.txt > gpurun_out/conc_fixed_off.json 2> gpurun_out/conc_fixed_off.err || { tail -30 gpurun_out/conc_fixed_off.err; exit 1; }
cut -c1-600 gpurun_out/conc_fixed_off.json
timeout -k 10 300 python tools/concurrency_bench.py --sf 100 --clients 64 --procs 8 --qps 0 --duration 15 --warmup 3 --workload varied --prewarm 2000 --coalesce off > gpurun_out/conc_varied_warm_off.json 2> gpurun_out/conc_varied_warm_off.err || { tail -30 gpurun_out/conc_varied_warm_off.err; exit 1; }
cut -c1-600 gpurun_out/conc_varied_warm_off.json
