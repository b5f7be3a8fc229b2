#!/bin/bash
# GPU box: kernel trace of TPC-H Q19 / Q21 / Q2 at SF100 (regression hunt)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_q19
cd /tmp && export TMPDIR=/tmp
SDO_BENCH_ONLY=Q19,Q21,Q2 timeout -k 10 170 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_q19" -o run -- python3 "$R/bench.py" --model tpch22 --steps 2 --warmup 1 --verbose > "$R/gpurun_out/prof_q19.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_q19.log"; exit 1; }
cd "$R"
grep "\[bench\] Q" gpurun_out/prof_q19.log
DB=$(find gpurun_out/prof_q19 -name "*.db" | head -1)
python tools/rocpd_summary.py "$DB" --tail-ms 35 --top 25 --timeline-ms 35 > gpurun_out/prof_q19_summary.txt
rm -rf gpurun_out/prof_q19
head -28 gpurun_out/prof_q19_summary.txt
