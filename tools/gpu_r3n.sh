#!/bin/bash
# GPU box: headline bench, TPC-H 22 sweep, SSB sweep at SF100 + kernel-time share of the 22 sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 170 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/bench1_n.json 2> gpurun_out/bench1_n.err || { tail -30 gpurun_out/bench1_n.err; exit 1; }
cut -c1-200 gpurun_out/bench1_n.json
timeout -k 10 170 python bench.py --model tpch22 --steps 2 --warmup 1 --verbose > gpurun_out/tpch22_n.json 2> gpurun_out/tpch22_n.err || { tail -30 gpurun_out/tpch22_n.err; exit 1; }
cut -c1-200 gpurun_out/tpch22_n.json
timeout -k 10 170 python bench.py --model ssb --steps 5 --warmup 2 --verbose > gpurun_out/ssb_n.json 2> gpurun_out/ssb_n.err || { tail -30 gpurun_out/ssb_n.err; exit 1; }
cut -c1-200 gpurun_out/ssb_n.json
rm -rf gpurun_out/prof_t22
cd /tmp && export TMPDIR=/tmp
timeout -k 10 170 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_t22" -o run -- python3 "$R/bench.py" --model tpch22 --steps 1 --warmup 1 > "$R/gpurun_out/prof_t22.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_t22.log"; exit 1; }
cd "$R"
DB=$(find gpurun_out/prof_t22 -name "*.db" | head -1)
python tools/rocpd_summary.py "$DB" --tail-ms 400 --top 30 --timeline-ms 1 > gpurun_out/prof_t22_summary.txt
rm -rf gpurun_out/prof_t22
head -34 gpurun_out/prof_t22_summary.txt
