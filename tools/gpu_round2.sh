#!/bin/bash
# GPU box: tests, TPC-H + SSB benches, SF100 Thrift concurrency, SSB kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --verbose > gpurun_out/bench_tpch.json 2> gpurun_out/bench_tpch.log \
  || { tail -30 gpurun_out/bench_tpch.log; exit 1; }
cut -c1-250 gpurun_out/bench_tpch.json
timeout -k 10 300 python bench.py --model ssb --sf 100 --steps 3 --warmup 1 --verbose > gpurun_out/bench_ssb.json 2> gpurun_out/bench_ssb.log \
  || { tail -30 gpurun_out/bench_ssb.log; exit 1; }
grep "\[bench\] " gpurun_out/bench_ssb.log
cut -c1-250 gpurun_out/bench_ssb.json
timeout -k 10 150 python tools/concurrency_bench.py --sf 100 --clients 64 --procs 16 --qps 0 --duration 8 --warmup 2 \
  > gpurun_out/conc100_closed_c64.json 2> gpurun_out/conc100_closed_c64.log || { tail -20 gpurun_out/conc100_closed_c64.log; exit 1; }
cut -c1-300 gpurun_out/conc100_closed_c64.json
timeout -k 10 150 python tools/concurrency_bench.py --sf 100 --clients 64 --procs 16 --qps 250 --duration 10 --warmup 2 \
  > gpurun_out/conc100_qps250.json 2> gpurun_out/conc100_qps250.log || { tail -20 gpurun_out/conc100_qps250.log; exit 1; }
cut -c1-300 gpurun_out/conc100_qps250.json
rm -rf gpurun_out/prof_ssb
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ssb -o ssb -- python bench.py --model ssb --sf 100 --steps 2 --warmup 1 \
  > gpurun_out/prof_ssb.log 2>&1 || { tail -20 gpurun_out/prof_ssb.log; exit 1; }
find gpurun_out/prof_ssb -name "*kernel_stats.csv" | head -3
