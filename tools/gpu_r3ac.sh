#!/bin/bash
# GPU box: whole-chunk fast path -- kernel tests, A/B kernel times, headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_hllcode.py tests/test_gpu_partition.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_full.log 2>&1 || { tail -40 gpurun_out/t_full.log; exit 1; }
tail -2 gpurun_out/t_full.log
for F in 0 1; do
SDO_JIT_FULL=$F timeout -k 10 300 python tools/query_probe.py 100 reg0pipe0 -- "Basic Aggregation" "Ship Date Range" "TPCH Q1" "x:count-only" "x:nodims-count" "x:sum-ext" "x:no-hll" > gpurun_out/full$F.txt 2>&1 || { tail -30 gpurun_out/full$F.txt; exit 1; }
echo "full=$F"; grep "med" gpurun_out/full$F.txt | cut -c1-75
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/h_full.json 2> gpurun_out/h_full.err || { tail -30 gpurun_out/h_full.err; exit 1; }
cat gpurun_out/h_full.json
