#!/bin/bash
# GPU box: HLL code planes -- kernel tests, Q1-shaped kernel times, headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
timeout -k 10 300 python -u -m pytest tests/test_hllcode.py tests/test_sketch_rollup.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_hllcode.log 2>&1 || { tail -40 gpurun_out/t_hllcode.log; exit 1; }
tail -2 gpurun_out/t_hllcode.log
timeout -k 10 300 python tools/query_probe.py 100 reg0pipe0 -- "Basic Aggregation" "TPCH Q1" "x:hll-only" "SubQuery + nation,Type predicates + ShipDate Range" > gpurun_out/q1code.txt 2>&1 || { tail -30 gpurun_out/q1code.txt; exit 1; }
grep -v "^$" gpurun_out/q1code.txt | tail -6
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/h_code.json 2> gpurun_out/h_code.err || { tail -30 gpurun_out/h_code.err; exit 1; }
cat gpurun_out/h_code.json
