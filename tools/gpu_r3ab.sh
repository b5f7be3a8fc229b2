#!/bin/bash
# GPU box: ballot counts for tiny key spaces -- kernel tests, A/B kernel times, headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_hllcode.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ballot.log 2>&1 || { tail -40 gpurun_out/t_ballot.log; exit 1; }
tail -2 gpurun_out/t_ballot.log
for B in 0 8; do
SDO_JIT_BALLOT_G=$B timeout -k 10 300 python tools/query_probe.py 100 reg0pipe0 -- "Basic Aggregation" "Ship Date Range" "SubQuery + nation,Type predicates + ShipDate Range" "TPCH Q1" "TPCH Q8" "x:count-only" "x:nodims-count" > gpurun_out/ballot$B.txt 2>&1 || { tail -30 gpurun_out/ballot$B.txt; exit 1; }
echo "ballot=$B"; grep "med" gpurun_out/ballot$B.txt | cut -c1-75
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/h_ballot.json 2> gpurun_out/h_ballot.err || { tail -30 gpurun_out/h_ballot.err; exit 1; }
cat gpurun_out/h_ballot.json
