#!/bin/bash
# GPU box: in-order walk of dense prefiltered chunks -- kernel tests, A/B kernel times, bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_tpch22.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_dense.log 2>&1 || { tail -40 gpurun_out/t_dense.log; exit 1; }
tail -2 gpurun_out/t_dense.log
for DW in 0 24 8; do
SDO_JIT_DENSE_WORDS=$DW timeout -k 10 300 python tools/query_probe.py 100 reg0pipe0 -- "SubQuery + nation,Type predicates + ShipDate Range" "TPCH Q3" "TPCH Q5" "TPCH Q7" "TPCH Q8" > gpurun_out/dense$DW.txt 2>&1 || { tail -30 gpurun_out/dense$DW.txt; exit 1; }
echo "dense=$DW"; grep "med" gpurun_out/dense$DW.txt | cut -c1-75
done
for DW in 0 24; do
SDO_JIT_DENSE_WORDS=$DW timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/h_dense$DW.json 2> gpurun_out/h_dense$DW.err || { tail -30 gpurun_out/h_dense$DW.err; exit 1; }
echo "dense=$DW $(cut -c1-140 gpurun_out/h_dense$DW.json)"
done
