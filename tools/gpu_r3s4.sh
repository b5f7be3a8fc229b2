#!/bin/bash
# GPU box: row-blocked full-chunk staging (SDO_JIT_BLOCKED) -- kernel tests, then A/B on Q1-shaped kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
Q=("Basic Aggregation" "TPCH Q1" "x:count-only" "x:no-hll" "x:hll-only" "x:sum-ext" "Ship Date Range" "TPCH Q5" "TPCH Q7")
SDO_JIT_REGPIPE=1 SDO_JIT_NARROW_LDS=1 SDO_JIT_HLL32LDS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_hllcode.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_regpipe.log 2>&1 || { tail -40 gpurun_out/t_regpipe.log; exit 1; }
tail -2 gpurun_out/t_regpipe.log
for V in "base::" "rp:SDO_JIT_REGPIPE=1:" "rpall:SDO_JIT_REGPIPE=1:SDO_JIT_NARROW_LDS=1:SDO_JIT_HLL32LDS=1" "rpx2:SDO_JIT_REGPIPE=1:SDO_PK_X2=1"; do
  name=${V%%:*}; rest=${V#*:}
  envs=$(echo "$rest" | tr ':' ' ')
  echo "== $name ($envs)"
  env $envs timeout -k 10 300 python tools/query_probe.py 100 reg0pipe0 -- "${Q[@]}" > gpurun_out/ab4_$name.txt 2>&1 || { tail -30 gpurun_out/ab4_$name.txt; exit 1; }
  grep " med " gpurun_out/ab4_$name.txt | cut -c1-120
done
