#!/bin/bash
# GPU box: A/B of 32-bit LDS accumulator cells (SDO_JIT_NARROW_LDS) and u32 LDS HLL registers
# (SDO_JIT_HLL32LDS) on the Q1-shaped kernels; kernel tests with both switches on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
Q=("Basic Aggregation" "TPCH Q1" "x:count-only" "x:no-hll" "x:hll-only" "x:sum-ext" "SubQuery + nation,Type predicates + ShipDate Range")
SDO_JIT_NARROW_LDS=1 SDO_JIT_HLL32LDS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_hllcode.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_narrow.log 2>&1 || { tail -40 gpurun_out/t_narrow.log; exit 1; }
tail -2 gpurun_out/t_narrow.log
for V in "base::" "narrow:SDO_JIT_NARROW_LDS=1:" "hll32b3:SDO_JIT_HLL32LDS=1:" "hll32b2:SDO_JIT_HLL32LDS=1:SDO_JIT_BLOCKS=2" "both:SDO_JIT_NARROW_LDS=1:SDO_JIT_HLL32LDS=1" "bothb2:SDO_JIT_NARROW_LDS=1:SDO_JIT_HLL32LDS=1:SDO_JIT_BLOCKS=2"; do
  name=${V%%:*}; rest=${V#*:}
  envs=$(echo "$rest" | tr ':' ' ')
  echo "== $name ($envs)"
  env $envs timeout -k 10 300 python tools/query_probe.py 100 reg0pipe0 -- "${Q[@]}" > gpurun_out/ab_$name.txt 2>&1 || { tail -30 gpurun_out/ab_$name.txt; exit 1; }
  grep " med " gpurun_out/ab_$name.txt
done
