#!/bin/bash
# GPU box: Q1-shaped kernel A/B (accumulator placement, copies, occupancy, staging) + cost isolation
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
timeout -k 10 400 python tools/query_probe.py 100 reg0pipe0 reg1pipe0 reg0pipe0c64 reg0pipe0c32 reg0pipe0b2 reg0pipe0b4 reg0pipe0slds reg0pipe0sreg -- "Basic Aggregation" "TPCH Q1" "x:count-only" "x:no-hll" "x:hll-only" "x:sum-ext" "x:nodims-count" > gpurun_out/q1ab.txt 2>&1 || { tail -30 gpurun_out/q1ab.txt; exit 1; }
grep -v "^$" gpurun_out/q1ab.txt | tail -70
