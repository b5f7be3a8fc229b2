#!/bin/bash
# GPU box: host profile of TPC-H Q3 (finalize) and Q1 (SQL operators) at SF100
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
timeout -k 10 170 python tools/host_profile.py --sf 100 --steps 30 --query "TPCH Q3" --top 40 > gpurun_out/hostprof_q3.txt 2>&1 || { tail -30 gpurun_out/hostprof_q3.txt; exit 1; }
timeout -k 10 170 python tools/host_profile.py --sf 100 --steps 30 --query "TPCH Q1" --top 40 > gpurun_out/hostprof_q1.txt 2>&1 || { tail -30 gpurun_out/hostprof_q1.txt; exit 1; }
echo done
