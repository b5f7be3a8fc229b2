#!/bin/bash
# GPU box: per-Druid-query breakdown + host profile of mid-range TPC-H queries (Q2, Q9, Q11, Q22, Q17)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/sql_probe.py 100 Q2 Q9 Q11 Q22 Q17 > gpurun_out/sql_probe_mid.txt 2>&1 || { tail -30 gpurun_out/sql_probe_mid.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/sql_probe_mid.txt | grep -v "planning\|running" | cut -c1-150
timeout -k 10 400 python tools/tpch22_host_profile.py --sf 100 --query Q2 --query Q9 --query Q11 --query Q22 --query Q17 --reps 3 --top 30 > gpurun_out/hp_mid.txt 2>&1 || { tail -30 gpurun_out/hp_mid.txt; exit 1; }
