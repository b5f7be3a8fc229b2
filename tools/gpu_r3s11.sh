#!/bin/bash
# GPU box: host phases of the headline queries + per-Druid-query breakdown / host profile of the
# TPC-H long tail (Q17, Q13, Q16, Q18)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
timeout -k 10 300 python tools/host_phases.py --sf 100 --reps 200 > gpurun_out/host_phases.txt 2>&1 || { tail -30 gpurun_out/host_phases.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/host_phases.txt
timeout -k 10 400 python tools/sql_probe.py 100 Q17 Q13 Q16 Q18 > gpurun_out/sql_probe_tail.txt 2>&1 || { tail -30 gpurun_out/sql_probe_tail.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/sql_probe_tail.txt | tail -60
timeout -k 10 300 python tools/tpch22_host_profile.py --sf 100 --query Q17 --reps 3 --top 35 > gpurun_out/hp_q17.txt 2>&1 || { tail -30 gpurun_out/hp_q17.txt; exit 1; }
