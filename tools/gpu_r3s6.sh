#!/bin/bash
# GPU box: host-side cProfile of the small headline queries (where e2e - kernel goes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
timeout -k 10 300 python tools/host_profile.py --sf 100 --mode sql --steps 200 --top 70 --query "Ship Date,SubQuery,Q5,Q8,Q7" > gpurun_out/hp_small.txt 2>&1 || { tail -30 gpurun_out/hp_small.txt; exit 1; }
head -30 gpurun_out/hp_small.txt
timeout -k 10 200 python tools/stage_probe.py --sf 100 --reps 40 > gpurun_out/stage_probe.txt 2>&1 || { tail -30 gpurun_out/stage_probe.txt; exit 1; }
grep -v Warn gpurun_out/stage_probe.txt | tail -10
