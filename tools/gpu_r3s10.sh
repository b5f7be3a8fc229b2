#!/bin/bash
# GPU box: host phases of the headline queries (pre-launch / GPU+wait / post-wait)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
timeout -k 10 300 python tools/host_phases.py --sf 100 --reps 200 > gpurun_out/host_phases.txt 2>&1 || { tail -30 gpurun_out/host_phases.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/host_phases.txt
