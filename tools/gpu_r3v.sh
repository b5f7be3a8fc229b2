#!/bin/bash
# GPU box: per-stage host / GPU latency of the headline queries
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
timeout -k 10 170 python tools/stage_probe.py --sf 100 --reps 30 > gpurun_out/stage_probe.txt 2>&1 || { tail -30 gpurun_out/stage_probe.txt; exit 1; }
tail -14 gpurun_out/stage_probe.txt
