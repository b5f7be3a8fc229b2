#!/bin/bash
# GPU box: headline bench on the host fast path (packing off), then PMC A/B packed vs plain for Q1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/bench1_fast.json 2> gpurun_out/bench1_fast.err || { tail -30 gpurun_out/bench1_fast.err; exit 1; }
cat gpurun_out/bench1_fast.json
Q="TPCH Q1" SF=20 bash tools/pmc_ab.sh
