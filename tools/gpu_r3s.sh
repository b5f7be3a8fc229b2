#!/bin/bash
# GPU box: TPC-H 22 A/B -- literal specialization off/sync, VGPR-parked constants on/off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "off 1" "sync 1" "off 0" "sync 0"; do
set -- $cfg
SDO_JIT_SPECIALIZE=$1 SDO_JIT_VREG=$2 timeout -k 10 170 python bench.py --model tpch22 --steps 3 --warmup 2 --verbose > gpurun_out/t22_$1_$2.json 2> gpurun_out/t22_$1_$2.err || { tail -30 gpurun_out/t22_$1_$2.err; exit 1; }
echo "spec=$1 vreg=$2 $(cut -c60-100 gpurun_out/t22_$1_$2.json)"
done
