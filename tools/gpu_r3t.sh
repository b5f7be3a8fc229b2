#!/bin/bash
# GPU box: SSB A/B -- default vs literal constants everywhere vs specialization off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "sync 0" "sync 1" "off 0"; do
set -- $cfg
SDO_JIT_SPECIALIZE=$1 SDO_JIT_LITERALS=$2 timeout -k 10 170 python bench.py --model ssb --steps 5 --warmup 2 --verbose > gpurun_out/ssb_$1_$2.json 2> gpurun_out/ssb_$1_$2.err || { tail -30 gpurun_out/ssb_$1_$2.err; exit 1; }
echo "spec=$1 lit=$2 $(cut -c50-90 gpurun_out/ssb_$1_$2.json)"
done
