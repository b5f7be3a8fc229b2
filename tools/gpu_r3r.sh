#!/bin/bash
# GPU box: A/B of descriptor-loaded vs literal query constants in the JIT (TPC-H Q19/Q21/Q2 + headline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for L in 0 1; do
SDO_JIT_LITERALS=$L SDO_BENCH_ONLY=Q19,Q21,Q2,Q6,Q1 timeout -k 10 170 python bench.py --model tpch22 --steps 3 --warmup 1 --verbose > gpurun_out/lit$L.json 2> gpurun_out/lit$L.err || { tail -30 gpurun_out/lit$L.err; exit 1; }
echo "literals=$L"; grep "\[bench\] Q" gpurun_out/lit$L.err
SDO_JIT_LITERALS=$L timeout -k 10 170 python bench.py --steps 10 --warmup 3 > gpurun_out/lith$L.json 2> gpurun_out/lith$L.err || { tail -30 gpurun_out/lith$L.err; exit 1; }
cut -c1-120 gpurun_out/lith$L.json
done
