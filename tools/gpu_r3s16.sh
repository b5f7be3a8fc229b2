#!/bin/bash
# GPU box: the multi-rank path rehearsed on one GPU (2 ranks, gloo, shards on the GPU): weak
# (SF20 per rank) and strong (--total-sf 40) headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SDO_GLOO_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --sf 20 --steps 5 --warmup 2 --verbose > gpurun_out/reh2_weak.json 2> gpurun_out/reh2_weak.err || { tail -30 gpurun_out/reh2_weak.err; exit 1; }
grep "\[bench\]" gpurun_out/reh2_weak.err | cut -c1-100; cut -c1-400 gpurun_out/reh2_weak.json
SDO_GLOO_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --total-sf 40 --steps 5 --warmup 2 > gpurun_out/reh2_strong.json 2> gpurun_out/reh2_strong.err || { tail -30 gpurun_out/reh2_strong.err; exit 1; }
cut -c1-400 gpurun_out/reh2_strong.json
