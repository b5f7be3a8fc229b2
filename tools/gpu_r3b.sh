#!/bin/bash
# GPU box: 2-rank gloo rehearsal with per-rank query means (results on rank 0 vs on every rank),
# then a kernel-trace profile of the 1-GPU headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 1 0; do
SDO_RESULTS_ON_ROOT=$r SDO_BENCH_PER_RANK=1 SDO_GLOO_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --sf 20 --steps 5 --warmup 2 --verbose > gpurun_out/bench2_gloo_root$r.json 2> gpurun_out/bench2_gloo_root$r.err || { tail -30 gpurun_out/bench2_gloo_root$r.err; exit 1; }
grep "rank \|Q3\|Q5" gpurun_out/bench2_gloo_root$r.err
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_headline -o prof -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_headline.out 2>&1 || { tail -30 gpurun_out/prof_headline.out; exit 1; }
tail -2 gpurun_out/prof_headline.out
find gpurun_out/prof_headline -name "*kernel_stats.csv" | head -3
