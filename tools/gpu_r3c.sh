#!/bin/bash
# GPU box: profile the peer rank (rank 1) of the 2-rank gloo rehearsal on TPC-H Q3 / Q5, then a
# host profile (cProfile) of the small headline queries on one GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SDO_BENCH_ONLY="TPCH Q3,TPCH Q5" SDO_BENCH_PROFILE=1 SDO_BENCH_PROFILE_RANK=1 SDO_BENCH_PER_RANK=1 SDO_GLOO_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --sf 20 --steps 5 --warmup 2 --verbose > gpurun_out/bench2_prof_r1.json 2> gpurun_out/bench2_prof_r1.err || { tail -30 gpurun_out/bench2_prof_r1.err; exit 1; }
grep "rank " gpurun_out/bench2_prof_r1.err
SDO_BENCH_ONLY="Ship Date Range,TPCH Q8,TPCH Q5,SubQuery + nation,Type predicates + ShipDate Range" SDO_BENCH_PROFILE=1 timeout -k 10 300 python bench.py --sf 20 --steps 200 --warmup 5 --verbose > gpurun_out/bench1_hostprof.json 2> gpurun_out/bench1_hostprof.err || { tail -30 gpurun_out/bench1_hostprof.err; exit 1; }
tail -1 gpurun_out/bench1_hostprof.json
