#!/bin/bash
# GPU box (round 3, first pass): smoke + whole GPU suite + 1-GPU headline bench + rocprof kernel
# stats of the headline + 2-rank rehearsal of the multi-rank path on one card (gloo between two
# processes sharing the GPU; RCCL refuses two ranks per device) with results gathered to rank 0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_gpu.log | tail -20; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -30 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
SDO_GLOO_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --sf 20 --steps 5 --warmup 2 --verbose > gpurun_out/bench2_gloo.json 2> gpurun_out/bench2_gloo.err || { tail -30 gpurun_out/bench2_gloo.err; exit 1; }
cat gpurun_out/bench2_gloo.json
timeout -k 10 300 python bench.py --sf 20 --steps 5 --warmup 2 --verbose > gpurun_out/bench1_sf20.json 2> gpurun_out/bench1_sf20.err || { tail -30 gpurun_out/bench1_sf20.err; exit 1; }
cat gpurun_out/bench1_sf20.json
