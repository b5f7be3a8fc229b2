#!/bin/bash
# GPU box: partition / kernel tests, then the headline, TPC-H 22 and SSB sweeps at SF100
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_partition.py tests/test_gpu_kernels.py tests/test_gpu_tpch22.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_p.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_p.log | tail -5; tail -40 gpurun_out/pytest_p.log; exit 1; }
tail -2 gpurun_out/pytest_p.log
timeout -k 10 170 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/bench1_p.json 2> gpurun_out/bench1_p.err || { tail -30 gpurun_out/bench1_p.err; exit 1; }
cut -c1-200 gpurun_out/bench1_p.json
timeout -k 10 170 python bench.py --model tpch22 --steps 3 --warmup 1 --verbose > gpurun_out/tpch22_p.json 2> gpurun_out/tpch22_p.err || { tail -30 gpurun_out/tpch22_p.err; exit 1; }
cut -c1-200 gpurun_out/tpch22_p.json
timeout -k 10 170 python bench.py --model ssb --steps 5 --warmup 2 --verbose > gpurun_out/ssb_p.json 2> gpurun_out/ssb_p.err || { tail -30 gpurun_out/ssb_p.err; exit 1; }
cut -c1-200 gpurun_out/ssb_p.json
