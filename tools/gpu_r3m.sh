#!/bin/bash
# GPU box: fused stored-HLL + partition + kernel tests, then the concurrency runs (tools/gpu_r3l.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_sketch_rollup.py tests/test_gpu_partition.py tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_m.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_m.log | tail -5; tail -40 gpurun_out/pytest_m.log; exit 1; }
tail -2 gpurun_out/pytest_m.log
bash tools/gpu_r3l.sh
