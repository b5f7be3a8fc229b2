#!/bin/bash
# GPU box: the whole GPU suite + smoke on the final tree of this session
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_end.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_end.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_end.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_end.log 2>&1 || { tail -20 gpurun_out/smoke_end.log; exit 1; }
tail -1 gpurun_out/smoke_end.log | cut -c1-120
