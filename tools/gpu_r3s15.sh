#!/bin/bash
# GPU box: the whole GPU suite + smoke + the headline bench (driver-equivalent) on the final tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -30 gpurun_out/bench_final.err; exit 1; }
grep "\[bench\]" gpurun_out/bench_final.err | cut -c1-100; cat gpurun_out/bench_final.json
