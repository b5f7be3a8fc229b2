#!/bin/bash
# GPU box: build check of the JIT with bit-packed columns, the GPU suite, then the headline bench
# and a kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_kernels.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_gpu_kernels.log | tail -20; tail -40 gpurun_out/pytest_gpu_kernels.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_kernels.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -30 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
SDO_PK_X2=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/bench1_x2.json 2> gpurun_out/bench1_x2.err || { tail -30 gpurun_out/bench1_x2.err; exit 1; }
cat gpurun_out/bench1_x2.json
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_headline2 -o prof -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_headline2.out 2>&1 || { tail -30 gpurun_out/prof_headline2.out; exit 1; }
tail -1 gpurun_out/prof_headline2.out
