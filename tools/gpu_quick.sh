#!/bin/bash
# quick GPU iteration: build + gpu tests + per-query kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python tools/qprofile.py --sf ${SF:-100} --unroll ${UNROLLS:-2} ${BOTH:+--both} > gpurun_out/qprof.log 2>&1 || { tail -30 gpurun_out/qprof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qprof.log
