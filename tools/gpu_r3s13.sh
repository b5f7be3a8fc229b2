#!/bin/bash
# GPU box: deferred join/sort gathers -- TPC-H 22 GPU tests, the 22-query bench at SF100, then the
# concurrency bench (64 clients, sharing off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tpch22.py tests/test_gpu_ssb.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_tpch22.log 2>&1 || { tail -40 gpurun_out/t_tpch22.log; exit 1; }
tail -2 gpurun_out/t_tpch22.log
timeout -k 10 400 python bench.py --model tpch22 --steps 3 --warmup 2 --verbose > gpurun_out/tpch22_s13.json 2> gpurun_out/tpch22_s13.err || { tail -30 gpurun_out/tpch22_s13.err; exit 1; }
grep "\[bench\]" gpurun_out/tpch22_s13.err | cut -c1-90; cut -c1-160 gpurun_out/tpch22_s13.json
bash tools/gpu_r3s12.sh
