#!/bin/bash
# GPU box: small results written into pinned host memory by the kernels (SDO_ZERO_COPY=1) --
# kernel tests with it on, then the headline bench A/B (alternating)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SDO_ZERO_COPY=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ssb.py tests/test_hllcode.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_zc.log 2>&1 || { tail -40 gpurun_out/t_zc.log; exit 1; }
tail -2 gpurun_out/t_zc.log
for V in 0 1 0 1; do
  SDO_ZERO_COPY=$V timeout -k 10 300 python bench.py --steps 30 --warmup 5 --verbose > gpurun_out/h_zc$V.json 2> gpurun_out/h_zc$V.err || { tail -30 gpurun_out/h_zc$V.err; exit 1; }
  echo "== SDO_ZERO_COPY=$V"; grep "\[bench\]" gpurun_out/h_zc$V.err | cut -c1-100 | tail -8; cut -c1-120 gpurun_out/h_zc$V.json
done
