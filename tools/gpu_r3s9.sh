#!/bin/bash
# GPU box: result waits by polling (SDO_SPIN_SYNC=1) vs hipStreamSynchronize -- headline bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for V in 0 1 0 1; do
  SDO_SPIN_SYNC=$V timeout -k 10 300 python bench.py --steps 30 --warmup 5 --verbose > gpurun_out/h_spin$V.json 2> gpurun_out/h_spin$V.err || { tail -30 gpurun_out/h_spin$V.err; exit 1; }
  echo "== SDO_SPIN_SYNC=$V"; grep "\[bench\]" gpurun_out/h_spin$V.err | cut -c1-100 | tail -8; cut -c1-120 gpurun_out/h_spin$V.json
done
