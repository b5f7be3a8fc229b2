#!/bin/bash
# GPU box: TPC-H 22 sweep A/B on the device-buffer budget (LRU release between queries or not)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for B in 25769803776 214748364800; do
SDO_SCAN_BUF_BUDGET=$B timeout -k 10 170 python bench.py --model tpch22 --steps 3 --warmup 1 --verbose > gpurun_out/tpch22_b$B.json 2> gpurun_out/tpch22_b$B.err || { tail -30 gpurun_out/tpch22_b$B.err; exit 1; }
echo "budget $B: $(cut -c1-120 gpurun_out/tpch22_b$B.json)"
done
