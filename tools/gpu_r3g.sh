#!/bin/bash
# GPU box: partitioned group-by tests, TPC-H Q18/Q13/Q16 at SF100 with the partitioned plan on/off,
# then the 2-rank root-only rehearsal and the varied-workload concurrency bench (coalescing off/on)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_partition.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_partition.log 2>&1 || { tail -60 gpurun_out/pytest_partition.log; exit 1; }
tail -3 gpurun_out/pytest_partition.log
for P in 1 0; do
SDO_PARTITIONED=$P SDO_BENCH_ONLY=Q18,Q13,Q16 timeout -k 10 400 python bench.py --model tpch22 --steps 5 --warmup 2 --verbose > gpurun_out/tpch22_long_p$P.json 2> gpurun_out/tpch22_long_p$P.err || { tail -30 gpurun_out/tpch22_long_p$P.err; exit 1; }
grep "\[bench\] Q" gpurun_out/tpch22_long_p$P.err
done
bash tools/gpu_r3f.sh
