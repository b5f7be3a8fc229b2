#!/bin/bash
# GPU box: partition tests + Q18 kernel trace + PMC of the split kernels (LDS / VMEM behaviour)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_partition.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_partition.log 2>&1 || { tail -60 gpurun_out/pytest_partition.log; exit 1; }
tail -2 gpurun_out/pytest_partition.log
rm -rf gpurun_out/prof_q18j gpurun_out/pmc_split*
cd /tmp && export TMPDIR=/tmp
SDO_BENCH_ONLY=Q18 timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_q18j" -o run -- python3 "$R/bench.py" --model tpch22 --steps 3 --warmup 1 \
  > "$R/gpurun_out/prof_q18j.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_q18j.log"; exit 1; }
grep -h "tpch_flat" "$R/gpurun_out/prof_q18j.log" | cut -c1-200
i=0
for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "FETCH_SIZE"; do
  i=$((i+1))
  SDO_BENCH_ONLY=Q18 timeout -k 10 -s KILL 150 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_split_$i" -o p -- python3 "$R/bench.py" --model tpch22 --steps 1 --warmup 1 > "$R/gpurun_out/pmc_split_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_split_$i.log"; exit 1; }
done
cd "$R"
DB=$(find gpurun_out/prof_q18j -name "*.db" | head -1)
python tools/rocpd_summary.py "$DB" --tail-ms 20 --top 12 --timeline-ms 20 > gpurun_out/prof_q18j_summary.txt
head -14 gpurun_out/prof_q18j_summary.txt
for k in part_split part_agg sdo_jit; do echo "== $k"; python tools/pmc_summary.py gpurun_out $k "pmc_split_*"; done
