#!/bin/bash
# A/B PMC counters of one query's scan kernel: SDO_PACKED=0 (plain columns) vs 1 (bit-packed).
# usage (GPU box): Q='TPCH Q1' SF=20 bash tools/pmc_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for P in 0 1; do
i=0
for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS" "FETCH_SIZE"; do
  i=$((i+1))
  SDO_PACKED=$P timeout -k 10 240 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d "$R/gpurun_out/pmcab_p${P}_$i" -o p -- python3 "$R/tools/kbench_one.py" --sf ${SF:-20} --query "${Q:-TPCH Q1}" --iters 3 > "$R/gpurun_out/pmcab_p${P}_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/pmcab_p${P}_$i.log"; exit 1; }
done
done
echo pmc-done
