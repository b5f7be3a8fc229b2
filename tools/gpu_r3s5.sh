#!/bin/bash
# GPU box: PMC counters + kernel durations of the Q1 and count-only JIT scan kernels at SF100
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=off
cd /tmp && export TMPDIR=/tmp
Q="${Q:-TPCH Q1,x:count-only,x:nodims-count}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt5" -o kt -- python3 "$R/tools/kbench_one.py" --sf 100 --query "$Q" --iters 5 > "$R/gpurun_out/kt5.log" 2>&1 || { tail -20 "$R/gpurun_out/kt5.log"; exit 1; }
i=0
for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC FETCH_SIZE" "TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d "$R/gpurun_out/pmc5_$i" -o p -- python3 "$R/tools/kbench_one.py" --sf 100 --query "$Q" --iters 3 > "$R/gpurun_out/pmc5_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc5_$i.log"; echo "pass $i failed"; }
done
cd "$R"
find gpurun_out/kt5 -name "*kernel_stats*" -exec head -12 {} \;
python3 - <<'PY'
import csv, glob, collections
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc5_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "sdo_jit" in k:
            vals[k[:20] + ":" + r.get("Grid_Size", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print("==", k)
    for c in sorted(d):
        v = d[c]
        print(f"  {c:30s} n={len(v):3d} mean={sum(v)/len(v):16.1f}")
PY
