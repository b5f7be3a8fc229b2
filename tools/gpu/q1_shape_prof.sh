# Q1 scan kernel PMC with the kernel the benchmark runs: the JIT code cache is filled by an
# unprofiled run first (kernels compiled under rocprofv3 carry scratch, see profiles/r5/q1_pmc_note.md)
set -o pipefail
R="$PWD"
export SDO_JIT_TRACE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
C="SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_SALU TCC_EA0_RDREQ_sum"
timeout -k 10 300 python -u tools/kbench_one.py --sf 100 --query "TPCH Q1" --iters 1 > gpurun_out/q1_shape_plain.txt 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/q1pmc" -o p -- python3 "$R/tools/kbench_one.py" --sf 100 --query "TPCH Q1" --iters 3 > "$R/gpurun_out/q1_shape_pmc.txt" 2>&1) &&
python tools/pmc_summary.py gpurun_out "sdo_" "q1pmc" by-kernel > gpurun_out/q1_shape_pmc_summary.txt
rc=$?
rm -rf gpurun_out/q1pmc
exit $rc
