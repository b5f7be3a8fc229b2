# SQ_INSTS_VMEM_RD calibration: kernels with a known load count (tools/stream_probe.py: sp_x4 = one
# 16-byte load per lane per 1 KiB, q1_il = 2.625 dword loads per 64-row word over Q1's packed
# columns) against the TPC-H Q1 scan kernel (tools/kbench_one.py), same counters.
set -o pipefail
R="$PWD"
mkdir -p gpurun_out
C="SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_SALU TCC_EA0_RDREQ_sum"
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv \
  -d "$R/gpurun_out/pmcv1" -o p -- python3 "$R/tools/stream_probe.py" 1.8 > "$R/gpurun_out/pmcv1.log" 2>&1) &&
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv \
  -d "$R/gpurun_out/pmcv2" -o p -- python3 "$R/tools/kbench_one.py" --sf 100 --query "TPCH Q1" --iters 3 \
  > "$R/gpurun_out/pmcv2.log" 2>&1) &&
python tools/pmc_summary.py gpurun_out "" "pmcv1" by-kernel > gpurun_out/pmc_vmem_probe.txt &&
python tools/pmc_summary.py gpurun_out "sdo_" "pmcv2" by-kernel > gpurun_out/pmc_vmem_q1.txt
rc=$?
rm -rf gpurun_out/pmcv1 gpurun_out/pmcv2
exit $rc
