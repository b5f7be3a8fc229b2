# Write efficiency of the radix-partition split kernels (tools/part_probe.py, 2-word records, the
# TPC-H Q18 shape): HBM write requests vs full 64-byte ones, and read requests, per kernel.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$PWD"
mkdir -p gpurun_out/r6
rm -rf gpurun_out/r6/pmc_split
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum \
    --kernel-trace --output-format csv -d "$R/gpurun_out/r6/pmc_split" -o run -- \
    python3 "$R/tools/part_probe.py" --n ${N:-600e6} --g 150e6 --rw ${RW:-2} --pu 8 --iters 1 --check 0 \
    > "$R/gpurun_out/r6/pmc_split.log" 2>&1)
