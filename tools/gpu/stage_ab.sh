set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
SDO_JIT_STAGE=lds timeout -k 10 600 python -u bench.py --model tpch22 --steps 3 --warmup 1 > gpurun_out/bench_tpch22_lds.json 2> gpurun_out/bench_tpch22_lds.err &&
SDO_JIT_STAGE=reg timeout -k 10 600 python -u bench.py --model tpch22 --steps 3 --warmup 1 > gpurun_out/bench_tpch22_reg.json 2> gpurun_out/bench_tpch22_reg.err
