set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
SDO_JIT_BLOCKS=2 timeout -k 10 600 python -u bench.py --model tpch22 --steps 3 --warmup 1 > gpurun_out/bench_tpch22_b2.json 2> gpurun_out/b2.err &&
SDO_JIT_BLOCKS=4 timeout -k 10 600 python -u bench.py --model tpch22 --steps 3 --warmup 1 > gpurun_out/bench_tpch22_b4.json 2> gpurun_out/b4.err
