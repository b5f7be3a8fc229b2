set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
SDO_JIT_TRACE=1 timeout -k 10 300 python -u tools/kbench_one.py --sf 100 --query "TPCH Q1" --iters 1 > gpurun_out/q1_shape.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_headline.json 2> gpurun_out/bench_headline.err
