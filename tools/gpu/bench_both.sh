set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u bench.py --model tpch22 --steps 3 --warmup 1 > gpurun_out/bench_tpch22.json 2> gpurun_out/bench_tpch22.err &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_headline.json 2> gpurun_out/bench_headline.err
