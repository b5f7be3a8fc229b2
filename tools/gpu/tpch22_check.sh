set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_tpch22.py tests/test_gpu_post.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_tpch22.log 2>&1 &&
timeout -k 10 600 python -u bench.py --model tpch22 --steps 3 --warmup 1 > gpurun_out/bench_tpch22.json 2> gpurun_out/bench_tpch22.err &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_theta.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_theta.log 2>&1 &&
timeout -k 10 300 python -u tools/theta_probe.py --sf 10 --iters 10 > gpurun_out/theta_probe.txt 2>&1
