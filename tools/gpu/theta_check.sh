set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_theta.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_theta.log 2>&1 &&
timeout -k 10 300 python -u tools/theta_probe.py --sf 10 --iters 10 > gpurun_out/theta_probe.txt 2>&1 &&
PY_ARGS="--sf 10 --iters 4" PYPROF_ARGS="--top 25" bash tools/gpu.sh pyprof:tools/theta_probe.py > gpurun_out/theta_prof.log 2>&1
