set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
PY_ARGS="--sf 10 --iters 4" PYPROF_ARGS="--top 25 --tail-ms 5 --timeline-ms 5" bash tools/gpu.sh pyprof:tools/theta_probe.py > gpurun_out/theta_prof.log 2>&1
