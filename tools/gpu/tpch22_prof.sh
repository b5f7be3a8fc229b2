set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
PY_TIMEOUT=900 PY_ARGS="--model tpch22 --steps 2 --warmup 1" PYPROF_ARGS="--top 400 --tail-ms 80" bash tools/gpu.sh pyprof:bench.py > gpurun_out/tpch22_prof.log 2>&1
