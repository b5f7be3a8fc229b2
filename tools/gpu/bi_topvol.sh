set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
PY_ARGS="--sf 100 --iters 3 --only TopVolume" PYPROF_ARGS="--top 25 --tail-ms 40 --timeline-ms 20" bash tools/gpu.sh pyprof:tools/bi_probe.py > gpurun_out/bi_topvol.log 2>&1
