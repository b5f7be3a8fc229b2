set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
PY_ARGS="--sf 100 --template TopVolume" PYPROF_ARGS="--top 20 --tail-ms 14 --timeline-ms 14" bash tools/gpu.sh pyprof:tools/op_trace.py > gpurun_out/topvol_tl.log 2>&1
