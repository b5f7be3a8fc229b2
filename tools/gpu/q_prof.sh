set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
PY_ARGS="100 ${QS:-Q11}" PYPROF_ARGS="--top 25 --tail-ms ${TAIL:-12} --timeline-ms ${TAIL:-12}" bash tools/gpu.sh pyprof:tools/sql_probe.py > gpurun_out/q_prof.log 2>&1
